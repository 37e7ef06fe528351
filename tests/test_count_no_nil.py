"""BATcount_no_nil (gdk/gdk_batop.c:3078): the candidates whose value is not
nil, per type (flt / dbl: NaN; str: the 0x80 nil string through 1-, 2- and
4-byte offsets), with the shortcuts the reference takes (tnonil, msk, void)
and its "we learned something" tnonil update (:3179).  The oracle is checked
against a numpy model; the device against the oracle on every type and
candidate form.  No reference fixture holds the counts (parity unpinned
beyond the model)."""
import numpy as np
import pytest

from helpers import rng

TYPES = {"bte": (np.int8, -128), "sht": (np.int16, -(1 << 15)), "int": (np.int32, -(1 << 31)),
         "lng": (np.int64, -(1 << 63)), "date": (np.int32, -(1 << 31)), "timestamp": (np.int64, -(1 << 63)),
         "flt": (np.float32, np.nan), "dbl": (np.float64, np.nan)}


def _values(r, tname, n):
    dt, nil = TYPES[tname]
    v = r.integers(-100, 100, n).astype(dt)
    v[r.random(n) < 0.2] = nil
    return v


def _isnil(v):
    if v.dtype.kind == "f":
        return np.isnan(v)
    return v == np.iinfo(v.dtype).min


def _cands(gdk, ora, r, n, form):
    if form == "none":
        return None, None, np.arange(n)
    if form == "oids":
        c = np.sort(r.choice(n, n // 2, replace=False)).astype(np.uint64)
        return (gdk.BAT.from_numpy(gdk.TYPE_oid, c, sorted_=True, key=True, nonil=True),
                ora.Bat.from_array(ora.TYPE_oid, c, sorted_=True, key=True, nonil=True), c.astype(np.int64))
    if form == "neg":
        d = np.sort(r.choice(n, n // 5, replace=False)).astype(np.uint64)
        keep = np.setdiff1d(np.arange(n), d.astype(np.int64))
        return (gdk.BATnegcands(0, n, gdk.BAT.from_numpy(gdk.TYPE_oid, d, sorted_=True, key=True, nonil=True)),
                ora.negcands(0, n, ora.Bat.from_array(ora.TYPE_oid, d, sorted_=True, key=True, nonil=True)), keep)
    bits = r.random(n) < 0.3
    return (gdk.BATmaskedcands(0, n, gdk.BAT.msk(bits), True), ora.maskedcands(0, n, ora.Bat.msk(bits), True),
            np.nonzero(bits)[0])


@pytest.mark.parametrize("tname", list(TYPES))
def test_oracle_count_no_nil_model(ora, tname):
    r = rng(2611)
    v = _values(r, tname, 500)
    b = ora.Bat.from_array(getattr(ora, "TYPE_" + tname), v)
    assert ora.BATcount_no_nil(b) == int((~_isnil(v)).sum())
    c = np.sort(r.choice(500, 123, replace=False)).astype(np.uint64)
    s = ora.Bat.from_array(ora.TYPE_oid, c, sorted_=True, key=True, nonil=True)
    assert ora.BATcount_no_nil(b, s) == int((~_isnil(v[c.astype(np.int64)])).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("tname", list(TYPES))
@pytest.mark.parametrize("form", ["none", "oids", "neg", "mask"])
def test_gpu_count_no_nil(gdk, ora, tname, form):
    r = rng(2612)
    n = 300_001
    v = _values(r, tname, n)
    B = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tname), v, sorted_=False, revsorted=False, key=False, nonil=False)
    O = ora.Bat.from_array(getattr(ora, "TYPE_" + tname), v)
    gs, os_, idx = _cands(gdk, ora, r, n, form)
    want = int((~_isnil(v[idx])).sum())
    assert ora.BATcount_no_nil(O, os_) == want
    assert gdk.BATcount_no_nil(B, gs) == want
    assert B.s.tnonil == 0


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 2, 4])
def test_gpu_count_no_nil_str(gdk, ora, width):
    from strheap import NIL, WORDS, sample
    r = rng(2613)
    n = 50_000
    t, h, wi = sample(r, n, width, copies=2 if width == 1 else 6)
    B = gdk.BAT.from_numpy(gdk.TYPE_str, t, vheap=h, sorted_=False, revsorted=False, key=False, nonil=False)
    O = ora.Bat.from_array(ora.TYPE_str, t, vheap=h)
    isnil = np.asarray([WORDS[k] == NIL for k in wi])
    assert gdk.BATcount_no_nil(B) == ora.BATcount_no_nil(O) == int((~isnil).sum())
    gs, os_, idx = _cands(gdk, ora, r, n, "oids")
    assert gdk.BATcount_no_nil(B, gs) == ora.BATcount_no_nil(O, os_) == int((~isnil[idx]).sum())


@pytest.mark.gpu
def test_gpu_count_no_nil_shortcuts(gdk):
    # void: every candidate, none with a nil sequence; msk: every candidate
    D = gdk.BAT.dense(5, 100)
    assert gdk.BATcount_no_nil(D) == 100
    s = gdk.BAT.from_numpy(gdk.TYPE_oid, np.array([0, 3, 7], np.uint64), sorted_=True, key=True, nonil=True)
    assert gdk.BATcount_no_nil(D, s) == 3
    M = gdk.BAT.msk(np.arange(64) % 3 == 0)
    assert gdk.BATcount_no_nil(M) == 64
    # a count of every row records tnonil; a partial one does not
    v = np.arange(1000, dtype=np.int32)
    B = gdk.BAT.from_numpy(gdk.TYPE_int, v, sorted_=False, revsorted=False, key=False, nonil=False)
    assert gdk.BATcount_no_nil(B, s) == 3 and B.s.tnonil == 0
    assert gdk.BATcount_no_nil(B) == 1000 and B.s.tnonil == 1
    # tnonil set: the candidate count, the tail not read
    v[5] = -(1 << 31)
    B = gdk.BAT.from_numpy(gdk.TYPE_int, v, sorted_=False, revsorted=False, key=False, nonil=True)
    assert gdk.BATcount_no_nil(B) == 1000
