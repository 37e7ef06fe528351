"""Dictionary / frame-of-reference compressed inputs (sql/backends/monet5/
dict.c, for.c): compression round trips, and selections on the codes equal
the oracle's selection over the decompressed values (the reference's general
path: BATselect on the dictionary, then the semijoin on the codes)."""
import numpy as np
import pytest

from helpers import rng, with_nils

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tname,dt", [("int", np.int32), ("lng", np.int64), ("sht", np.int16)])
@pytest.mark.parametrize("ordered", [True, False])
def test_dict_roundtrip(gdk, tname, dt, ordered):
    r = rng(501)
    tp = getattr(gdk, "TYPE_" + tname)
    nil = gdk.NIL[tp]
    v = with_nils(r.choice(r.integers(-10**4, 10**4, 300), 80_000).astype(dt), nil, 0.01, r)
    o, u = gdk.DICTcompress(gdk.BAT.from_numpy(tp, v), ordered=ordered)
    uv, cv = u.to_numpy(), o.to_numpy()
    assert o.ttype == gdk.TYPE_sht           # 301 distinct values -> sht codes
    assert np.array_equal(uv[cv.astype(np.uint16)], v)
    _, first = np.unique(v, return_index=True)
    if ordered:
        assert np.array_equal(uv, np.sort(np.unique(v)))
    else:
        assert np.array_equal(uv, v[np.sort(first)])
    d = gdk.DICTdecompress(o, u)
    assert np.array_equal(d.to_numpy(), v)


def test_dict_bte_codes_above_127(gdk):
    # 200 distinct values: bte codes 128..199 are stored negative and read unsigned
    v = np.repeat(np.arange(200, dtype=np.int32) * 3, 5)
    o, u = gdk.DICTcompress(gdk.BAT.from_numpy(gdk.TYPE_int, v))
    assert o.ttype == gdk.TYPE_bte
    assert np.array_equal(gdk.DICTdecompress(o, u).to_numpy(), v)


SEL = [(10, 500, True, True, False), (10, 500, False, True, False), (10, 500, True, False, True),
       (None, 100, True, True, False), (-200, None, True, True, False), (None, None, True, True, False),
       (None, None, False, False, True), (7, 7, True, True, False)]


@pytest.mark.parametrize("lo,hi,li,hi_,anti", SEL)
@pytest.mark.parametrize("with_cands", [False, True])
def test_dict_select(gdk, ora, lo, hi, li, hi_, anti, with_cands):
    r = rng(502)
    tp = gdk.TYPE_int
    nil = gdk.NIL[tp]
    v = with_nils(r.choice(np.arange(-1000, 1000, 7), 60_000).astype(np.int32), nil, 0.02, r)
    o, u = gdk.DICTcompress(gdk.BAT.from_numpy(tp, v))
    cand = np.sort(r.choice(60_000, 25_000, replace=False)).astype(np.uint64) if with_cands else None
    L = nil if lo is None else lo
    H = nil if hi is None else hi
    got = gdk.DICTselect(o, gdk.BAT.from_numpy(gdk.TYPE_oid, cand) if with_cands else None, u, L, H, li, hi_, anti)
    # dict.c:965-977 normalisation, then the selection over the values
    nl, nh, nli, nhi, nanti = L, H, li, hi_, anti
    if not nanti:
        if nli and nl == nil:
            nl, nli = nh, False
        if nhi and nh == nil:
            nh, nhi = nl, False
        if nl == nh and nh == nil:
            nanti = True
    want = ora.BATselect(ora.Bat.from_array(ora.TYPE_int, v),
                         ora.Bat.from_array(ora.TYPE_oid, cand, sorted_=True) if with_cands else None,
                         nl, nh, nli, nhi, nanti)
    assert np.array_equal(got.to_numpy(), want.values())


@pytest.mark.parametrize("op", ["<", "<=", ">", ">=", "==", "!="])
def test_dict_thetaselect(gdk, ora, op):
    r = rng(503)
    v = with_nils(r.choice(np.arange(0, 5000, 3), 50_000).astype(np.int64), gdk.NIL[gdk.TYPE_lng], 0.02, r)
    o, u = gdk.DICTcompress(gdk.BAT.from_numpy(gdk.TYPE_lng, v), ordered=False)
    got = gdk.DICTthetaselect(o, None, u, 2400, op)
    want = ora.BATthetaselect(ora.Bat.from_array(ora.TYPE_lng, v), None, 2400, op)
    assert np.array_equal(got.to_numpy(), want.values())


def test_for_roundtrip_and_errors(gdk):
    r = rng(504)
    v = r.integers(10**12, 10**12 + 50, 70_000).astype(np.int64)
    o, mn = gdk.FORcompress(gdk.BAT.from_numpy(gdk.TYPE_lng, v))
    assert o.ttype == gdk.TYPE_bte and mn == v.min()
    assert np.array_equal(gdk.FORdecompress(o, mn, gdk.TYPE_lng).to_numpy(), v)
    w = r.integers(-5000, 5000, 70_000).astype(np.int64)
    o2, mn2 = gdk.FORcompress(gdk.BAT.from_numpy(gdk.TYPE_lng, w))
    assert o2.ttype == gdk.TYPE_sht
    assert np.array_equal(gdk.FORdecompress(o2, mn2, gdk.TYPE_int).to_numpy(), w.astype(np.int32))
    with pytest.raises(gdk.GDKError, match="too large value spread"):
        gdk.FORcompress(gdk.BAT.from_numpy(gdk.TYPE_lng, np.array([0, 40000], np.int64)))
    with pytest.raises(gdk.GDKError, match="cannot have NULL"):
        gdk.FORcompress(gdk.BAT.from_numpy(gdk.TYPE_lng, np.array([0, gdk.NIL[gdk.TYPE_lng]], np.int64)))
