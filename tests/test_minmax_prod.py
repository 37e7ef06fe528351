"""Whole-column BATmin / BATmax (gdk/gdk_aggr.c:3570-3844), BATprod (:1650) /
BATgroupprod (:1575) and BATunmask (gdk/gdk_cand.c:1464).

The oracle (oracle/gdk_oracle_grp.c ora_minmax / ora_prod / ora_groupprod)
restates the reference; here it is checked against Python models written
from the same source -- min / max: the ordered-column shortcuts (a sorted
column's max is its LAST row, so without skipnil a sorted column with nils
still answers its largest value) and do_groupmin / do_groupmax's first row
holding the extreme (without skipnil the first nil); prod: doprod's three
macro shapes (AGGR_PROD forgets a nil that comes before a group's first
value when nil_if_empty; AGGR_PROD_HGE marks a group seen on any row) with
the exact overflow rule (an overflow of any prefix product, so a zero before
the overflow hides it and one after does not).  The device is compared with
the oracle, at sizes that take its parallel forms (10M rows).  No reference
fixture holds these (parity unpinned beyond the models); `aggr.prod` and
`aggr.min` / `aggr.max` are the MAL bindings (aggr.c:189-218, algebra.c:
155-194)."""
import math

import numpy as np
import pytest

from helpers import rng

NI = -(1 << 31)
NL = -(1 << 63)


def _nil(tname):
    return {"bte": -128, "sht": -(1 << 15), "int": NI, "lng": NL}.get(tname)


def _minmax_model(vals, isnil, sorted_, revsorted, skipnil, domax):
    """value index per the reference's path (None: nil)"""
    n = len(vals)
    if n == 0:
        return None
    if sorted_ or revsorted:
        if not domax:
            if skipnil and any(isnil):
                if sorted_:
                    q = next((i for i in range(n) if not isnil[i]), n)
                    return None if q == n else q
                q = next((i for i in range(n) if isnil[i]), n)
                return None if q == 0 else q - 1
            return 0 if sorted_ else n - 1
        p = n - 1 if sorted_ else 0
        return None if skipnil and isnil[p] else p
    best = None
    for i in range(n):
        if skipnil and isnil[i]:
            continue
        if best is None:
            best = i
        elif not isnil[best] and (isnil[i] or (vals[i] > vals[best] if domax else vals[i] < vals[best])):
            best = i
    return best


def _mm_cases():
    r = rng(1501)
    a = r.integers(-1000, 1000, 5000).astype(np.int32)
    an = a.copy()
    an[r.choice(5000, 50, replace=False)] = NI
    yield "int", a, False
    yield "int_nils", an, False
    yield "int_sorted_nils", np.sort(an), True
    yield "int_revsorted_nils", np.sort(an)[::-1].copy(), True
    yield "int_allnil", np.full(300, NI, np.int32), True
    yield "lng", r.integers(-(1 << 62), 1 << 62, 4000).astype(np.int64), False
    f = (r.integers(-50, 50, 3000) / 7).astype(np.float64)
    f[::17] = np.nan
    f[5], f[9] = -0.0, 0.0
    yield "dbl", f, False
    yield "flt", f.astype(np.float32), False
    z = np.array([0.0, -0.0, 1.0, -0.0, 0.0], np.float64)
    yield "dbl_zero_ties", -np.abs(z) if False else np.array([-0.0, 0.0, -1.0, 0.0], np.float64), False
    yield "sht", r.integers(-300, 300, 2000).astype(np.int16), False


def _tname(a):
    return {np.dtype(np.int8): "bte", np.dtype(np.int16): "sht", np.dtype(np.int32): "int",
            np.dtype(np.int64): "lng", np.dtype(np.float32): "flt", np.dtype(np.float64): "dbl"}[a.dtype]


def _isnil(a, tname):
    return np.isnan(a) if tname in ("flt", "dbl") else a == _nil(tname)


def _same(x, y):
    if isinstance(x, float) or isinstance(y, float):
        return (math.isnan(x) and math.isnan(y)) or (x == y and math.copysign(1, x) == math.copysign(1, y))
    return x == y


@pytest.mark.parametrize("name,a,ordered", list(_mm_cases()))
@pytest.mark.parametrize("skipnil", [True, False])
@pytest.mark.parametrize("domax", [False, True])
def test_oracle_minmax_model(ora, name, a, ordered, skipnil, domax):
    tn = _tname(a)
    B = ora.Bat.from_array(getattr(ora, "TYPE_" + tn), a)
    isn = list(_isnil(a, tn))
    srt = bool(np.all(_key(a[:-1], isn[:-1]) <= _key(a[1:], isn[1:]))) if len(a) > 1 else True
    rsrt = bool(np.all(_key(a[:-1], isn[:-1]) >= _key(a[1:], isn[1:]))) if len(a) > 1 else True
    p = _minmax_model(list(a), isn, srt, rsrt and not srt, skipnil, domax)
    got = ora.BATminmax(B, skipnil, domax)
    want = (float("nan") if tn in ("flt", "dbl") else _nil(tn)) if p is None else a[p].item()
    assert _same(got, want), (got, want, p)


def _key(a, isn):
    """order keys with nil smallest (BAT_ORDERED / BAT_ORDERED_FP)"""
    k = np.where(np.asarray(isn), -np.inf, np.nan_to_num(a.astype(np.float64)))
    return k


def test_oracle_minmax_str(ora):
    from strheap import build_heap, tail
    words = [b"pear", b"apple", b"\x80", b"zebra", b"apple", b"mango"]
    heap, offs = build_heap(words, 1)
    t = tail([offs[i][0] for i in range(len(words))], 2)
    B = ora.Bat.from_array(ora.TYPE_str, t, vheap=heap)
    assert ora.BATminmax(B) == b"apple"
    assert ora.BATminmax(B, domax=True) == b"zebra"
    B = ora.Bat.from_array(ora.TYPE_str, t, vheap=heap)
    assert ora.BATminmax(B, skipnil=False) == b"\x80"


def _prod_model(vals, isnil, tp2, skip, ne):
    """doprod for one group (gdk_aggr.c:1340-1548): (value or None for nil) or
    'overflow'"""
    kind = "hge" if tp2 == "hge" else "float" if tp2 in ("flt", "dbl") else "int"
    mx = {"bte": 127, "sht": 32767, "int": 2**31 - 1, "lng": 2**63 - 1, "hge": 2**127 - 1}.get(tp2)
    p, nil, seen = 1, ne, False
    for v, n in zip(vals, isnil):
        if kind == "hge" and ne and not seen:
            seen, nil, p = True, False, 1
        if n:
            if not skip:
                nil = True
            continue
        if kind != "hge" and ne and not seen:
            seen, nil, p = True, False, 1
        if nil:
            continue
        if kind == "float":
            fmax = np.finfo(np.float32 if tp2 == "flt" else np.float64).max
            ft = np.float32 if tp2 == "flt" else np.float64
            x = ft(v)
            ax, ap = abs(x), abs(ft(p))
            if ax > 1 and fmax / ax < ap:
                return "overflow"
            p = ft(ft(p) * x)
        else:
            p = int(v) * p
            if abs(p) > mx:
                return "overflow"
    return None if nil else p


def _prod_cases():
    r = rng(1502)
    yield "small", r.integers(-3, 4, 40).astype(np.int32), ["lng", "hge", "dbl"]
    v = r.integers(1, 4, 200).astype(np.int32)
    v[150] = 0
    yield "zero_hides_later_overflow", v, ["int", "lng"]
    v2 = v.copy()
    v2[150] = 5
    v2[199] = 0
    yield "overflow_before_zero", v2, ["lng", "hge"]
    n = np.array([NI, 3, NI, 5, -2, NI], np.int32)
    yield "nils_around_first", n, ["int", "lng", "hge", "dbl"]
    yield "all_nil", np.full(7, NI, np.int32), ["lng", "hge", "flt"]
    f = (r.integers(-20, 20, 300) / 8).astype(np.float64)
    f[::31] = np.nan
    yield "dbl", f, ["dbl"]
    yield "flt_overflow", np.full(60, 1e30, np.float32), ["flt", "dbl"]


@pytest.mark.parametrize("name,v,tps", list(_prod_cases()))
@pytest.mark.parametrize("skip", [True, False])
@pytest.mark.parametrize("ne", [True, False])
def test_oracle_prod_model(ora, name, v, tps, skip, ne):
    tn = _tname(v)
    B = ora.Bat.from_array(getattr(ora, "TYPE_" + tn), v)
    isn = list(_isnil(v, tn))
    for tp2 in tps:
        want = _prod_model(list(v), isn, tp2, skip, ne)
        if want == "overflow":
            with pytest.raises(Exception, match="overflow in product"):
                ora.BATprod(getattr(ora, "TYPE_" + tp2), B, None, skip, ne)
            continue
        got = ora.BATprod(getattr(ora, "TYPE_" + tp2), B, None, skip, ne)
        if want is None:
            assert got != got if tp2 in ("flt", "dbl") else got == {"int": NI, "lng": NL,
                                                                      "hge": -(1 << 127)}[tp2], (tp2, got)
        else:
            assert got == want, (tp2, got, want)


def test_oracle_groupprod_model(ora):
    r = rng(1503)
    n = 3000
    g = r.integers(0, 50, n).astype(np.uint64)
    v = r.integers(-2, 3, n).astype(np.int32)
    v[r.choice(n, 100, replace=False)] = NI
    B = ora.Bat.from_array(ora.TYPE_int, v)
    G = ora.Bat.from_array(ora.TYPE_oid, g)
    for skip in (True, False):
        got = ora.BATgroupprod(B, G, None, ora.TYPE_lng, skip).values()
        for k in range(50):
            rows = np.flatnonzero(g == k)
            w = _prod_model(list(v[rows]), list(v[rows] == NI), "lng", skip, True)
            assert got[k] == (NL if w is None else w), (k, skip)


# ---- device ---------------------------------------------------------------


@pytest.mark.gpu
@pytest.mark.parametrize("name,a,ordered", list(_mm_cases()))
@pytest.mark.parametrize("skipnil", [True, False])
@pytest.mark.parametrize("domax", [False, True])
def test_gpu_minmax(gdk, ora, name, a, ordered, skipnil, domax):
    tn = _tname(a)
    B = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tn), a, sorted_=False, revsorted=False, key=False)
    O = ora.Bat.from_array(getattr(ora, "TYPE_" + tn), a)
    got = (gdk.BATmax if domax else gdk.BATmin)(B, skipnil)
    assert _same(got, ora.BATminmax(O, skipnil, domax))
    # the position is cached: the second call answers from it, as the
    # reference does whatever skipnil asks
    assert _same((gdk.BATmax if domax else gdk.BATmin)(B, not skipnil), ora.BATminmax(O, not skipnil, domax))


@pytest.mark.gpu
@pytest.mark.parametrize("tn", ["bte", "int", "lng", "hge", "flt", "dbl", "date", "timestamp"])
def test_gpu_minmax_large(gdk, ora, tn):
    """10M rows: the device's one-pass scan, every extreme tied many times
    (the first row holding it is the answer), nils spread"""
    r = rng(1504)
    n = 10_000_000
    if tn in ("flt", "dbl"):
        a = (r.integers(-1000, 1000, n) / 4).astype(np.float32 if tn == "flt" else np.float64)
        a[r.choice(n, 1000, replace=False)] = np.nan
        a[r.choice(n, 10, replace=False)] = -0.0
    elif tn == "hge":
        lo = r.integers(-(1 << 62), 1 << 62, n, dtype=np.int64)
        a = np.stack([lo.view(np.uint64), (lo >> 63).view(np.uint64)], axis=1)   # sign-extended
    else:
        dt = {"bte": np.int8, "int": np.int32, "date": np.int32, "lng": np.int64, "timestamp": np.int64}[tn]
        a = r.integers(-100, 100, n).astype(dt)
        a[r.choice(n, 1000, replace=False)] = np.iinfo(dt).min
    tg, to = getattr(gdk, "TYPE_" + tn), getattr(ora, "TYPE_" + tn)
    for skipnil in (True, False):
        for domax in (False, True):
            B = gdk.BAT.from_numpy(tg, a, sorted_=False, revsorted=False, key=False)
            O = ora.Bat.from_array(to, a)
            got = (gdk.BATmax if domax else gdk.BATmin)(B, skipnil)
            assert _same(got, ora.BATminmax(O, skipnil, domax)), (skipnil, domax)


@pytest.mark.gpu
def test_gpu_minmax_str_void_empty(gdk, ora):
    from strheap import build_heap, tail
    words = [b"pear", b"apple", b"\x80", b"zebra", b"apple", b"mango"] * 300
    heap, offs = build_heap(words[:6], 1)
    t = tail([offs[i % 6][0] for i in range(len(words))], 2)
    for skipnil in (True, False):
        B = gdk.BAT.from_numpy(gdk.TYPE_str, t, vheap=heap, sorted_=False, revsorted=False, key=False, nonil=False)
        O = ora.Bat.from_array(ora.TYPE_str, t, vheap=heap)
        assert gdk.BATmin(B, skipnil) == ora.BATminmax(O, skipnil)
        B = gdk.BAT.from_numpy(gdk.TYPE_str, t, vheap=heap, sorted_=False, revsorted=False, key=False, nonil=False)
        assert gdk.BATmax(B, skipnil) == ora.BATminmax(O, skipnil, True)
    assert gdk.BATmin(gdk.BAT.dense(7, 100)) == 7 and gdk.BATmax(gdk.BAT.dense(7, 100)) == 106
    assert gdk.BATmin(gdk.BAT.from_numpy(gdk.TYPE_int, np.zeros(0, np.int32))) == NI


@pytest.mark.gpu
@pytest.mark.parametrize("name,v,tps", list(_prod_cases()))
@pytest.mark.parametrize("skip", [True, False])
@pytest.mark.parametrize("ne", [True, False])
def test_gpu_prod(gdk, ora, name, v, tps, skip, ne):
    tn = _tname(v)
    B = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tn), v, sorted_=False, revsorted=False, key=False)
    O = ora.Bat.from_array(getattr(ora, "TYPE_" + tn), v)
    for tp2 in tps:
        try:
            want = ora.BATprod(getattr(ora, "TYPE_" + tp2), O, None, skip, ne)
        except Exception:
            with pytest.raises(gdk.GDKError, match="overflow in product"):
                gdk.BATprod(getattr(gdk, "TYPE_" + tp2), B, None, skip, ne)
            continue
        got = gdk.BATprod(getattr(gdk, "TYPE_" + tp2), B, None, skip, ne)
        assert _same(got, want), (tp2, got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["ones", "zero_late", "overflow_late", "nil_cut", "cands"])
def test_gpu_prod_large(gdk, ora, case):
    """10M-row integer products through the parallel form: saturated
    magnitudes, the first zero and the nil cut combined across workgroups"""
    r = rng(1505)
    n = 10_000_000
    v = np.where(r.random(n) < 0.5, 1, -1).astype(np.int64)
    s = None
    if case == "zero_late":
        v[r.choice(n, 40, replace=False)] = 3
        v[n - 5] = 0
    elif case == "overflow_late":
        v[r.choice(n // 2, 30, replace=False) + n // 2] = 1 << 20
    elif case == "nil_cut":
        v[r.choice(n // 2, 30, replace=False) + n // 2] = 1 << 20
        v[n // 3] = NL
    elif case == "cands":
        v[r.choice(n, 25, replace=False)] = 7
        s = np.sort(r.choice(n, n // 2, replace=False)).astype(np.uint64)
    B = gdk.BAT.from_numpy(gdk.TYPE_lng, v, sorted_=False, revsorted=False, key=False)
    O = ora.Bat.from_array(ora.TYPE_lng, v)
    gs = gdk.BAT.from_numpy(gdk.TYPE_oid, s, sorted_=True, key=True, nonil=True) if s is not None else None
    os_ = ora.Bat.from_array(ora.TYPE_oid, s, sorted_=True, key=True, nonil=True) if s is not None else None
    for tp in ("lng", "hge"):
        for skip in (True, False):
            try:
                want = ora.BATprod(getattr(ora, "TYPE_" + tp), O, os_, skip, True)
            except Exception:
                with pytest.raises(gdk.GDKError, match="overflow in product"):
                    gdk.BATprod(getattr(gdk, "TYPE_" + tp), B, gs, skip, True)
                continue
            assert gdk.BATprod(getattr(gdk, "TYPE_" + tp), B, gs, skip, True) == want, (tp, skip)


@pytest.mark.gpu
@pytest.mark.parametrize("tn,tp", [("int", "lng"), ("lng", "hge"), ("sht", "int"), ("dbl", "dbl"), ("int", "flt")])
def test_gpu_groupprod(gdk, ora, tn, tp):
    r = rng(1506)
    n = 200_000
    g = r.integers(0, 5000, n).astype(np.uint64)
    dt = {"int": np.int32, "lng": np.int64, "sht": np.int16}.get(tn)
    if tn == "dbl":
        v = (r.integers(-8, 9, n) / 4).astype(np.float64)
        v[::97] = np.nan
    else:
        v = r.integers(-2, 3, n).astype(dt)
        v[::97] = np.iinfo(dt).min
    B = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tn), v, sorted_=False, revsorted=False, key=False)
    O = ora.Bat.from_array(getattr(ora, "TYPE_" + tn), v)
    G = gdk.BAT.from_numpy(gdk.TYPE_oid, g, sorted_=False, revsorted=False, key=False)
    OG = ora.Bat.from_array(ora.TYPE_oid, g)
    for skip in (True, False):
        try:
            want = ora.BATgroupprod(O, OG, None, getattr(ora, "TYPE_" + tp), skip)
        except Exception:
            with pytest.raises(gdk.GDKError, match="overflow in product"):
                gdk.BATgroupprod(B, G, None, getattr(gdk, "TYPE_" + tp), skip)
            continue
        got = gdk.BATgroupprod(B, G, None, getattr(gdk, "TYPE_" + tp), skip)
        if tp == "hge":
            assert list(got.values()) == [int(x) for x in want.values()]
            continue
        w, x = np.asarray(want.values()), got.to_numpy()
        if tp in ("flt", "dbl"):
            assert np.array_equal(w.view(np.uint8), x.view(np.uint8))
        else:
            assert np.array_equal(w, x)


@pytest.mark.gpu
def test_gpu_unmask(gdk, ora):
    """BATunmask of a msk BAT (the oid list of its set bits) and of cand_mask
    lists: under half the bits set -> an oid list, over half -> the negative
    (cand_except) list of the unset bits below the last set one"""
    r = rng(1507)
    for frac in (0.1, 0.9):
        bits = r.random(70_001) < frac
        m = gdk.BAT.from_bits(bits, hseqbase=40) if hasattr(gdk.BAT, "from_bits") else None
        c = gdk.BAT.mask_cand(1000, bits)
        u = gdk.BATunmask(c)
        assert np.array_equal(np.asarray(gdk.cand_oids(u), np.uint64), 1000 + np.flatnonzero(bits).astype(np.uint64))
        if frac > 0.5:
            assert u.ttype == gdk.TYPE_void          # the cand_except form
        if m is not None:
            um = gdk.BATunmask(m)
            assert np.array_equal(np.asarray(gdk.cand_oids(um), np.uint64), 40 + np.flatnonzero(bits).astype(np.uint64))


# ---- BATcalcavg (gdk_aggr.c:2987) -----------------------------------------


def test_oracle_calcavg_model(ora):
    r = rng(1520)
    v = r.integers(-1000, 1000, 5000).astype(np.int32)
    v[::7] = NI
    a, n = ora.BATcalcavg(ora.Bat.from_array(ora.TYPE_int, v))
    ok = v[v != NI].astype(np.int64)
    assert n == len(ok) and a == float(ok.sum()) / len(ok)
    a, n = ora.BATcalcavg(ora.Bat.from_array(ora.TYPE_int, v), scale=2)
    assert a == float(ok.sum()) / len(ok) / 100.0
    f = r.standard_normal(3000)
    f[::11] = np.nan
    a, n = ora.BATcalcavg(ora.Bat.from_array(ora.TYPE_dbl, f))
    m = 0.0
    k = 0
    for x in f:
        if np.isnan(x):
            continue
        k += 1
        m = m + (x - m) / k if (m > 0) == (x > 0) else m - m / k + x / k
    assert n == k and a == m
    a, n = ora.BATcalcavg(ora.Bat.from_array(ora.TYPE_int, np.full(4, NI, np.int32)))
    assert np.isnan(a) and n == 0


@pytest.mark.gpu
@pytest.mark.parametrize("tp", ["bte", "int", "lng", "hge", "flt", "dbl"])
@pytest.mark.parametrize("cands", [False, True])
def test_gpu_calcavg(gdk, ora, tp, cands):
    r = rng(1521)
    n = 200_000
    if tp in ("flt", "dbl"):
        v = (r.standard_normal(n) * 50).astype(np.float32 if tp == "flt" else np.float64)
        v[::13] = np.nan
    elif tp == "hge":
        vals = [int(x) << 70 if i % 17 else -(1 << 127) for i, x in enumerate(r.integers(-99, 99, n))]
        v = np.array([[x & (2**64 - 1), (x >> 64) & (2**64 - 1)] for x in vals], np.uint64)
    else:
        dt = {"bte": np.int8, "int": np.int32, "lng": np.int64}[tp]
        v = r.integers(np.iinfo(dt).min + 1, np.iinfo(dt).max, n).astype(dt)
        v[::13] = np.iinfo(dt).min
    G = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tp), v)
    O = ora.Bat.from_array(getattr(ora, "TYPE_" + tp), v)
    s = os_ = None
    if cands:
        c = np.sort(r.choice(n, n // 3, replace=False)).astype(np.uint64)
        s = gdk.BAT.from_numpy(gdk.TYPE_oid, c, sorted_=True, key=True, nonil=True)
        os_ = ora.Bat.from_array(ora.TYPE_oid, c, sorted_=True, key=True, nonil=True)
    for scale in (0, 3):
        a, k = gdk.BATcalcavg(G, s, scale)
        oa, ok_ = ora.BATcalcavg(O, os_, scale)
        assert k == ok_
        assert (np.isnan(a) and np.isnan(oa)) or a == oa, (a, oa)
    prev = gdk.set_fp_parallel_min(1000)
    try:
        a, k = gdk.BATcalcavg(G, s)
    finally:
        gdk.set_fp_parallel_min(prev)
    oa, ok_ = ora.BATcalcavg(O, os_)
    assert k == ok_
    if tp in ("flt", "dbl"):
        xs = np.abs(np.asarray(v, np.float64))
        assert abs(a - oa) <= 4 * k * 2.0 ** -53 * float(np.nanmax(xs))
    else:
        assert a == oa
