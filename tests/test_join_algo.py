"""BATjoin's algorithm choice (gdk/gdk_join.c:4542-4618) and the result order
and properties it implies.

CPU: the oracle takes the algorithm the reference takes for each shape
(selectjoin, mergejoin_void, mergejoin on sorted sides or on one cheaper
sorted side, hashjoin, and the swapped variants), and its pairs follow that
algorithm's order rule (helpers.join_expected).
GPU: the device returns the same pairs, result types (void / oid), sequence
bases and properties (tsorted, trevsorted, tkey, tnonil, tnil) as the oracle,
and caches the same ordering knowledge on its inputs."""
import numpy as np
import pytest

from helpers import join_cases, join_expected

CASES = join_cases()
IDS = [c["name"] for c in CASES]
NILS = {"bte": -(1 << 7), "sht": -(1 << 15), "int": -(1 << 31), "lng": -(1 << 63), "oid": 1 << 63}


def _cand(M, c, which):
    s = c["sl" if which == "l" else "sr"]
    if s is None:
        return None
    if isinstance(s, tuple):
        if M.__name__.endswith("gdk"):
            return M.BAT.dense(s[1], s[2])
        return M.Bat.dense(s[1], s[2])
    if M.__name__.endswith("gdk"):
        return M.BAT.from_numpy(M.TYPE_oid, s, sorted_=True, revsorted=len(s) <= 1, key=True, nonil=True)
    return M.Bat.from_array(M.TYPE_oid, s, sorted_=True, revsorted=len(s) <= 1, key=True, nonil=True)


def _side(M, c, which):
    vals, void, h = (c["lv"], c["lvoid"], c["lh"]) if which == "l" else (c["rv"], c["rvoid"], c["rh"])
    fl = c["lflags"] if which == "l" else c["rflags"]
    isgdk = M.__name__.endswith("gdk")
    if void is not None:
        return M.BAT.dense(void[0], void[1], hseqbase=h) if isgdk else M.Bat.dense(void[0], void[1], hseqbase=h)
    tp = getattr(M, "TYPE_" + c["tp"])
    kw = dict(sorted_=fl.get("sorted", False), revsorted=fl.get("revsorted", False), key=fl.get("key", False),
              nonil=bool((vals != NILS[c["tp"]]).all()))
    if isgdk:
        return M.BAT.from_numpy(tp, vals, hseqbase=h, **kw)
    return M.Bat.from_array(tp, vals, hseqbase=h, **kw)


def _pylist(vals, void, tp):
    if void is not None:
        return list(range(void[0], void[0] + void[1]))
    nil = NILS[tp]
    return [None if int(v) == nil else int(v) for v in vals]


def _cands(c, which, n, h):
    s = c["sl" if which == "l" else "sr"]
    allc = range(h, h + n)
    if s is None:
        return list(allc)
    if isinstance(s, tuple):
        return [o for o in range(s[1], s[1] + s[2]) if h <= o < h + n]
    return [int(o) for o in s if h <= o < h + n]


def _model(c):
    lv = _pylist(c["lv"], c["lvoid"], c["tp"])
    rv = _pylist(c["rv"], c["rvoid"], c["tp"])
    lc = _cands(c, "l", len(lv), c["lh"])
    rc = _cands(c, "r", len(rv), c["rh"])
    return join_expected(c, lv, rv, lc, rc)


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_oracle_join_algorithm_and_order(ora, c):
    l, r = _side(ora, c, "l"), _side(ora, c, "r")
    sl, sr = _cand(ora, c, "l"), _cand(ora, c, "r")
    assert ora.join_algo(l, r, sl, sr) == c["algo"]
    l, r = _side(ora, c, "l"), _side(ora, c, "r")
    a, b = ora.BATjoin(l, r, sl, sr, nil_matches=c["nil_matches"])
    got = list(zip(a.values().tolist(), b.values().tolist()))
    assert got == _model(c)


def test_oracle_join_swap_example(ora):
    """l = [1, 2, 1], r = [1, 1, 3, 1]: joincost with exact unique counts
    (BATs of <= 1000 rows are sampled whole) gives lcost 12.6 < rcost 14.6,
    so the reference hashes l and drives from r: r1 = [2, 0, 2, 0, 2, 0]."""
    l = ora.Bat.from_array(ora.TYPE_int, np.array([1, 2, 1], np.int32))
    r = ora.Bat.from_array(ora.TYPE_int, np.array([1, 1, 3, 1], np.int32))
    a, b = ora.BATjoin(l, r)
    assert a.values().tolist() == [2, 0, 2, 0, 2, 0]
    assert b.values().tolist() == [0, 0, 1, 1, 3, 3]
    pa, pb = ora.props(a), ora.props(b)
    assert (pa["sorted"], pa["key"], pb["sorted"], pb["revsorted"]) == (False, False, True, False)


def test_oracle_join_caches_order(ora):
    """BATordered on a sorted, strictly increasing input records tsorted and
    tkey on it (gdk_batop.c:2112-2121), as BATjoin's first test does."""
    l = ora.Bat.from_array(ora.TYPE_int, np.arange(10, dtype=np.int32))
    r = ora.Bat.from_array(ora.TYPE_int, np.array([3, 1, 2, 2], np.int32))
    ora.BATjoin(l, r)
    assert l.s.sorted and l.s.key and not l.s.revsorted
    assert not r.s.sorted


def _dprops(b):
    s = b.s
    return dict(type="void" if s.ttype == 0 else "oid" if s.ttype == 6 else s.ttype, count=s.count,
                tseqbase=s.tseqbase, sorted=bool(s.tsorted), revsorted=bool(s.trevsorted), key=bool(s.tkey),
                nonil=bool(s.tnonil), nil=bool(s.tnil))


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_gpu_join_matches_oracle(gdk, ora, c):
    ol, orr = _side(ora, c, "l"), _side(ora, c, "r")
    osl, osr = _cand(ora, c, "l"), _cand(ora, c, "r")
    oa, ob = ora.BATjoin(ol, orr, osl, osr, nil_matches=c["nil_matches"])
    dl, dr = _side(gdk, c, "l"), _side(gdk, c, "r")
    dsl, dsr = _cand(gdk, c, "l"), _cand(gdk, c, "r")
    a, b = gdk.BATjoin(dl, dr, dsl, dsr, nil_matches=c["nil_matches"])
    assert np.array_equal(a.to_numpy(), oa.values()), c["name"]
    assert np.array_equal(b.to_numpy(), ob.values()), c["name"]
    assert _dprops(a) == ora.props(oa), ("r1", c["name"])
    assert _dprops(b) == ora.props(ob), ("r2", c["name"])
    # the ordering knowledge both cached on their inputs
    for d, o in ((dl, ol), (dr, orr)):
        assert (d.s.tsorted, d.s.trevsorted, d.s.tkey) == (o.s.sorted, o.s.revsorted, o.s.key), c["name"]


@pytest.mark.gpu
def test_gpu_join_swap_example(gdk):
    l = gdk.BAT.from_numpy(gdk.TYPE_int, np.array([1, 2, 1], np.int32), sorted_=False, revsorted=False, key=False)
    r = gdk.BAT.from_numpy(gdk.TYPE_int, np.array([1, 1, 3, 1], np.int32), sorted_=False, revsorted=False,
                           key=False)
    a, b = gdk.BATjoin(l, r)
    assert a.to_numpy().tolist() == [2, 0, 2, 0, 2, 0]
    assert b.to_numpy().tolist() == [0, 0, 1, 1, 3, 3]


def _ordered_model(vals, isnil):
    """BAT_ORDERED / BAT_ORDERED_FP (gdk/gdk_batop.c:1950-1995): nil below
    every value, two nils equal; returns (sorted, revsorted)."""
    def cmp(i):
        a, b = isnil[i - 1], isnil[i]
        if a or b:
            return -int(not b) if a else 1
        return (vals[i - 1] > vals[i]) - (vals[i - 1] < vals[i])
    cs = [cmp(i) for i in range(1, len(vals))]
    return all(c <= 0 for c in cs), all(c >= 0 for c in cs)


@pytest.mark.gpu
@pytest.mark.parametrize("tp", ["flt", "dbl", "hge"])
@pytest.mark.parametrize("shape", ["asc", "desc", "asc_nils", "desc_nils_end", "mixed", "const", "negzero"])
def test_gpu_ordered_fp_hge(gdk, tp, shape):
    """BATordered / BATordered_rev scan flt / dbl (NaN nil smallest) and hge
    columns as the reference does instead of answering 'not ordered'."""
    r = np.random.default_rng(hash((tp, shape)) & 0xffff)
    n = 5000
    v = np.sort(r.integers(-10**6, 10**6, n)).astype(np.float64) / 7
    isnil = np.zeros(n, bool)
    if shape == "desc":
        v = v[::-1].copy()
    elif shape == "asc_nils":
        isnil[:40] = True
    elif shape == "desc_nils_end":
        v = v[::-1].copy()
        isnil[-40:] = True
    elif shape == "mixed":
        v[100], v[101] = v[101], v[100] - 1
    elif shape == "const":
        v[:] = -3.5
    elif shape == "negzero":
        v = np.array([-1.0, -0.0, 0.0, -0.0, 2.0] * 1, np.float64)
        isnil = np.zeros(v.size, bool)
    if tp == "hge":
        iv = [int(x * 7) * (1 << 70) + 5 for x in v]
        words = [gdk.int_to_hge_words(gdk.NIL[gdk.TYPE_hge] if isnil[i] else iv[i]) for i in range(v.size)]
        arr = np.array(words, np.uint64)
        mv = iv
        b = gdk.BAT.from_numpy(gdk.TYPE_hge, arr, sorted_=False, revsorted=False, key=False)
    else:
        dt = np.float32 if tp == "flt" else np.float64
        arr = v.astype(dt)
        arr[isnil] = np.nan
        mv = arr.tolist()
        b = gdk.BAT.from_numpy(gdk.TYPE_flt if tp == "flt" else gdk.TYPE_dbl, arr, sorted_=False,
                               revsorted=False, key=False)
    want = _ordered_model(mv, isnil)
    assert (gdk.BATordered(b), gdk.BATordered_rev(b)) == want


def _fl_cases():
    r = np.random.default_rng(77)
    out = []
    for dt in (np.float32, np.float64):
        lv = (r.integers(-50, 50, 3000) / 4).astype(dt)
        rv = (r.integers(-50, 50, 700) / 4).astype(dt)
        lv[::37] = np.nan
        rv[::41] = np.nan
        lv[5], rv[9] = -0.0, 0.0
        lv[6], rv[10] = 0.0, -0.0
        out.append((dt, lv, rv, "shuffled"))
        out.append((dt, np.sort(lv), np.sort(rv), "sorted"))
        uq = np.unique(rv[~np.isnan(rv)])
        out.append((dt, lv, r.permutation(uq).astype(dt), "unique_build"))
    return out


@pytest.mark.parametrize("case", range(6))
@pytest.mark.parametrize("nil_matches", [False, True])
def test_oracle_float_join_pairs(ora, case, nil_matches):
    """Float keys join by dbl_cmp equality (-0.0 == +0.0, NaN nil matches
    only with nil_matches): the oracle's pairs equal a brute-force model."""
    dt, lv, rv, _ = _fl_cases()[case]
    tp = ora.TYPE_flt if dt == np.float32 else ora.TYPE_dbl
    a, b = ora.BATjoin(ora.Bat.from_array(tp, lv), ora.Bat.from_array(tp, rv), nil_matches=nil_matches)
    got = sorted(zip(np.asarray(a.values()).tolist(), np.asarray(b.values()).tolist()))
    want = sorted((i, j) for i, x in enumerate(lv) for j, y in enumerate(rv)
                  if (x == y) or (nil_matches and np.isnan(x) and np.isnan(y)))
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(6))
@pytest.mark.parametrize("nil_matches", [False, True])
def test_gpu_float_join(gdk, ora, case, nil_matches):
    """BATjoin on flt / dbl keys: the device (integer images that keep
    equality and order) gives the oracle's pairs in the oracle's order, and
    both cache the same order properties."""
    dt, lv, rv, _ = _fl_cases()[case]
    tg = gdk.TYPE_flt if dt == np.float32 else gdk.TYPE_dbl
    to = ora.TYPE_flt if dt == np.float32 else ora.TYPE_dbl
    L = gdk.BAT.from_numpy(tg, lv, hseqbase=3, sorted_=False, revsorted=False, key=False)
    R = gdk.BAT.from_numpy(tg, rv, hseqbase=5, sorted_=False, revsorted=False, key=False)
    a, b = gdk.BATjoin(L, R, nil_matches=nil_matches)
    oa, ob = ora.BATjoin(ora.Bat.from_array(to, lv, hseqbase=3), ora.Bat.from_array(to, rv, hseqbase=5),
                         nil_matches=nil_matches)
    assert np.array_equal(a.to_numpy(), oa.values())
    assert np.array_equal(b.to_numpy(), ob.values())
