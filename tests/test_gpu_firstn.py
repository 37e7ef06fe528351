"""BATfirstn (gdk/gdk_firstn.c:1280).  The plain variant (no group ids, not
distinct) is compared with the oracle's restatement of the reference's heap
(oracle/gdk_oracle_firstn.c) -- including which tied rows survive -- and
with the reference's own known answers (pqueue*.maltest).  The variants
with group ids / distinct are compared with a numpy restatement of their
documented semantics (:18-58, :1023-1278): rank by (g asc, value asc/desc
with nils first/last), every row tied with the last one returned."""
import numpy as np
import pytest

from helpers import rng, with_nils

pytestmark = pytest.mark.gpu


def rank_of(v, nil, asc, nilslast):
    # float64 ranks are exact here (|v| < 2^53)
    x = v.astype(np.float64)
    isn = (v == nil) if nil is not None else np.isnan(x)
    r = x if asc else -x
    big = np.inf
    return np.where(isn, big if nilslast else -big, r)


def want_topn(v, nil, n, asc, nilslast, all_ties, cand=None, g=None):
    cand = np.arange(len(v)) if cand is None else cand
    vals = v[cand]
    r = rank_of(vals, nil, asc, nilslast)
    gg = np.zeros(len(cand)) if g is None else g.astype(np.float64)
    order = np.lexsort((r, gg))
    if n >= len(cand):
        return cand
    last = order[n - 1]
    lt = (gg < gg[last]) | ((gg == gg[last]) & (r < r[last]))
    eq = (gg == gg[last]) & (r == r[last])
    if all_ties:
        sel = lt | eq
    else:
        need = n - int(lt.sum())
        eqpos = np.flatnonzero(eq)[:need]
        sel = lt.copy()
        sel[eqpos] = True
    return cand[sel]


@pytest.mark.parametrize("tname,dt", [("int", np.int32), ("lng", np.int64), ("sht", np.int16)])
@pytest.mark.parametrize("asc,nilslast", [(True, False), (True, True), (False, False), (False, True)])
@pytest.mark.parametrize("gids", [False, True])
def test_firstn(gdk, ora, tname, dt, asc, nilslast, gids):
    r = rng(401)
    tp = getattr(gdk, "TYPE_" + tname)
    nil = gdk.NIL[tp]
    v = with_nils(r.integers(-50, 50, 40_000).astype(dt), nil, 0.02, r)
    for n in (1, 7, 100, 1000):
        t, gi = gdk.BATfirstn(gdk.BAT.from_numpy(tp, v), n, asc=asc, nilslast=nilslast, want_gids=gids)
        if gids:
            want = want_topn(v, nil, n, asc, nilslast, True)
        else:
            want = np.array(ora.BATfirstn(ora.Bat.from_array(tp, v), n, asc=asc, nilslast=nilslast).values(),
                            np.int64)
        assert np.array_equal(t.to_numpy().astype(np.int64), want), n
        if gids:
            sel = v[want]
            rk = rank_of(sel, nil, asc, not asc)           # gids: order (!asc, !asc) per the reference
            u = np.unique(rk)
            assert np.array_equal(gi.to_numpy(), np.searchsorted(u, rk).astype(np.uint64))


def test_firstn_maltest_fixture(gdk):
    """Every int algebra.firstn of pqueue*.maltest: the reference's rows
    (and group ids), cascades fed with the reference's own previous output."""
    from helpers import firstn_cases
    n = 0
    for src, c in firstn_cases():
        b = gdk.BAT.from_numpy(gdk.TYPE_int, np.array(c["values"], np.int32))
        s = g = None
        if c["s"]:
            s = gdk.BAT.from_numpy(gdk.TYPE_oid, np.array(c["s_values"], np.uint64))
            g = gdk.BAT.from_numpy(gdk.TYPE_oid, np.array(c["g_values"], np.uint64))
        t, gi = gdk.BATfirstn(b, c["n"], s=s, g=g, asc=c["asc"], nilslast=c["nilslast"],
                              distinct=c["distinct"], want_gids=c["gids"] is not None)
        assert [int(x) for x in t.to_numpy()] == c["expected"]["topn"], (src, c)
        if "gids" in c["expected"]:
            assert [int(x) for x in gi.to_numpy()] == c["expected"]["gids"], (src, c)
        n += 1
    assert n >= 50


@pytest.mark.parametrize("asc,nilslast", [(True, False), (True, True), (False, False), (False, True)])
@pytest.mark.parametrize("shape", ["random", "sorted", "revsorted", "ascending-ish"])
def test_firstn_heap_ties(gdk, ora, asc, nilslast, shape):
    """Heavy ties at the n-th value: the device replays the reference's heap."""
    r = rng(404)
    N = 300_000
    v = r.integers(0, 40, N).astype(np.int32)
    v[r.random(N) < 0.03] = gdk.NIL[gdk.TYPE_int]
    if shape == "sorted":
        v = np.sort(v)
    elif shape == "revsorted":
        v = np.sort(v)[::-1].copy()
    elif shape == "ascending-ish":
        v = (np.arange(N) // 1000 + r.integers(0, 3, N)).astype(np.int32)
    B, OB = gdk.BAT.from_numpy(gdk.TYPE_int, v), ora.Bat.from_array(ora.TYPE_int, v)
    for n in (1, 5, 999, 4096, 70_000):
        t, _ = gdk.BATfirstn(B, n, asc=asc, nilslast=nilslast)
        want = np.array(ora.BATfirstn(OB, n, asc=asc, nilslast=nilslast).values(), np.int64)
        assert np.array_equal(t.to_numpy().astype(np.int64), want), (n, shape)


@pytest.mark.parametrize("tname,dt", [("lng", np.int64), ("dbl", np.float64), ("bte", np.int8)])
def test_firstn_heap_types_and_candidates(gdk, ora, tname, dt):
    r = rng(405)
    N = 100_000
    tp = getattr(gdk, "TYPE_" + tname)
    if dt == np.float64:
        v = r.integers(-20, 20, N).astype(dt)
        v[r.random(N) < 0.02] = np.nan
    else:
        v = r.integers(-20, 20, N).astype(dt)
        v[r.random(N) < 0.02] = gdk.NIL[tp]
    cand = np.sort(r.choice(N, 60_000, replace=False)).astype(np.uint64)
    B, OB = gdk.BAT.from_numpy(tp, v), ora.Bat.from_array(tp, v)
    S, OS = gdk.BAT.from_numpy(gdk.TYPE_oid, cand), ora.Bat.from_array(ora.TYPE_oid, cand)
    for asc in (True, False):
        for nilslast in (True, False):
            for n in (3, 250, 20_000):
                t, _ = gdk.BATfirstn(B, n, s=S, asc=asc, nilslast=nilslast)
                want = np.array(ora.BATfirstn(OB, n, s=OS, asc=asc, nilslast=nilslast).values(), np.int64)
                assert np.array_equal(t.to_numpy().astype(np.int64), want), (n, asc, nilslast)


def test_firstn_heap_with_groups(gdk, ora):
    """BATfirstn_unique_with_groups: heap over (group, value) pairs."""
    r = rng(406)
    N = 80_000
    v = r.integers(0, 10, N).astype(np.int32)
    cand = np.sort(r.choice(N, 50_000, replace=False)).astype(np.uint64)
    g = np.sort(r.integers(0, 30, cand.size)).astype(np.uint64)
    g = r.permutation(g).astype(np.uint64)
    B, OB = gdk.BAT.from_numpy(gdk.TYPE_int, v), ora.Bat.from_array(ora.TYPE_int, v)
    S, OS = gdk.BAT.from_numpy(gdk.TYPE_oid, cand), ora.Bat.from_array(ora.TYPE_oid, cand)
    G, OG = gdk.BAT.from_numpy(gdk.TYPE_oid, g), ora.Bat.from_array(ora.TYPE_oid, g)
    for asc in (True, False):
        for n in (1, 17, 3000):
            t, _ = gdk.BATfirstn(B, n, s=S, g=G, asc=asc, nilslast=not asc)
            want = np.array(ora.BATfirstn(OB, n, s=OS, g=OG, asc=asc, nilslast=not asc).values(), np.int64)
            assert np.array_equal(t.to_numpy().astype(np.int64), want), (n, asc)


def test_firstn_candidates_and_distinct(gdk, ora):
    r = rng(402)
    v = r.integers(0, 300, 50_000).astype(np.int32)
    s = np.sort(r.choice(50_000, 20_000, replace=False)).astype(np.uint64)
    B, S = gdk.BAT.from_numpy(gdk.TYPE_int, v), gdk.BAT.from_numpy(gdk.TYPE_oid, s)
    t, _ = gdk.BATfirstn(B, 50, s=S)
    want = ora.BATfirstn(ora.Bat.from_array(ora.TYPE_int, v), 50, s=ora.Bat.from_array(ora.TYPE_oid, s)).values()
    assert np.array_equal(t.to_numpy(), np.array(want, np.uint64))
    # distinct: the 5 smallest distinct values, every candidate holding one
    t, _ = gdk.BATfirstn(B, 5, s=S, distinct=True)
    vs = v[s.astype(np.int64)]
    best = np.unique(vs)[:5]
    assert np.array_equal(t.to_numpy(), s[np.isin(vs, best)])


def test_firstn_cascade_three_columns(gdk):
    # the documented cascade (gdk_firstn.c:50-55): first n rows of (b1, b2, b3)
    r = rng(403)
    N = 30_000
    b1 = r.integers(0, 30, N).astype(np.int32)
    b2 = r.integers(0, 30, N).astype(np.int64)
    b3 = r.permutation(N).astype(np.int32)            # unique: no ties at the end
    B1, B2, B3 = (gdk.BAT.from_numpy(gdk.TYPE_int, b1), gdk.BAT.from_numpy(gdk.TYPE_lng, b2),
                  gdk.BAT.from_numpy(gdk.TYPE_int, b3))
    n = 500
    s1, g1 = gdk.BATfirstn(B1, n, want_gids=True)
    s2, g2 = gdk.BATfirstn(B2, n, s=s1, g=g1, want_gids=True)
    s3, _ = gdk.BATfirstn(B3, n, s=s2, g=g2)
    want = np.sort(np.lexsort((b3, b2, b1))[:n])
    assert np.array_equal(s3.to_numpy().astype(np.int64), want)


def test_firstn_trivial(gdk):
    B = gdk.BAT.from_numpy(gdk.TYPE_int, np.array([5, 3, 9], np.int32))
    t, g = gdk.BATfirstn(B, 0, want_gids=True)
    assert t.count() == 0 and g.count() == 0
    t, _ = gdk.BATfirstn(B, 10)
    assert list(t.to_numpy()) == [0, 1, 2]
