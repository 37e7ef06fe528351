"""BATfirstn (gdk/gdk_firstn.c:1280) against a numpy restatement of its
documented semantics (:18-58, :1023-1278): rank by (g asc, value asc/desc
with nils first/last); with gids or distinct every row tied with the last
one is returned; the plain variant returns the first tied rows (the
reference's choice among ties follows its heap -- see firstn.hip)."""
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
def test_firstn(gdk, tname, dt, asc, nilslast, gids):
    r = rng(401)
    tp = getattr(gdk, "TYPE_" + tname)
    nil = gdk.NIL[tp]
    v = with_nils(r.integers(-50, 50, 40_000).astype(dt), nil, 0.02, r)
    for n in (1, 7, 100, 1000):
        t, gi = gdk.BATfirstn(gdk.BAT.from_numpy(tp, v), n, asc=asc, nilslast=nilslast, want_gids=gids)
        want = want_topn(v, nil, n, asc, nilslast, gids)
        assert np.array_equal(t.to_numpy().astype(np.int64), want), n
        if gids:
            sel = v[want]
            rk = rank_of(sel, nil, asc, not asc)           # gids: order (!asc, !asc) per the reference
            u = np.unique(rk)
            assert np.array_equal(gi.to_numpy(), np.searchsorted(u, rk).astype(np.uint64))


def test_firstn_candidates_and_distinct(gdk):
    r = rng(402)
    v = r.integers(0, 300, 50_000).astype(np.int32)
    s = np.sort(r.choice(50_000, 20_000, replace=False)).astype(np.uint64)
    B, S = gdk.BAT.from_numpy(gdk.TYPE_int, v), gdk.BAT.from_numpy(gdk.TYPE_oid, s)
    t, _ = gdk.BATfirstn(B, 50, s=S)
    assert np.array_equal(t.to_numpy(), want_topn(v, None if False else gdk.NIL[gdk.TYPE_int], 50, True, False,
                                                  False, cand=s.astype(np.int64)).astype(np.uint64))
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
