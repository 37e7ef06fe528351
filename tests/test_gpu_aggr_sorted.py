"""Grouped aggregates over SORTED group ids (every group a run of rows: what
BATgroup returns for ordered keys and clustered columns such as l_orderkey)
on the device's segmented reduction against the oracle: sums (lng / hge
results, nil rules with and without skip_nils, overflow), counts, exact
averages (avg3, avg), min / max positions and avg3combine, with candidate
lists, runs across the kernel's 1024-row ranges, singleton runs and gids
outside the extents' range."""
import numpy as np
import pytest

from helpers import rng

pytestmark = pytest.mark.gpu

NIL64 = -(1 << 63)


def _runs(r, n, mean):
    lens = r.integers(1, 2 * mean, 2 * (n // mean) + 2)
    g = np.repeat(np.arange(len(lens)), lens)[:n]
    return g.astype(np.uint64)


def _cols(gdk, ora, tname, vals, gids, hseq=0):
    tp = getattr(gdk, "TYPE_" + tname)
    kw = dict(sorted_=False, revsorted=False, key=False, nonil=False)
    V = (gdk.BAT.from_numpy(tp, vals, hseqbase=hseq, **kw), ora.Bat.from_array(getattr(ora, "TYPE_" + tname), vals,
                                                                               hseqbase=hseq, **kw))
    gk = dict(sorted_=True, revsorted=False, key=False, nonil=True)
    G = (gdk.BAT.from_numpy(gdk.TYPE_oid, gids, hseqbase=hseq, **gk),
         ora.Bat.from_array(ora.TYPE_oid, gids, hseqbase=hseq, sorted_=True, nonil=True))
    assert G[0].s.tsorted
    return V, G


def _eq(d, o):
    assert np.array_equal(np.asarray(d.values()), np.asarray(o.values()))
    assert bool(d.s.tnil) == bool(o.s.nil) or o.s.count == 0


@pytest.mark.parametrize("mean", [1, 4, 700, 5000])
@pytest.mark.parametrize("skip", [True, False])
def test_sorted_groupsum_count_minmax(gdk, ora, mean, skip):
    r = rng(800 + mean)
    n = 300_007
    gids = _runs(r, n, mean)
    vals = r.integers(-10**6, 10**6, n).astype(np.int64)
    vals[r.random(n) < 0.02] = NIL64
    (V, OV), (G, OG) = _cols(gdk, ora, "lng", vals, gids)
    for tp in ("lng", "hge"):
        _eq(gdk.BATgroupsum(V, G, None, getattr(gdk, "TYPE_" + tp), skip),
            ora.BATgroupsum(OV, OG, None, getattr(ora, "TYPE_" + tp), skip))
    _eq(gdk.BATgroupcount(V, G, None, skip), ora.BATgroupcount(OV, OG, None, skip))
    _eq(gdk.BATgroupmin(V, G, None, skip), ora.BATgroupminmax(OV, OG, None, False, skip))
    _eq(gdk.BATgroupmax(V, G, None, skip), ora.BATgroupminmax(OV, OG, None, True, skip))
    a, rm, c = gdk.BATgroupavg3(V, G, None, skip)
    oa, orm, oc = ora.BATgroupavg3(OV, OG, None, skip)
    for d, o in ((a, oa), (rm, orm), (c, oc)):
        assert np.array_equal(np.asarray(d.values()), np.asarray(o.values()))
    av, ac = gdk.BATgroupavg(V, G, None, skip)
    oav, oac = ora.BATgroupavg(OV, OG, None, skip)
    assert np.array_equal(av.to_numpy().view(np.uint64), np.asarray(oav.values()).view(np.uint64))
    assert np.array_equal(ac.to_numpy(), oac.values())
    # the avg3 partials combined again (the mergetable rewrite)
    ng = int(gids.max()) + 1
    pg = (np.arange(ng) // 3).astype(np.uint64)
    PG = gdk.BAT.from_numpy(gdk.TYPE_oid, pg, sorted_=True, revsorted=False, key=False, nonil=True)
    OPG = ora.Bat.from_array(ora.TYPE_oid, pg, sorted_=True, nonil=True)
    _eq(gdk.BATgroupavg3combine(a, rm, c, PG, None, skip), ora.BATgroupavg3combine(oa, orm, oc, OPG, None, skip))


def test_sorted_groupsum_cands_extents_and_narrow(gdk, ora):
    """candidate lists, an extents BAT fixing the group range (gids beyond it
    ignored), int values, and the lng overflow error"""
    r = rng(810)
    n = 200_003
    gids = _runs(r, n, 6)
    vals = r.integers(-1000, 1000, n).astype(np.int32)
    (V, OV), (G, OG) = _cols(gdk, ora, "int", vals, gids, hseq=4)
    cand = np.sort(r.choice(n, 120_000, replace=False)).astype(np.uint64) + 4
    S = gdk.BAT.from_numpy(gdk.TYPE_oid, cand, sorted_=True, revsorted=False, key=True, nonil=True)
    OS = ora.Bat.from_array(ora.TYPE_oid, cand, sorted_=True, key=True, nonil=True)
    gs = gids[(cand - 4).astype(np.int64)]
    Gs = gdk.BAT.from_numpy(gdk.TYPE_oid, gs, hseqbase=int(cand[0]), sorted_=True, revsorted=False, key=False,
                            nonil=True)
    OGs = ora.Bat.from_array(ora.TYPE_oid, gs, hseqbase=int(cand[0]), sorted_=True, nonil=True)
    _eq(gdk.BATgroupsum(V, Gs, None, gdk.TYPE_lng, True, s=S), ora.BATgroupsum(OV, OGs, None, ora.TYPE_lng, True, s=OS))
    ne = int(gids.max()) // 2
    E = gdk.BAT.dense(0, ne)
    OE = ora.Bat.dense(0, ne)
    _eq(gdk.BATgroupsum(V, G, E, gdk.TYPE_lng, True), ora.BATgroupsum(OV, OG, OE, ora.TYPE_lng, True))
    _eq(gdk.BATgroupcount(V, G, E, True), ora.BATgroupcount(OV, OG, OE, True))
    big = np.full(n, 1 << 62, np.int64)
    (B, OB), (G2, _) = _cols(gdk, ora, "lng", big, gids)
    with pytest.raises(gdk.GDKError, match="22003!overflow in sum aggregate"):
        gdk.BATgroupsum(B, G2, None, gdk.TYPE_lng, True)


@pytest.mark.parametrize("shift", [1, 3])
def test_sorted_groupsum_unaligned_views(gdk, ora, shift):
    """values and group ids as slices starting off a 16-byte boundary (the
    kernel's scalar-load path), runs spanning lanes and ranges"""
    r = rng(820 + shift)
    n = 150_011
    gids = _runs(r, n + shift, 37)
    vals = r.integers(-10**9, 10**9, n + shift).astype(np.int64)
    vals[r.random(n + shift) < 0.01] = NIL64
    (V, OV), (G, OG) = _cols(gdk, ora, "lng", vals, gids)
    Vs, Gs = gdk.BATslice(V, shift, n + shift), gdk.BATslice(G, shift, n + shift)
    OVs = ora.Bat.from_array(ora.TYPE_lng, vals[shift:], hseqbase=shift, sorted_=False, revsorted=False,
                             key=False, nonil=False)
    OGs = ora.Bat.from_array(ora.TYPE_oid, gids[shift:], hseqbase=shift, sorted_=True, nonil=True)
    _eq(gdk.BATgroupsum(Vs, Gs, None, gdk.TYPE_hge, True), ora.BATgroupsum(OVs, OGs, None, ora.TYPE_hge, True))
    _eq(gdk.BATgroupcount(Vs, Gs, None, False), ora.BATgroupcount(OVs, OGs, None, False))
    _eq(gdk.BATgroupmax(Vs, Gs, None, True), ora.BATgroupminmax(OVs, OGs, None, True, True))


def test_sorted_groupsum_empty_groups(gdk, ora):
    """groups without rows: ids starting above 0, gaps between runs (inside a
    lane, between lanes and between ranges), groups after the last id"""
    r = rng(830)
    n = 100_003
    gids = _runs(r, n, 9)
    gids = gids * 3 + 5 + (gids // 700) * 50
    vals = r.integers(-10**6, 10**6, n).astype(np.int64)
    (V, OV), (G, OG) = _cols(gdk, ora, "lng", vals, gids)
    ne = int(gids.max()) + 77
    E, OE = gdk.BAT.dense(0, ne), ora.Bat.dense(0, ne)
    for skip in (True, False):
        _eq(gdk.BATgroupsum(V, G, E, gdk.TYPE_lng, skip), ora.BATgroupsum(OV, OG, OE, ora.TYPE_lng, skip))
        _eq(gdk.BATgroupcount(V, G, E, skip), ora.BATgroupcount(OV, OG, OE, skip))
        _eq(gdk.BATgroupmin(V, G, E, skip), ora.BATgroupminmax(OV, OG, OE, False, skip))
        _eq(gdk.BATgroupmax(V, G, E, skip), ora.BATgroupminmax(OV, OG, OE, True, skip))
        a, rm, c = gdk.BATgroupavg3(V, G, E, skip)
        oa, orm, oc = ora.BATgroupavg3(OV, OG, OE, skip)
        for d, o in ((a, oa), (rm, orm), (c, oc)):
            assert np.array_equal(np.asarray(d.values()), np.asarray(o.values()))


@pytest.mark.parametrize("tname", ["bte", "int", "lng"])
def test_sorted_groupminmax_ties_nils_cands(gdk, ora, tname):
    """first row of the extreme on ties, the first nil without skip_nils,
    candidate oids in the result, groups spanning lanes and ranges"""
    r = rng(840)
    n = 250_001
    gids = _runs(r, n, 300)
    vals = r.integers(-3, 4, n).astype({"bte": np.int8, "int": np.int32, "lng": np.int64}[tname])
    nil = {"bte": -128, "int": -(1 << 31), "lng": NIL64}[tname]
    vals[r.random(n) < 0.001] = nil
    (V, OV), _ = _cols(gdk, ora, tname, vals, gids)
    cand = np.sort(r.choice(n, 200_000, replace=False)).astype(np.uint64)
    S = gdk.BAT.from_numpy(gdk.TYPE_oid, cand, sorted_=True, revsorted=False, key=True, nonil=True)
    OS = ora.Bat.from_array(ora.TYPE_oid, cand, sorted_=True, key=True, nonil=True)
    gs = gids[cand.astype(np.int64)]
    Gs = gdk.BAT.from_numpy(gdk.TYPE_oid, gs, hseqbase=int(cand[0]), sorted_=True, revsorted=False, key=False,
                            nonil=True)
    OGs = ora.Bat.from_array(ora.TYPE_oid, gs, hseqbase=int(cand[0]), sorted_=True, nonil=True)
    for skip in (True, False):
        _eq(gdk.BATgroupmin(V, Gs, None, skip, s=S), ora.BATgroupminmax(OV, OGs, None, False, skip, s=OS))
        _eq(gdk.BATgroupmax(V, Gs, None, skip, s=S), ora.BATgroupminmax(OV, OGs, None, True, skip, s=OS))


@pytest.mark.parametrize("tname", ["int", "lng"])
def test_one_row_groups(gdk, ora, tname):
    """strictly increasing group ids covering the group range (one row per
    group: what the owner of a distributed GROUP BY sees for clustered keys):
    sums, counts, min / max positions with nils, with and without extents,
    and ids that skip a group (not one row per group)"""
    r = rng(850)
    n = 200_003
    vals = r.integers(-10**6, 10**6, n).astype(np.int32 if tname == "int" else np.int64)
    nil = np.iinfo(vals.dtype).min
    vals[r.random(n) < 0.01] = nil
    tp, otp = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
    V = gdk.BAT.from_numpy(tp, vals, sorted_=False, revsorted=False, key=False, nonil=False)
    OV = ora.Bat.from_array(otp, vals)
    for gids, ext in ((np.arange(n, dtype=np.uint64), False), (np.arange(n, dtype=np.uint64), True),
                      (np.arange(n, dtype=np.uint64) + (np.arange(n) > n // 2), False)):
        G = gdk.BAT.from_numpy(gdk.TYPE_oid, gids, sorted_=True, revsorted=False, key=True, nonil=True)
        OG = ora.Bat.from_array(ora.TYPE_oid, gids, sorted_=True, key=True, nonil=True)
        E, OE = (gdk.BAT.dense(0, n), ora.Bat.dense(0, n)) if ext else (None, None)
        for skip in (True, False):
            _eq(gdk.BATgroupsum(V, G, E, gdk.TYPE_hge, skip), ora.BATgroupsum(OV, OG, OE, ora.TYPE_hge, skip))
            _eq(gdk.BATgroupmin(V, G, E, skip), ora.BATgroupminmax(OV, OG, OE, False, skip))
            _eq(gdk.BATgroupmax(V, G, E, skip), ora.BATgroupminmax(OV, OG, OE, True, skip))
    big = np.full(n, 1 << 40, np.int64)
    B = gdk.BAT.from_numpy(gdk.TYPE_lng, big, sorted_=False, revsorted=False, key=False, nonil=True)
    G = gdk.BAT.from_numpy(gdk.TYPE_oid, np.arange(n, dtype=np.uint64), sorted_=True, revsorted=False, key=True,
                           nonil=True)
    with pytest.raises(gdk.GDKError, match="22003!overflow in sum aggregate"):
        gdk.BATgroupsum(B, G, None, gdk.TYPE_int, True)
