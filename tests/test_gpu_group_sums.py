"""mgdk_group_sums_ordered: GROUP BY an ordered key with exact hge sums in
one fused pass over the values, against the oracle's BATgroup +
BATgroupsum(TYPE_hge, skip_nils) + BATproject(e, keys) on the same columns
(gdk_group.c:940-975, gdk_aggr.c:1009).  Runs of 1..7 rows (lineitem per
order), groups spanning many 2048-row tiles, one group over everything,
nil keys and values, all-nil groups, int / lng keys and values, 1..4 value
columns, reverse-sorted keys, row counts around the tile and lane sizes;
unordered keys are refused (None)."""
import numpy as np
import pytest

from helpers import rng

pytestmark = pytest.mark.gpu


def _keys(r, n, shape, dt):
    if shape == "orders":
        lens = r.integers(1, 8, n)
        k = np.repeat(np.arange(lens.size, dtype=np.int64) * 3 + 5, lens)[:n]
    elif shape == "long":
        k = np.arange(n, dtype=np.int64) // 10_007
    elif shape == "one":
        k = np.full(n, 42, np.int64)
    elif shape == "singles":
        k = np.arange(n, dtype=np.int64) * 2 - n
    else:   # "mixed": singletons, pairs and a few long runs
        lens = np.where(r.random(n) < 0.01, r.integers(2000, 9000, n), r.integers(1, 3, n))
        k = np.repeat(np.arange(lens.size, dtype=np.int64), lens)[:n]
    return k.astype(dt)


def _model(ora, okeys, ovals):
    g, e, h = ora.BATgroup(okeys)
    sums = [ora.BATgroupsum(v, g, e, ora.TYPE_hge) for v in ovals]
    return e, h, ora.BATproject(e, okeys), sums


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("n", [1, 7, 8, 2047, 2049, 1_000_003])
@pytest.mark.parametrize("shape", ["orders", "long", "one", "singles", "mixed"])
def test_group_sums_ordered(gdk, ora, n, shape, fused, monkeypatch):
    # fused: group ids by the look-back inside the sums pass (default);
    # "0": the count pass + scan first (MGDK_GS_FUSED, read per call)
    monkeypatch.setenv("MGDK_GS_FUSED", fused)
    r = rng(n + len(shape))
    k = _keys(r, n, shape, np.int64)
    vals = [r.integers(-10**12, 10**12, n).astype(np.int64) for _ in range(2)]
    vals[0][r.random(n) < 0.02] = np.iinfo(np.int64).min
    if shape == "orders" and n > 100:
        # an all-nil group in the second column: rows of the key k[50]
        vals[1][k == k[50]] = np.iinfo(np.int64).min
    kb = gdk.BAT.from_numpy(gdk.TYPE_lng, k, hseqbase=13)
    kb.s.tsorted, kb.s.trevsorted = 1, int(shape == "one" or n <= 1)
    vb = [gdk.BAT.from_numpy(gdk.TYPE_lng, v, hseqbase=13) for v in vals]
    res = gdk.group_sums_ordered(kb, vb)
    assert res is not None
    e, h, gk, sums = res
    ok = ora.Bat.from_array(ora.TYPE_lng, k, hseqbase=13, sorted_=True)
    ov = [ora.Bat.from_array(ora.TYPE_lng, v, hseqbase=13) for v in vals]
    oe, oh, ogk, osums = _model(ora, ok, ov)
    assert np.array_equal(e.to_numpy(), oe.values())
    assert np.array_equal(h.to_numpy(), oh.values())
    assert np.array_equal(gk.to_numpy(), ogk.values())
    for s, os_ in zip(sums, osums):
        assert s.values() == list(os_.values())


@pytest.mark.parametrize("nv", [1, 3, 4])
@pytest.mark.parametrize("kt,vt", [("int", "int"), ("int", "lng"), ("lng", "int")])
def test_group_sums_types(gdk, ora, nv, kt, vt):
    r = rng(nv * 7 + len(kt + vt))
    n = 300_011
    kd = np.int32 if kt == "int" else np.int64
    vd = np.int32 if vt == "int" else np.int64
    k = _keys(r, n, "mixed", kd)
    k[:100] = np.iinfo(kd).min            # nil keys group together (sorted first)
    vals = [r.integers(-10**6, 10**6, n).astype(vd) for _ in range(nv)]
    for v in vals:
        v[r.random(n) < 0.05] = np.iinfo(vd).min
    tk, tv = getattr(gdk, "TYPE_" + kt), getattr(gdk, "TYPE_" + vt)
    kb = gdk.BAT.from_numpy(tk, k, hseqbase=0)
    kb.s.tsorted, kb.s.trevsorted = 1, 0
    res = gdk.group_sums_ordered(kb, [gdk.BAT.from_numpy(tv, v) for v in vals])
    assert res is not None
    e, h, gk, sums = res
    otk, otv = getattr(ora, "TYPE_" + kt), getattr(ora, "TYPE_" + vt)
    ok = ora.Bat.from_array(otk, k, sorted_=True)
    oe, oh, ogk, osums = _model(ora, ok, [ora.Bat.from_array(otv, v) for v in vals])
    assert np.array_equal(e.to_numpy(), oe.values())
    assert np.array_equal(h.to_numpy(), oh.values())
    # keys come back widened to lng (nil stays nil)
    want = np.asarray(ogk.values()).astype(np.int64)
    if kt == "int":
        want[want == np.iinfo(np.int32).min] = np.iinfo(np.int64).min
    assert np.array_equal(gk.to_numpy(), want)
    for s, os_ in zip(sums, osums):
        assert s.values() == list(os_.values())


def test_group_sums_revsorted_and_refused(gdk, ora):
    r = rng(5)
    n = 100_000
    k = _keys(r, n, "orders", np.int64)[::-1].copy()
    v = r.integers(0, 1000, n).astype(np.int64)
    kb = gdk.BAT.from_numpy(gdk.TYPE_lng, k, sorted_=False, revsorted=False, key=False)
    res = gdk.group_sums_ordered(kb, [gdk.BAT.from_numpy(gdk.TYPE_lng, v)])
    assert res is not None                    # found reverse ordered by the scan
    e, h, gk, sums = res
    ok = ora.Bat.from_array(ora.TYPE_lng, k, revsorted=True)
    oe, oh, ogk, osums = _model(ora, ok, [ora.Bat.from_array(ora.TYPE_lng, v)])
    assert np.array_equal(e.to_numpy(), oe.values())
    assert np.array_equal(h.to_numpy(), oh.values())
    assert sums[0].values() == list(osums[0].values())
    shuffled = r.permutation(k)
    kb2 = gdk.BAT.from_numpy(gdk.TYPE_lng, shuffled, sorted_=False, revsorted=False, key=False)
    assert gdk.group_sums_ordered(kb2, [gdk.BAT.from_numpy(gdk.TYPE_lng, v)]) is None


@pytest.mark.parametrize("case", ["late", "early", "over_limit_late"])
def test_group_prefix_then_all(gdk, ora, case):
    """BATgroup's low-cardinality path numbers the groups of a prefix of the
    column first; a key first seen past the prefix makes it read every tile
    and assign again -- ids, extents and histogram equal the oracle's either
    way, and more than 3072 groups appearing late still leave the path."""
    r = rng(len(case))
    n = 2_000_003
    k = r.integers(0, 10, n).astype(np.int32)
    if case == "late":
        k[1_500_000:] = r.integers(0, 40, n - 1_500_000)       # 30 new keys late
    elif case == "over_limit_late":
        k[1_500_000:] = r.integers(0, 5000, n - 1_500_000)
    kb = gdk.BAT.from_numpy(gdk.TYPE_int, k, hseqbase=3)
    g, e, h = gdk.BATgroup(kb)
    og, oe, oh = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, k, hseqbase=3))
    assert np.array_equal(g.to_numpy(), og.values())
    assert np.array_equal(e.to_numpy(), oe.values())
    assert np.array_equal(h.to_numpy(), oh.values())


@pytest.mark.parametrize("glen", [20_000_000, 3_000_017, 40_000])
def test_group_sums_long_runs(gdk, ora, glen):
    """groups spanning thousands of tiles: the edge records combine over
    several fold levels (k_gs_edges_fold) instead of one serial walk"""
    n = 20_000_000
    r = rng(glen)
    k = (np.arange(n, dtype=np.int64) // glen) * 7 - 3
    v = r.integers(-10**12, 10**12, n).astype(np.int64)
    v[r.random(n) < 0.01] = np.iinfo(np.int64).min
    kb = gdk.BAT.from_numpy(gdk.TYPE_lng, k)
    kb.s.tsorted, kb.s.trevsorted = 1, int(glen >= n)
    res = gdk.group_sums_ordered(kb, [gdk.BAT.from_numpy(gdk.TYPE_lng, v)])
    assert res is not None
    e, h, gk, sums = res
    oe, oh, ogk, osums = _model(ora, ora.Bat.from_array(ora.TYPE_lng, k, sorted_=True),
                                [ora.Bat.from_array(ora.TYPE_lng, v)])
    assert np.array_equal(h.to_numpy(), oh.values())
    assert np.array_equal(gk.to_numpy(), ogk.values())
    assert sums[0].values() == list(osums[0].values())
