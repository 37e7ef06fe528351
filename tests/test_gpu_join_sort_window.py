"""Parity of the device hash join, radix sort and RANGE window bounds with the
oracle (bit-exact oid lists, permutations and bounds)."""
import numpy as np
import pytest

from helpers import rng, with_nils

pytestmark = pytest.mark.gpu


def mk(G, tp, vals, **kw):
    # the ordering flags start unknown, as the oracle's (BATjoin computes them)
    for f in ("sorted_", "revsorted", "key"):
        kw.setdefault(f, False)
    return G.BAT.from_numpy(tp, np.asarray(vals), **kw)


def omk(O, tp, vals, **kw):
    return O.Bat.from_array(tp, np.asarray(vals), **kw)


# ---- hash join -----------------------------------------------------------------

@pytest.mark.parametrize("tname,dt", [("int", np.int32), ("lng", np.int64), ("sht", np.int16)])
@pytest.mark.parametrize("nil_matches", [False, True])
def test_join_random(gdk, ora, tname, dt, nil_matches):
    r = rng(81)
    tp = getattr(gdk, "TYPE_" + tname)
    nl, nr = 100_000, 30_000
    lv = with_nils(r.integers(-5000, 5000, nl).astype(dt), gdk.NIL[tp], 0.01, r)
    rv = with_nils(r.integers(-5000, 5000, nr).astype(dt), gdk.NIL[tp], 0.01, r)
    a, b = gdk.BATjoin(mk(gdk, tp, lv, hseqbase=10), mk(gdk, tp, rv, hseqbase=7),
                       nil_matches=nil_matches)
    oa, ob = ora.BATjoin(omk(ora, tp, lv, hseqbase=10), omk(ora, tp, rv, hseqbase=7),
                         nil_matches=nil_matches)
    assert np.array_equal(a.to_numpy(), oa.values())
    assert np.array_equal(b.to_numpy(), ob.values())


def test_join_candidates_and_orders(gdk, ora):
    r = rng(82)
    nl, nr = 50_000, 20_000
    # orders-like unique sparse keys, lineitem-like 1..7 lines per key, shuffled
    okeys = np.arange(nr, dtype=np.int32) * 32 + (np.arange(nr) % 8)
    r.shuffle(okeys)
    lkeys = r.choice(okeys, nl).astype(np.int32)
    sl = np.sort(r.choice(nl, 30_000, replace=False)).astype(np.uint64)
    a, b = gdk.BATjoin(mk(gdk, gdk.TYPE_int, lkeys), mk(gdk, gdk.TYPE_int, okeys),
                       sl=mk(gdk, gdk.TYPE_oid, sl), sr=gdk.BAT.dense(100, 15_000))
    oa, ob = ora.BATjoin(omk(ora, ora.TYPE_int, lkeys), omk(ora, ora.TYPE_int, okeys),
                         sl=omk(ora, ora.TYPE_oid, sl, sorted_=True), sr=ora.Bat.dense(100, 15_000))
    assert np.array_equal(a.to_numpy(), oa.values())
    assert np.array_equal(b.to_numpy(), ob.values())


@pytest.mark.parametrize("tname,dt", [("int", np.int32), ("lng", np.int64)])
def test_join_heavy_duplicates_fallback(gdk, ora, tname, dt):
    # one key repeated 1500 times on the build side exceeds the open-addressing
    # displacement bound -> CSR fallback; must give the same order
    r = rng(83)
    tp = getattr(gdk, "TYPE_" + tname)
    rv = np.concatenate([np.full(1500, 7), r.integers(0, 3000, 5000)]).astype(dt)
    r.shuffle(rv)
    lv = r.integers(0, 3000, 20_000).astype(dt)
    lv[::50] = 7
    a, b = gdk.BATjoin(mk(gdk, tp, lv), mk(gdk, tp, rv, hseqbase=5))
    oa, ob = ora.BATjoin(omk(ora, tp, lv), omk(ora, tp, rv, hseqbase=5))
    assert np.array_equal(a.to_numpy(), oa.values())
    assert np.array_equal(b.to_numpy(), ob.values())


@pytest.mark.parametrize("tname,dt", [("int", np.int32), ("oid", np.uint64), ("bte", np.int8)])
def test_join_unique_build(gdk, ora, tname, dt):
    # FK -> PK shape: every probe row has at most one match (single-pass path)
    r = rng(84)
    tp = getattr(gdk, "TYPE_" + tname)
    hi = 120 if tname == "bte" else 1 << 30
    rv = r.choice(np.arange(0, hi), min(100_000, hi), replace=False).astype(dt)
    lv = r.choice(np.arange(0, hi), 300_000).astype(dt)
    a, b = gdk.BATjoin(mk(gdk, tp, lv, hseqbase=3), mk(gdk, tp, rv))
    oa, ob = ora.BATjoin(omk(ora, tp, lv, hseqbase=3), omk(ora, tp, rv))
    assert np.array_equal(a.to_numpy(), oa.values())
    assert np.array_equal(b.to_numpy(), ob.values())


@pytest.mark.parametrize("part", ["1", "3"])
@pytest.mark.parametrize("nil_matches", [False, True])
@pytest.mark.parametrize("case", ["plain", "cands", "dups", "date", "skew", "big", "big_cands", "big_dups",
                                  "big_skew"])
def test_join_partitioned(gdk, ora, nil_matches, case, part, monkeypatch):
    monkeypatch.setenv("MGDK_JOIN_PART", part)     # the big cases: probe-side cut (see below)
    """4-byte keys, >= 64 Ki unique build rows: the global-table path (build
    side cut into per-partition LDS tables stored as one table, one ordered
    probe pass), nils on both sides, candidate lists, a duplicate build key
    (falls back), and a skewed build side whose largest partition overflows
    its global-table region (-> the radix-partitioned path).  The "big"
    cases (more than 2M build rows) take the radix-partitioned path, with
    candidates, a duplicate build key, and 9000 build keys in one of its
    512 partitions."""
    r = rng(85)
    big = case.startswith("big")
    nr, nl = (2_100_003, 3_000_001) if big else (700_001, 2_500_003)
    rv = r.choice(np.arange(-(1 << 30), 1 << 30, 7), nr, replace=False).astype(np.int32)
    if case.endswith("skew"):
        # 9000 keys whose multiplicative hash (key * 0x9E3779B1; top 7 bits =
        # partition of 700K build rows, top 9 bits of 2.1M) lands in
        # partition 0
        cinv = pow(0x9E3779B1, -1, 1 << 32)
        t = r.choice(1 << (23 if big else 25), 9000, replace=False).astype(np.uint64)
        sk = ((t * np.uint64(cinv)) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
        sk = sk[(sk != -(1 << 31)) & ~np.isin(sk, rv)]
        rv[: sk.size] = sk
    rv[123] = -(1 << 31)                                   # one nil (unique)
    lv = r.choice(rv, nl).astype(np.int32)
    lv[r.random(nl) < 0.05] = r.integers(-100, 100)        # misses
    lv[::997] = -(1 << 31)
    tp = gdk.TYPE_date if case == "date" else gdk.TYPE_int
    otp = ora.TYPE_date if case == "date" else ora.TYPE_int
    if case.endswith("dups"):
        rv[5] = rv[6]
    kw, okw = {}, {}
    if case.endswith("cands"):
        sl = np.sort(r.choice(nl, nl // 2, replace=False)).astype(np.uint64) + 11
        sr = np.sort(r.choice(nr, nr - 1000, replace=False)).astype(np.uint64) + 4
        kw = dict(sl=mk(gdk, gdk.TYPE_oid, sl), sr=mk(gdk, gdk.TYPE_oid, sr))
        okw = dict(sl=omk(ora, ora.TYPE_oid, sl, sorted_=True), sr=omk(ora, ora.TYPE_oid, sr, sorted_=True))
    a, b = gdk.BATjoin(mk(gdk, tp, lv, hseqbase=11), mk(gdk, tp, rv, hseqbase=4), nil_matches=nil_matches, **kw)
    oa, ob = ora.BATjoin(omk(ora, otp, lv, hseqbase=11), omk(ora, otp, rv, hseqbase=4),
                         nil_matches=nil_matches, **okw)
    assert np.array_equal(a.to_numpy(), oa.values())
    assert np.array_equal(b.to_numpy(), ob.values())


@pytest.mark.parametrize("tname", ["lng", "oid"])
@pytest.mark.parametrize("case", ["gt", "part", "probe_wide", "build_wide", "part_build_wide"])
def test_join_8byte_keys(gdk, ora, tname, case):
    """8-byte keys run the global-table / partitioned paths by their 4-byte
    images when every build value has one: nils (nil_matches both ways),
    probe values beyond 32 bits (no match), and a build value beyond 32 bits
    (falls back to the open-addressing path; on the partitioned path the
    flag is read after the restore) -- all bit-exact with the oracle."""
    r = rng(86)
    nr, nl = (2_100_003, 3_000_001) if case.startswith("part") else (700_001, 2_500_003)
    tp = getattr(gdk, "TYPE_" + tname)
    otp = getattr(ora, "TYPE_" + tname)
    if tname == "lng":
        rv = r.choice(np.arange(-(1 << 30), 1 << 30, 7), nr, replace=False).astype(np.int64)
        nil = np.iinfo(np.int64).min
    else:
        rv = r.choice(np.arange(0, 1 << 31, 7), nr, replace=False).astype(np.uint64)
        nil = np.uint64(1 << 63)
    rv[123] = nil
    lv = r.choice(rv, nl)
    lv[::997] = nil
    if case == "probe_wide":
        lv[5::1013] = (1 << 40) + 3 if tname == "oid" else -(1 << 40) - 3
    if case.endswith("build_wide"):
        rv[77] = (1 << 33) + 5
    for nm in (False, True):
        a, b = gdk.BATjoin(mk(gdk, tp, lv, hseqbase=11), mk(gdk, tp, rv, hseqbase=4), nil_matches=nm)
        oa, ob = ora.BATjoin(omk(ora, otp, lv, hseqbase=11), omk(ora, otp, rv, hseqbase=4), nil_matches=nm)
        assert np.array_equal(a.to_numpy(), oa.values()), nm
        assert np.array_equal(b.to_numpy(), ob.values()), nm


@pytest.mark.parametrize("tname", ["int", "lng", "oid", "date"])
@pytest.mark.parametrize("case", ["plain", "cands", "dup", "one_tile"])
def test_join_broadcast_small_build(gdk, ora, tname, case):
    """Build sides of <= 6144 unique keys: every workgroup builds the table
    in LDS and claims probe tiles (one launch): nils both ways, candidate
    lists on both sides, a probe of one tile, a duplicate build key (falls
    back) -- bit-exact with the oracle."""
    r = rng(87)
    nr, nl = 5000, (1500 if case == "one_tile" else 400_003)
    tp, otp = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
    dt = {"int": np.int32, "date": np.int32, "lng": np.int64, "oid": np.uint64}[tname]
    lo = 0 if tname == "oid" else -(1 << 30)
    rv = r.choice(np.arange(lo, 1 << 30, 3), nr, replace=False).astype(dt)
    nil = {np.int32: np.iinfo(np.int32).min, np.int64: np.iinfo(np.int64).min, np.uint64: np.uint64(1 << 63)}[dt]
    rv[17] = nil
    if case == "dup":
        rv[3] = rv[4]
    lv = r.choice(rv, nl)
    lv[r.random(nl) < 0.1] = rv[0] + 1                       # misses (not a multiple of 3 apart)
    lv[::331] = nil
    kw, okw = {}, {}
    if case == "cands":
        sl = np.sort(r.choice(nl, nl // 3, replace=False)).astype(np.uint64) + 9
        sr = np.sort(r.choice(nr, nr - 300, replace=False)).astype(np.uint64) + 2
        kw = dict(sl=mk(gdk, gdk.TYPE_oid, sl), sr=mk(gdk, gdk.TYPE_oid, sr))
        okw = dict(sl=omk(ora, ora.TYPE_oid, sl, sorted_=True), sr=omk(ora, ora.TYPE_oid, sr, sorted_=True))
    for nm in (False, True):
        a, b = gdk.BATjoin(mk(gdk, tp, lv, hseqbase=9), mk(gdk, tp, rv, hseqbase=2), nil_matches=nm, **kw)
        oa, ob = ora.BATjoin(omk(ora, otp, lv, hseqbase=9), omk(ora, otp, rv, hseqbase=2), nil_matches=nm, **okw)
        assert np.array_equal(a.to_numpy(), oa.values()), nm
        assert np.array_equal(b.to_numpy(), ob.values()), nm


def test_join_empty_sides(gdk):
    e = mk(gdk, gdk.TYPE_int, np.zeros(0, np.int32))
    x = mk(gdk, gdk.TYPE_int, np.arange(10, dtype=np.int32))
    for l, rr in ((e, x), (x, e), (e, e)):
        a, b = gdk.BATjoin(l, rr)
        assert a.count() == 0 and b.count() == 0


def test_join_duplicates_descending(gdk):
    l = rng(7).permutation(30).astype(np.int32)
    r = np.array([1, 2, 1, 3, 4, 5, 6, 7], np.int32)
    a, b = gdk.BATjoin(mk(gdk, gdk.TYPE_int, l), mk(gdk, gdk.TYPE_int, r))
    # joincost keeps the hash on r (lcost 68.8 > rcost 53.7): per left row in
    # order, right matches in descending position (chains prepend)
    want = [(i, j) for i, v in enumerate(l) for j in range(len(r) - 1, -1, -1) if r[j] == v]
    assert list(zip(a.to_numpy().tolist(), b.to_numpy().tolist())) == want


# ---- sort -----------------------------------------------------------------------

@pytest.mark.parametrize("tname,dt", [("bte", np.int8), ("sht", np.int16), ("int", np.int32), ("lng", np.int64)])
@pytest.mark.parametrize("reverse", [False, True])
def test_sort_int(gdk, ora, tname, dt, reverse):
    r = rng(91)
    tp = getattr(gdk, "TYPE_" + tname)
    n = 200_001
    vals = with_nils(r.integers(-100, 100, n).astype(dt), gdk.NIL[tp], 0.02, r)
    s, o, g = gdk.BATsort(mk(gdk, tp, vals, hseqbase=3), reverse=reverse, nilslast=reverse)
    os_, oo = ora.BATsort(omk(ora, tp, vals, hseqbase=3), reverse=reverse, nilslast=reverse)
    assert np.array_equal(s.to_numpy(), os_.values())
    assert np.array_equal(o.to_numpy(), oo.values())
    sv = s.to_numpy()
    want_g = np.concatenate([[0], np.cumsum(sv[1:] != sv[:-1])]).astype(np.uint64)
    assert np.array_equal(g.to_numpy(), want_g)


def test_sort_wide_range(gdk, ora):
    r = rng(92)
    vals = r.integers(-2**62, 2**62, 100_000).astype(np.int64)
    s, o, _ = gdk.BATsort(mk(gdk, gdk.TYPE_lng, vals))
    os_, oo = ora.BATsort(omk(ora, ora.TYPE_lng, vals))
    assert np.array_equal(o.to_numpy(), oo.values())


@pytest.mark.parametrize("dt,tname", [(np.float64, "dbl"), (np.float32, "flt")])
def test_sort_float(gdk, dt, tname):
    r = rng(93)
    n = 50_000
    vals = (r.integers(-50, 50, n) / 4).astype(dt)
    vals[r.random(n) < 0.02] = np.nan
    vals[r.random(n) < 0.01] = -0.0
    tp = getattr(gdk, "TYPE_" + tname)
    s, o, _ = gdk.BATsort(mk(gdk, tp, vals))
    key = np.where(np.isnan(vals), -np.inf, vals)          # nil first
    key = np.where(key == 0, 0.0, key)                      # -0 == +0
    want = np.argsort(key, kind="stable").astype(np.uint64)
    assert np.array_equal(o.to_numpy(), want)


def test_sort_float_groups(gdk):
    r = rng(94)
    vals = (r.integers(-20, 20, 30_000) / 2).astype(np.float64)
    vals[r.random(30_000) < 0.05] = np.nan
    vals[r.random(30_000) < 0.05] = -0.0
    s, o, g = gdk.BATsort(mk(gdk, gdk.TYPE_dbl, vals))
    key = np.where(np.isnan(vals), -np.inf, vals)
    key = np.where(key == 0, 0.0, key)
    perm = np.argsort(key, kind="stable")
    assert np.array_equal(o.to_numpy(), perm.astype(np.uint64))
    sv = s.to_numpy()
    assert np.array_equal(sv.view(np.uint64), vals[perm].view(np.uint64))   # -0 kept bit-exact
    ks = key[perm]
    want_g = np.concatenate([[0], np.cumsum(ks[1:] != ks[:-1])]).astype(np.uint64)
    assert np.array_equal(g.to_numpy(), want_g)


@pytest.mark.parametrize("tname,dt", [("sht", np.int16), ("int", np.int32), ("lng", np.int64)])
def test_sort_unstable_nils_other_end(gdk, ora, tname, dt):
    # reverse != nilslast (only without `stable`): GDKqsort (do_sort,
    # gdk_batop.c:2284-2302) -- its order of equal values, from the oracle
    r = rng(95)
    tp = getattr(gdk, "TYPE_" + tname)
    nil = gdk.NIL[tp]
    vals = with_nils(r.integers(-1000, 1000, 50_000).astype(dt), nil, 0.03, r)
    for reverse, nilslast in ((False, True), (True, False)):
        s, o, g = gdk.BATsort(mk(gdk, tp, vals), reverse=reverse, nilslast=nilslast, stable=False)
        os_, oo, og = ora.BATsort_full(omk(ora, tp, vals), reverse=reverse, nilslast=nilslast, stable=False)
        assert np.array_equal(o.to_numpy(), oo.values())
        assert np.array_equal(s.to_numpy(), os_.values())
        assert np.array_equal(g.to_numpy(), og.values())
        sv = s.to_numpy()
        isn = sv == nil
        k = int(isn.sum())
        assert (isn[-k:].all() if nilslast else isn[:k].all())


@pytest.mark.parametrize("n", [0, 1, 4095, 4097, 70_000])
def test_sort_sizes_and_constant(gdk, ora, n):
    r = rng(96)
    for vals in (r.integers(-50, 50, n).astype(np.int32), np.full(n, 7, np.int32)):
        s, o, g = gdk.BATsort(mk(gdk, gdk.TYPE_int, vals))
        if n == 0:
            assert s.count() == 0
            continue
        os_, oo = ora.BATsort(omk(ora, ora.TYPE_int, vals))
        assert np.array_equal(s.to_numpy(), os_.values())
        assert np.array_equal(o.to_numpy(), oo.values())


def test_sort_errors(gdk):
    b = mk(gdk, gdk.TYPE_int, np.array([3, 1, 2], np.int32))
    with pytest.raises(gdk.GDKError, match="stable sort cannot have reverse != nilslast"):
        gdk.BATsort(b, reverse=True, nilslast=False, stable=True)


# ---- RANGE window bounds ------------------------------------------------------------

def _window_data(r, nparts, plen, desc=False, nil_frac=0.0, shuffle=False):
    vals, bits = [], []
    for _ in range(nparts):
        gaps = r.integers(0, 5, plen)
        v = np.cumsum(gaps).astype(np.int64) + r.integers(-1000, 1000)
        nn = int(plen * nil_frac)
        if desc:
            v = v[::-1].copy()
            if nn:
                v[-nn:] = np.iinfo(np.int64).min
        elif nn:
            v[:nn] = np.iinfo(np.int64).min
        if shuffle:
            r.shuffle(v)
        vals.append(v)
        p = np.zeros(plen, np.int8)
        p[0] = 1
        bits.append(p)
    return np.concatenate(vals), np.concatenate(bits)


@pytest.mark.parametrize("desc,nil_frac,shuffle", [(False, 0.0, False), (False, 0.05, False),
                                                   (True, 0.05, False), (False, 0.02, True)])
@pytest.mark.parametrize("limit", [0, 3, 100, 2**63 - 1])
@pytest.mark.parametrize("preceding", [True, False])
def test_window_range_bounds(gdk, ora, desc, nil_frac, shuffle, limit, preceding):
    r = rng(101)
    vals, bits = _window_data(r, 37, 523, desc, nil_frac, shuffle)
    got = gdk.GDKanalyticalwindowbounds(mk(gdk, gdk.TYPE_lng, vals), mk(gdk, gdk.TYPE_bit, bits),
                                        limit, preceding).to_numpy()
    want = ora.rangebounds(omk(ora, ora.TYPE_lng, vals), omk(ora, ora.TYPE_bit, bits), limit,
                           preceding).values()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("limit", [700, 3000, 10**7])
@pytest.mark.parametrize("preceding", [True, False])
@pytest.mark.parametrize("desc", [False, True])
def test_window_long_frames(gdk, ora, limit, preceding, desc):
    # frames longer than the fast kernel's halo: some rows (limit 700) or all
    # rows (10**7 -> unresolved list overflows) go through the fix-up paths
    r = rng(103)
    vals, bits = _window_data(r, 6, 21_000, desc, 0.01, False)
    got = gdk.GDKanalyticalwindowbounds(mk(gdk, gdk.TYPE_lng, vals), mk(gdk, gdk.TYPE_bit, bits),
                                        limit, preceding).to_numpy()
    want = ora.rangebounds(omk(ora, ora.TYPE_lng, vals), omk(ora, ora.TYPE_bit, bits), limit,
                           preceding).values()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("plen", [1, 2, 4095, 4097])
def test_window_partition_sizes(gdk, ora, plen):
    # partitions shorter than / straddling the fast kernel's tiles
    r = rng(104)
    nparts = max(3, 30_000 // plen)
    vals, bits = _window_data(r, nparts, plen, False, 0.0, False)
    for preceding in (True, False):
        got = gdk.GDKanalyticalwindowbounds(mk(gdk, gdk.TYPE_lng, vals), mk(gdk, gdk.TYPE_bit, bits),
                                            6, preceding).to_numpy()
        want = ora.rangebounds(omk(ora, ora.TYPE_lng, vals), omk(ora, ora.TYPE_bit, bits), 6,
                               preceding).values()
        assert np.array_equal(got, want)


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("limit", [0, 5, 300])
def test_window_ragged_partitions_global_order(gdk, ora, desc, limit):
    # one ordered column cut into partitions of 1..3000 rows (config 5's
    # shape): stages with 0, a few or more than 16 partition starts
    r = rng(105)
    n = 200_000
    vals = np.cumsum(r.integers(0, 5, n)).astype(np.int64) - 10**5
    if desc:
        vals = vals[::-1].copy()
    bits = np.zeros(n, np.int8)
    at, k = 0, 0
    while at < n:
        bits[at] = 1
        at += int(r.integers(1, 40)) if k % 7 == 3 else int(r.integers(1, 3000))
        k += 1
    for preceding in (True, False):
        got = gdk.GDKanalyticalwindowbounds(mk(gdk, gdk.TYPE_lng, vals), mk(gdk, gdk.TYPE_bit, bits),
                                            limit, preceding).to_numpy()
        want = ora.rangebounds(omk(ora, ora.TYPE_lng, vals), omk(ora, ora.TYPE_bit, bits), limit,
                               preceding).values()
        assert np.array_equal(got, want)


def test_window_no_partitions_and_errors(gdk, ora):
    r = rng(102)
    vals = np.sort(r.integers(0, 10**6, 100_000)).astype(np.int64)
    got = gdk.GDKanalyticalwindowbounds(mk(gdk, gdk.TYPE_lng, vals), None, 50, True).to_numpy()
    want = ora.rangebounds(omk(ora, ora.TYPE_lng, vals), None, 50, True).values()
    assert np.array_equal(got, want)
    with pytest.raises(gdk.GDKError, match="non negative and non null"):
        gdk.GDKanalyticalwindowbounds(mk(gdk, gdk.TYPE_lng, vals), None, -1, True)
    big = np.array([-2**62 * 3 // 2, 2**62 * 3 // 2], np.int64)
    with pytest.raises(gdk.GDKError, match="22003!overflow in calculation"):
        gdk.GDKanalyticalwindowbounds(mk(gdk, gdk.TYPE_lng, big), None, 5, True)
    with pytest.raises(ora.OracleError, match="22003!overflow in calculation"):
        ora.rangebounds(omk(ora, ora.TYPE_lng, big), None, 5, True)


# ---- sub-sorting (o, g) and BATunique -----------------------------------------------

def test_sort_multicolumn_chain(gdk):
    # the reference's documented 3-column idiom (gdk_batop.c:2330-2334)
    r = rng(97)
    n = 60_000
    c1 = r.integers(0, 20, n).astype(np.int32)
    c2 = r.integers(-5, 5, n).astype(np.int64)
    c3 = r.integers(0, 1000, n).astype(np.int16)
    B1, B2, B3 = (mk(gdk, gdk.TYPE_int, c1, hseqbase=4), mk(gdk, gdk.TYPE_lng, c2, hseqbase=4),
                  mk(gdk, gdk.TYPE_sht, c3, hseqbase=4))
    s1, o1, g1 = gdk.BATsort(B1)
    s2, o2, g2 = gdk.BATsort(B2, o=o1, g=g1)
    s3, o3, g3 = gdk.BATsort(B3, o=o2, g=g2)
    want = np.lexsort((c3, c2, c1))
    assert np.array_equal(o3.to_numpy().astype(np.int64) - 4, want)
    assert np.array_equal(s3.to_numpy(), c3[want])
    key = np.stack([c1[want], c2[want], c3[want].astype(np.int64)], 1)
    newg = np.concatenate([[0], np.cumsum(np.any(key[1:] != key[:-1], axis=1))]).astype(np.uint64)
    assert np.array_equal(g3.to_numpy(), newg)


def test_sort_with_order_only_and_reverse(gdk):
    r = rng(98)
    n = 30_000
    a = r.integers(0, 100, n).astype(np.int32)
    b = r.integers(0, 100, n).astype(np.int32)
    _, oa, ga = gdk.BATsort(mk(gdk, gdk.TYPE_int, a))
    # o only, stable: b ordered, ties in a-order
    _, ob, _ = gdk.BATsort(mk(gdk, gdk.TYPE_int, b), o=oa, stable=True)
    pa = np.argsort(a, kind="stable")
    want = pa[np.argsort(b[pa], kind="stable")]
    assert np.array_equal(ob.to_numpy().astype(np.int64), want)
    # descending inside groups
    _, od, _ = gdk.BATsort(mk(gdk, gdk.TYPE_int, b), o=oa, g=ga, reverse=True, nilslast=True)
    want = np.lexsort((-b.astype(np.int64), a))
    assert np.array_equal(od.to_numpy().astype(np.int64), want)


def test_sort_sub_errors(gdk):
    b = mk(gdk, gdk.TYPE_int, np.array([3, 1, 2], np.int32))
    bad_g = mk(gdk, gdk.TYPE_oid, np.array([2, 1, 0], np.uint64))
    with pytest.raises(gdk.GDKError, match="g must have type oid, sorted"):
        gdk.BATsort(b, g=bad_g)
    with pytest.raises(gdk.GDKError, match="o must have type oid"):
        gdk.BATsort(b, o=mk(gdk, gdk.TYPE_oid, np.array([0, 1], np.uint64)))


@pytest.mark.parametrize("tname,dt", [("int", np.int32), ("lng", np.int64), ("bte", np.int8)])
def test_unique(gdk, tname, dt):
    r = rng(99)
    tp = getattr(gdk, "TYPE_" + tname)
    v = r.integers(-40, 40, 50_000).astype(dt)
    u = gdk.BATunique(mk(gdk, tp, v, hseqbase=7))
    _, first = np.unique(v, return_index=True)
    assert np.array_equal(u.to_numpy(), np.sort(first).astype(np.uint64) + 7)
    s = np.sort(r.choice(50_000, 9_000, replace=False)).astype(np.uint64) + 7
    u2 = gdk.BATunique(mk(gdk, tp, v, hseqbase=7), mk(gdk, gdk.TYPE_oid, s))
    sv = v[(s - 7).astype(np.int64)]
    _, f2 = np.unique(sv, return_index=True)
    assert np.array_equal(u2.to_numpy(), s[np.sort(f2)])


def test_sort_maltest_fixture(gdk):
    """algebra.sort of orderidx00 / orderidx04.maltest (the reference's answers)."""
    from helpers import FIX
    for fx in FIX["sort"]:
        for c in fx["cases"]:
            b = gdk.BAT.from_numpy(gdk.TYPE_int, np.array(c["values"], np.int32))
            srt, order, _ = gdk.BATsort(b, reverse=c["reverse"], nilslast=c["nilslast"], stable=c["stable"])
            assert [int(v) for v in srt.to_numpy()] == c["sorted"]
            if c["order"]:
                assert [int(v) for v in order.to_numpy()] == c["order_oids"]


@pytest.mark.parametrize("part", ["1", "3"])
@pytest.mark.parametrize("case", ["fk", "probe_skew", "lng_cands", "sparse_hits"])
def test_join_region_partitioned(gdk, ora, case, part, monkeypatch):
    """More than 2M unique build rows: the radix-partitioned path, with the
    probe side cut into subtile-local runs (MGDK_JOIN_PART=1, the default) or
    into partition-major runs after a histogram pass ("3").  An FK-shaped
    join of 12M x 3M (every row matches), a probe side with 60 % of its rows
    on one key, 8-byte keys with candidate lists on both sides, and 1 % hits
    -- all bit-exact with the oracle."""
    monkeypatch.setenv("MGDK_JOIN_PART", part)
    r = rng(88)
    nr, nl = 3_000_017, 12_000_029
    dt, tp, otp = np.int32, gdk.TYPE_int, ora.TYPE_int
    if case == "lng_cands":
        dt, tp, otp = np.int64, gdk.TYPE_lng, ora.TYPE_lng
    rv = r.permutation(np.arange(1, 4 * nr + 1, 4))[:nr].astype(dt)
    lv = r.choice(rv, nl).astype(dt)
    if case == "probe_skew":
        lv[r.random(nl) < 0.6] = rv[1000]
    if case == "sparse_hits":
        lv[r.random(nl) < 0.99] += 2                               # off the 4-grid: no match
    kw, okw = {}, {}
    if case == "lng_cands":
        lv[::1001] = np.iinfo(np.int64).min
        sl = np.sort(r.choice(nl, nl - nl // 3, replace=False)).astype(np.uint64) + 7
        sr = np.sort(r.choice(nr, nr - 5000, replace=False)).astype(np.uint64) + 2
        kw = dict(sl=mk(gdk, gdk.TYPE_oid, sl), sr=mk(gdk, gdk.TYPE_oid, sr))
        okw = dict(sl=omk(ora, ora.TYPE_oid, sl, sorted_=True), sr=omk(ora, ora.TYPE_oid, sr, sorted_=True))
    a, b = gdk.BATjoin(mk(gdk, tp, lv, hseqbase=7), mk(gdk, tp, rv, hseqbase=2), **kw)
    oa, ob = ora.BATjoin(omk(ora, otp, lv, hseqbase=7), omk(ora, otp, rv, hseqbase=2), **okw)
    assert np.array_equal(a.to_numpy(), oa.values())
    assert np.array_equal(b.to_numpy(), ob.values())
