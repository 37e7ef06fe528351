"""Parity of the HIP path (libmgdk.so through the C ABI) with the oracle and
with the reference's own fixtures.  Bit-exact for every oid / integer result."""
import numpy as np
import pytest

from helpers import FIX, replay_project, replay_select, rng, with_nils

pytestmark = pytest.mark.gpu


def mk(G, tp, vals, **kw):
    return G.BAT.from_numpy(tp, np.asarray(vals), **kw)


def omk(O, tp, vals, **kw):
    return O.Bat.from_array(tp, np.asarray(vals), **kw)


# ---- select ---------------------------------------------------------------

def test_select_maltest_fixture(gdk):
    bad = replay_select(gdk, lambda tp, v: mk(gdk, tp, np.array(v, np.int32)), gdk.TYPE_int,
                        gdk.NIL[gdk.TYPE_int])
    assert not bad, bad[:3]


SEL_TYPES = [("bte", np.int8), ("sht", np.int16), ("int", np.int32), ("lng", np.int64),
             ("dbl", np.float64), ("flt", np.float32)]


def _cases(lo, hi, nil):
    vs = [lo, hi, (lo + hi) // 2 if not isinstance(lo, float) else (lo + hi) / 2]
    out = []
    for tl in vs + [nil]:
        for th in vs + [nil, None]:
            for li in (False, True):
                for hi_ in (False, True):
                    for anti in (False, True):
                        for nm in (False, True):
                            out.append((tl, th, li, hi_, anti, nm))
    return out


@pytest.mark.parametrize("tname,dt", SEL_TYPES)
def test_select_random_parity(gdk, ora, tname, dt):
    r = rng(11)
    tp = getattr(gdk, "TYPE_" + tname)
    n = 50_000
    if dt in (np.float32, np.float64):
        vals = (r.integers(-50, 50, n)).astype(dt)
        vals[r.random(n) < 0.05] = np.nan
        nil = float("nan")
        lo, hi = -20.0, 20.0
    else:
        vals = r.integers(-50, 50, n).astype(dt)
        nil = gdk.NIL[tp]
        vals = with_nils(vals, nil, 0.05, r)
        lo, hi = -20, 20
    b = mk(gdk, tp, vals)
    ob = omk(ora, tp, vals)
    # candidate lists: none, dense slice, materialized
    cands = [(None, None),
             (gdk.BAT.dense(1000, 30_000), ora.Bat.dense(1000, 30_000))]
    co = np.sort(r.choice(n, 20_000, replace=False)).astype(np.uint64)
    cands.append((mk(gdk, gdk.TYPE_oid, co, sorted_=True, key=True),
                  omk(ora, ora.TYPE_oid, co, sorted_=True, key=True)))
    for tl, th, li, hi_, anti, nm in _cases(lo, hi, nil):
        for gs, os_ in cands:
            try:
                want = ora.BATselect(ob, os_, tl, th, li, hi_, anti, nm).values()
            except ora.OracleError as e:
                with pytest.raises(gdk.GDKError):
                    gdk.BATselect(b, gs, tl, th, li, hi_, anti, nm)
                continue
            got = gdk.BATselect(b, gs, tl, th, li, hi_, anti, nm)
            gv = got.values()
            assert np.array_equal(np.asarray(gv, np.uint64), np.asarray(want, np.uint64)), \
                (tname, tl, th, li, hi_, anti, nm)
            # virtualised when dense, like virtualize()
            if len(gv) <= 1 or int(gv[-1]) - int(gv[0]) == len(gv) - 1:
                assert got.is_dense()


@pytest.mark.parametrize("tname,dt", SEL_TYPES)
def test_select_through_candidate_bitmap(gdk, ora, tname, dt):
    """A candidate list that is a select result of >= 1M oids keeps its scan
    bitmap; BATselect through it streams b and ANDs the candidate bits (no
    oid reads, lines without a candidate not fetched).  Every predicate form
    against the oracle with the same list as an ordinary oid list, chained
    selects (the Q6 shape), a head-offset b and an unaligned view (the oid
    path)."""
    r = rng(12)
    n = 3_000_017
    tp = getattr(gdk, "TYPE_" + tname)
    key = r.integers(0, 100, n).astype(np.int32)
    K = mk(gdk, gdk.TYPE_int, key, nonil=True, hseqbase=40)
    s1 = gdk.BATthetaselect(K, None, 60, "<")            # ~1.8M oids -> bitmap kept
    s1v = s1.to_numpy()
    assert s1v.size >= 1 << 20
    if dt in (np.float32, np.float64):
        vals = r.integers(-50, 50, n).astype(dt)
        vals[r.random(n) < 0.05] = np.nan
        nil, lo, hi = float("nan"), -20.0, 20.0
    else:
        vals = with_nils(r.integers(-50, 50, n).astype(dt), gdk.NIL[tp], 0.05, r)
        nil, lo, hi = gdk.NIL[tp], -20, 20
    b = mk(gdk, tp, vals, hseqbase=40)
    ob = omk(ora, tp, vals, hseqbase=40)
    os1 = omk(ora, ora.TYPE_oid, s1v, sorted_=True, key=True)
    for tl, th, li, hi_, anti, nm in _cases(lo, hi, nil):
        try:
            want = ora.BATselect(ob, os1, tl, th, li, hi_, anti, nm).values()
        except ora.OracleError:
            with pytest.raises(gdk.GDKError):
                gdk.BATselect(b, s1, tl, th, li, hi_, anti, nm)
            continue
        got = gdk.BATselect(b, s1, tl, th, li, hi_, anti, nm).values()
        assert np.array_equal(np.asarray(got, np.uint64), np.asarray(want, np.uint64)), \
            (tname, tl, th, li, hi_, anti, nm)
    # chain: the result of a bitmap select keeps its own bitmap
    s2 = gdk.BATselect(b, s1, type(lo)(-45), type(hi)(45), True, True, False)   # ~1.5M oids
    assert s2.count() >= 1 << 20
    k2 = gdk.BATthetaselect(K, s2, 30, "<").to_numpy()
    want2 = s2.to_numpy()[key[s2.to_numpy().astype(np.int64) - 40] < 30]
    assert np.array_equal(k2, want2)
    # a view of b three rows in: candidate slots no longer 16-B aligned
    # against it -> the oid-list path, same answer
    v = gdk.BAT(gdk.lib().mgdk_BATslice(b.ptr, 3, n))
    got = gdk.BATselect(v, s1, lo, hi, True, True, False).to_numpy()
    sel = s1v[s1v >= 43]
    vv = vals[sel.astype(np.int64) - 40]
    keep = (vv >= lo) & (vv <= hi) if dt not in (np.float32, np.float64) else (vv >= lo) & (vv <= hi)
    if dt not in (np.float32, np.float64):
        keep &= vv != nil
    assert np.array_equal(got, sel[keep])


def test_select_large_lookback(gdk):
    """Many tiles: exercises the decoupled look-back across the whole grid."""
    r = rng(3)
    n = 30_000_001
    vals = r.integers(0, 1000, n, dtype=np.int32)
    b = mk(gdk, gdk.TYPE_int, vals, nonil=True)
    for thr in (1, 100, 500, 999):
        got = gdk.BATthetaselect(b, None, thr, "<").to_numpy()
        want = np.flatnonzero(vals < thr).astype(np.uint64)
        assert np.array_equal(got, want), thr


def test_select_unaligned_view(gdk):
    r = rng(5)
    vals = r.integers(0, 10, 100_003, dtype=np.int32)
    b = mk(gdk, gdk.TYPE_int, vals)
    v = gdk.BAT(gdk.lib().mgdk_BATslice(b.ptr, 3, 100_001))
    got = gdk.BATthetaselect(v, None, 5, "<").to_numpy()
    want = (np.flatnonzero(vals[3:100_001] < 5) + 3).astype(np.uint64)
    assert np.array_equal(got, want)


# ---- project / calc / sum ---------------------------------------------------

@pytest.mark.parametrize("tname,dt", [("bte", np.int8), ("int", np.int32), ("lng", np.int64),
                                      ("dbl", np.float64)])
def test_project(gdk, ora, tname, dt):
    r = rng(21)
    tp = getattr(gdk, "TYPE_" + tname)
    vals = r.integers(-100, 100, 10_000).astype(dt)
    b = mk(gdk, tp, vals, hseqbase=500)
    l = np.sort(r.choice(np.arange(500, 10_500), 3000, replace=False)).astype(np.uint64)
    l2 = l.copy()
    l2[7] = gdk.OID_NIL
    for arr in (l, l2):
        got = gdk.BATproject(mk(gdk, gdk.TYPE_oid, arr), b).to_numpy()
        want = ora.BATproject(omk(ora, ora.TYPE_oid, arr), omk(ora, tp, vals, hseqbase=500)).values()
        assert np.array_equal(got.view(np.uint8), np.asarray(want, dt).view(np.uint8))
    bad = l.copy()
    bad[0] = 3
    with pytest.raises(gdk.GDKError, match="does not match always"):
        gdk.BATproject(mk(gdk, gdk.TYPE_oid, bad), b)
    # dense left: slice
    s = gdk.BATproject(gdk.BAT.dense(600, 100, hseqbase=7), b)
    assert s.hseqbase == 7 and np.array_equal(s.to_numpy(), vals[100:200])


@pytest.mark.parametrize("op", ["+", "-", "*"])
@pytest.mark.parametrize("t1,t2,tp", [("int", "int", "int"), ("int", "int", "lng"),
                                      ("lng", "lng", "lng"), ("lng", "lng", "hge"),
                                      ("sht", "bte", "sht")])
def test_calc(gdk, ora, op, t1, t2, tp):
    r = rng(31)
    T1, T2, TP = (getattr(gdk, "TYPE_" + x) for x in (t1, t2, tp))
    dt = {"bte": np.int8, "sht": np.int16, "int": np.int32, "lng": np.int64}
    n = 20_000
    a = with_nils(r.integers(-1000, 1000, n).astype(dt[t1]), gdk.NIL[T1], 0.02, r)
    b = with_nils(r.integers(-100, 100, n).astype(dt[t2]), gdk.NIL[T2], 0.02, r)
    fn = {"+": gdk.BATcalcadd, "-": gdk.BATcalcsub, "*": gdk.BATcalcmul}[op]
    ga, gb = mk(gdk, T1, a), mk(gdk, T2, b)
    oa, ob = omk(ora, T1, a), omk(ora, T2, b)
    try:
        want = ora.BATcalc(op, oa, ob, TP).values()
    except ora.OracleError as e:
        with pytest.raises(gdk.GDKError) as ei:
            fn(ga, gb, TP)
        assert str(ei.value) == str(e)
        return
    got = fn(ga, gb, TP).values()
    assert [int(x) for x in got] == [int(x) for x in want]


def test_calc_overflow_matches(gdk, ora):
    a = np.array([1, 5, 2**30, 7, 2**30], np.int32)
    ga, oa = mk(gdk, gdk.TYPE_int, a), omk(ora, ora.TYPE_int, a)
    with pytest.raises(gdk.GDKError) as ei:
        gdk.BATcalcmulcst(ga, 4, gdk.TYPE_int, gdk.TYPE_int)
    with pytest.raises(ora.OracleError) as eo:
        ora.BATcalc("*", oa, None, ora.TYPE_int, c2=4, t2=ora.TYPE_int)
    assert str(ei.value) == str(eo.value)
    assert str(ei.value).startswith("22003!overflow in calculation 1073741824*4")


def test_calc_cst_and_candidates(gdk, ora):
    r = rng(41)
    a = r.integers(0, 100, 5000).astype(np.int64)
    ga, oa = mk(gdk, gdk.TYPE_lng, a), omk(ora, ora.TYPE_lng, a)
    got = gdk.BATcalccstsub(100, gdk.TYPE_lng, ga, gdk.TYPE_lng).values()
    want = ora.BATcalc("-", None, oa, ora.TYPE_lng, c1=100, t1=ora.TYPE_lng).values()
    assert np.array_equal(got, want)
    s = gdk.BAT.dense(100, 2000)
    got = gdk.BATcalcmulcst(ga, 3, gdk.TYPE_lng, gdk.TYPE_hge, s=s)
    want = ora.BATcalc("*", oa, None, ora.TYPE_hge, s=ora.Bat.dense(100, 2000), c2=3,
                       t2=ora.TYPE_lng)
    assert got.values() == want.values()


@pytest.mark.parametrize("n", [1, 2, 7, 100_003])
def test_calc_pair_path(gdk, ora, n):
    """The paired kernel (two elements per lane, 16-byte loads / stores) for
    dense 8 / 16-byte operands: odd counts, sliced operands (element 0 on an
    8-byte boundary -> the single-element kernel), hge x lng -> hge (Q1's
    charge), constants, nils, and an overflow at an odd position."""
    r = rng(43)
    a = with_nils(r.integers(-10**6, 10**6, n + 3).astype(np.int64), gdk.NIL[gdk.TYPE_lng], 0.03, r)
    b = with_nils(r.integers(-10**6, 10**6, n + 3).astype(np.int64), gdk.NIL[gdk.TYPE_lng], 0.03, r)
    ga, gb = mk(gdk, gdk.TYPE_lng, a), mk(gdk, gdk.TYPE_lng, b)
    oa, ob = omk(ora, ora.TYPE_lng, a), omk(ora, ora.TYPE_lng, b)
    for lo in (0, 1, 2):
        sa, sb = gdk.BATslice(ga, lo, lo + n), gdk.BATslice(gb, lo, lo + n)
        wa, wb = omk(ora, ora.TYPE_lng, a[lo:lo + n]), omk(ora, ora.TYPE_lng, b[lo:lo + n])
        for tp in (gdk.TYPE_lng, gdk.TYPE_hge):
            got = gdk.BATcalcmul(sa, sb, tp)
            want = ora.BATcalc("*", wa, wb, tp)
            assert [int(x) for x in got.values()] == [int(x) for x in want.values()]
            assert (got.s.tnonil, got.s.tnil, got.count()) == (want.s.nonil, want.s.nil, want.s.count)
        dp = gdk.BATcalcmul(sa, sb, gdk.TYPE_hge)
        odp = ora.BATcalc("*", wa, wb, ora.TYPE_hge)
        got = gdk.BATcalcmul(dp, sb, gdk.TYPE_hge).values()
        want = ora.BATcalc("*", odp, wb, ora.TYPE_hge).values()
        assert [int(x) for x in got] == [int(x) for x in want]
        got = gdk.BATcalccstsub(100, gdk.TYPE_lng, sa, gdk.TYPE_lng).values()
        want = ora.BATcalc("-", None, wa, ora.TYPE_lng, c1=100, t1=ora.TYPE_lng).values()
        assert [int(x) for x in got] == [int(x) for x in want]
    if n >= 7:
        big = np.arange(n, dtype=np.int64)
        big[5] = 2**62
        g, o = mk(gdk, gdk.TYPE_lng, big), omk(ora, ora.TYPE_lng, big)
        with pytest.raises(gdk.GDKError) as ei:
            gdk.BATcalcmulcst(g, 4, gdk.TYPE_lng, gdk.TYPE_lng)
        with pytest.raises(ora.OracleError) as eo:
            ora.BATcalc("*", o, None, ora.TYPE_lng, c2=4, t2=ora.TYPE_lng)
        assert str(ei.value) == str(eo.value)


@pytest.mark.parametrize("tname,tp", [("int", "lng"), ("lng", "lng"), ("lng", "hge"),
                                      ("hge", "hge"), ("int", "dbl")])
def test_sum(gdk, ora, tname, tp):
    r = rng(51)
    T, TP = getattr(gdk, "TYPE_" + tname), getattr(gdk, "TYPE_" + tp)
    n = 100_000
    if tname == "hge":
        v = r.integers(-10**6, 10**6, n)
        raw = np.zeros((n, 2), np.uint64)
        raw[:, 0] = v.astype(np.int64).view(np.uint64)
        raw[:, 1] = np.where(v < 0, np.uint64(2**64 - 1), np.uint64(0))
        vals = raw
    else:
        dt = {"int": np.int32, "lng": np.int64}[tname]
        vals = with_nils(r.integers(-10**6, 10**6, n).astype(dt), gdk.NIL[T], 0.01, r)
    g, o = mk(gdk, T, vals), omk(ora, T, vals)
    for skip in (True, False):
        for nie in (True, False):
            a = gdk.BATsum(TP, g, skip_nils=skip, nil_if_empty=nie)
            b = ora.BATsum(TP, o, skip_nils=skip, nil_if_empty=nie)
            if tp == "dbl":
                assert (np.isnan(a) and np.isnan(b)) or a == b
            else:
                assert a == b


def test_sum_overflow(gdk, ora):
    big = np.array([2**62, 2**62, -2**62, 5], np.int64)
    g, o = mk(gdk, gdk.TYPE_lng, big), omk(ora, ora.TYPE_lng, big)
    with pytest.raises(ora.OracleError, match="overflow in sum"):
        ora.BATsum(ora.TYPE_lng, o)
    with pytest.raises(gdk.GDKError, match="22003!overflow in sum aggregate"):
        gdk.BATsum(gdk.TYPE_lng, g)
    ok = np.array([2**62, -2**62, 2**62, 5], np.int64)
    assert gdk.BATsum(gdk.TYPE_lng, mk(gdk, gdk.TYPE_lng, ok)) == 2**62 + 5


def test_bigsum_fixture(gdk):
    fx = FIX["bigsum"]
    vals = np.full(fx["repeat_count"] + 1, fx["repeat_value"], np.int64)
    vals[0] = fx["first"]
    s = gdk.BATsum(gdk.TYPE_dbl, mk(gdk, gdk.TYPE_lng, vals))
    assert "%.10g" % s == fx["expected"]


# ---- group and grouped aggregates --------------------------------------------

def test_project_maltest_fixture(gdk):
    """algebra.projection of algebra.select results (tst033 / tst034 /
    orderidx02.maltest) on the device"""
    bad = replay_project(gdk, lambda tp, v: mk(gdk, tp, np.array(v, np.int32)), gdk.TYPE_int,
                         gdk.NIL[gdk.TYPE_int])
    assert not bad, bad[:3]


@pytest.mark.parametrize("name", ["group_tst1500", "group_tst1503"])
def test_group_fixture(gdk, name):
    fx = FIX[name]
    g, e, h = gdk.BATgroup(mk(gdk, gdk.TYPE_bte, np.array(fx["values"], np.int8)))
    assert list(g.values()) == fx["expected"]["g1"]
    assert list(e.values()) == fx["expected"]["e1"]
    assert list(h.values()) == fx["expected"]["h1"]


@pytest.mark.parametrize("tname,dt,card", [("bte", np.int8, 20), ("int", np.int32, 1000),
                                           ("lng", np.int64, 100_000), ("sht", np.int16, 3000)])
def test_group_random(gdk, ora, tname, dt, card):
    r = rng(61)
    tp = getattr(gdk, "TYPE_" + tname)
    n = 200_000
    vals = with_nils(r.integers(-card // 2, card // 2, n).astype(dt), gdk.NIL[tp], 0.01, r)
    g, e, h = gdk.BATgroup(mk(gdk, tp, vals))
    og, oe, oh = ora.BATgroup(omk(ora, tp, vals))
    assert np.array_equal(g.to_numpy(), og.values())
    assert np.array_equal(e.to_numpy(), oe.values())
    assert np.array_equal(h.to_numpy(), oh.values())
    # subgroup by a second column
    v2 = r.integers(0, 7, n).astype(np.int8)
    g2, e2, h2 = gdk.BATgroup(mk(gdk, gdk.TYPE_bte, v2), None, g)
    og2, oe2, oh2 = ora.BATgroup(omk(ora, ora.TYPE_bte, v2), None, og)
    assert np.array_equal(g2.to_numpy(), og2.values())
    assert np.array_equal(e2.to_numpy(), oe2.values())
    assert np.array_equal(h2.to_numpy(), oh2.values())


@pytest.mark.parametrize("tname,dt", [("lng", np.int64), ("dbl", np.float64)])
def test_group_low_cardinality_edges(gdk, ora, tname, dt):
    """LDS path: the all-ones key image (lng -1), -0.0 == 0.0, NaN nils,
    candidate lists and tiles of 64 Ki rows; > 3072 groups fall back."""
    r = rng(62)
    tp = getattr(gdk, "TYPE_" + tname)
    n = 300_001
    vals = r.integers(-3, 40, n).astype(dt)
    if dt == np.float64:
        vals[r.random(n) < 0.01] = np.nan
        vals[r.random(n) < 0.01] = -0.0
    cand = np.sort(r.choice(n, 200_000, replace=False)).astype(np.uint64)
    for s in (None, cand):
        S = mk(gdk, gdk.TYPE_oid, s) if s is not None else None
        OS = omk(ora, ora.TYPE_oid, s, sorted_=True) if s is not None else None
        g, e, h = gdk.BATgroup(mk(gdk, tp, vals), S)
        og, oe, oh = ora.BATgroup(omk(ora, tp, vals), OS)
        assert np.array_equal(g.to_numpy(), og.values())
        assert np.array_equal(e.to_numpy(), oe.values())
        assert np.array_equal(h.to_numpy(), oh.values())
    wide = r.integers(0, 5000, n).astype(dt)
    g, e, h = gdk.BATgroup(mk(gdk, tp, wide))
    og, oe, oh = ora.BATgroup(omk(ora, tp, wide))
    assert np.array_equal(g.to_numpy(), og.values()) and np.array_equal(h.to_numpy(), oh.values())


def test_grouped_aggregates(gdk, ora):
    r = rng(71)
    n = 300_000
    for ng in (1, 3, 6, 500):
        gid = r.integers(0, ng, n).astype(np.uint64)
        vals = with_nils(r.integers(-10**9, 10**9, n).astype(np.int64), gdk.NIL[gdk.TYPE_lng],
                         0.001, r)
        gg, og = mk(gdk, gdk.TYPE_oid, gid), omk(ora, ora.TYPE_oid, gid)
        gv, ov = mk(gdk, gdk.TYPE_lng, vals), omk(ora, ora.TYPE_lng, vals)
        for skip in (True, False):
            assert gdk.BATgroupsum(gv, gg, None, gdk.TYPE_hge, skip).values() == \
                ora.BATgroupsum(ov, og, None, ora.TYPE_hge, skip).values()
            assert np.array_equal(gdk.BATgroupcount(gv, gg, None, skip).to_numpy(),
                                  ora.BATgroupcount(ov, og, None, skip).values())
            a, rr, c = gdk.BATgroupavg3(gv, gg, None, skip)
            oa, orr, oc = ora.BATgroupavg3(ov, og, None, skip)
            assert np.array_equal(a.to_numpy(), oa.values())
            assert np.array_equal(rr.to_numpy(), orr.values())
            assert np.array_equal(c.to_numpy(), oc.values())
            for domax in (False, True):
                f = gdk.BATgroupmax if domax else gdk.BATgroupmin
                assert np.array_equal(f(gv, gg, None, skip).to_numpy(),
                                      ora.BATgroupminmax(ov, og, None, domax, skip).values())


def test_groupsum_nil_rules(gdk, ora):
    L = gdk.NIL[gdk.TYPE_lng]
    vals = np.array([L, 1, 2, 3, L, 4], np.int64)
    gid = np.array([0, 0, 1, 1, 1, 0], np.uint64)
    got = gdk.BATgroupsum(mk(gdk, gdk.TYPE_lng, vals), mk(gdk, gdk.TYPE_oid, gid), None,
                          gdk.TYPE_lng, False).values()
    assert list(got) == [5, L]


# ---- TPC-H lineitem generation and pipelines ------------------------------------

def test_tpch_generator_matches_oracle(gdk, ora):
    n, row0 = 300_001, 12345
    cols = gdk.tpch_lineitem(42, row0, n, 20_000)
    want = ora.tpch_lineitem(42, row0, n, 20_000)
    for k in gdk.LINEITEM_COLS:
        assert np.array_equal(cols[k].to_numpy(), want[k]), k


@pytest.mark.parametrize("n", [1, 5, 1_000_003])
def test_q6_parity(gdk, ora, n):
    cols = gdk.tpch_lineitem(9, 0, n, 20_000)
    want = ora.q6(ora.tpch_lineitem(9, 0, n, 20_000), 4)
    d0, d1 = ora.mkdate(1994, 1, 1), ora.mkdate(1995, 1, 1)
    got = gdk.q6_fused(cols["shipdate"], cols["discount"], cols["quantity"],
                       cols["extendedprice"], d0, d1, 5, 7, 2400)
    assert got == want
    got = gdk.q6_opatatime(cols["shipdate"], cols["discount"], cols["quantity"],
                           cols["extendedprice"], d0, d1, 5, 7, 2400)
    assert got == want


def _q1_rows(rows):
    out = []
    for r in rows:
        out.append((r["returnflag"], r["linestatus"], r["sum_qty"], r["sum_base_price"],
                    r["sum_disc_price"], r["sum_charge"], r["count_order"],
                    r["avg_qty"], r["rem_qty"], r["avg_price"], r["rem_price"], r["avg_disc"], r["rem_disc"]))
    return sorted(out)


@pytest.mark.parametrize("n", [7, 2_000_003])
def test_q1_parity(gdk, ora, n):
    cols = gdk.tpch_lineitem(5, 0, n, 20_000)
    want = ora.q1(ora.tpch_lineitem(5, 0, n, 20_000), 4)
    got = gdk.q1_fused(cols, ora.mkdate(1998, 9, 2))
    assert _q1_rows(got) == _q1_rows(want)
    # first-occurrence group numbering (BATgroup) and first rows agree with
    # the op-at-a-time device plan
    op = gdk.q1_fused(cols, ora.mkdate(1998, 9, 2), fused=False)
    # the plan ends with ORDER BY l_returnflag, l_linestatus (algebra.sort +
    # subsort); the group first rows are BATgroup's
    assert [(r["returnflag"], r["linestatus"], r["first_row"]) for r in op] == \
        sorted((r["returnflag"], r["linestatus"], r["first_row"]) for r in got)
    assert _q1_rows(op) == _q1_rows(want)


@pytest.mark.parametrize("case", ["none", "tax_wide", "disc_neg_wide", "price_beyond_wide", "qty_nil",
                                  "price_lane_bound"])
def test_q1_value_ranges(gdk, ora, case):
    """The fused Q1 takes a 64-bit pass when every value is within narrow
    bounds, reruns with 128-bit accumulation otherwise, and falls back to
    the op-at-a-time plan beyond 2^31 or on nils; all must agree with the
    oracle."""
    # price_lane_bound: on ONE workgroup (tuning hook) a lane sees ~78k rows,
    # so the narrow price bound 2^45 / rows-per-lane drops to ~4.5e8
    n = 20_000_003 if case == "price_lane_bound" else 300_007
    cols = gdk.tpch_lineitem(11, 0, n, 20_000)
    host = ora.tpch_lineitem(11, 0, n, 20_000)
    if case == "tax_wide":
        host["tax"][::101] = 5000
    elif case == "disc_neg_wide":
        host["discount"][3::211] = -70000
    elif case == "price_beyond_wide":
        host["extendedprice"][::997] = (1 << 32) + 12345
    elif case == "price_lane_bound":
        host["extendedprice"][::99991] = 600_000_000
    elif case == "qty_nil":
        host["quantity"][5::1009] = np.iinfo(np.int64).min
    for k in ("tax", "discount", "extendedprice", "quantity"):
        cols[k] = gdk.BAT.from_numpy(gdk.TYPE_lng, host[k])
    import ctypes
    tune = gdk.lib().mgdk_q1_set_variant
    tune.argtypes = [ctypes.c_int, ctypes.c_int]
    if case == "price_lane_bound":
        tune(1, 1)
    gdk.prof_reset()
    gdk.prof_enable(True)
    try:
        got = gdk.q1_fused(cols, ora.mkdate(1998, 9, 2))
    finally:
        gdk.prof_enable(False)
        tune(1, 0)
    wide = gdk.prof_get("q1_wide")[1]
    opat = gdk.prof_get("q1_opatatime")[1]
    assert (wide, opat) == {"none": (0, 0), "tax_wide": (1, 0), "disc_neg_wide": (1, 0), "price_lane_bound": (1, 0),
                            "price_beyond_wide": (1, 1), "qty_nil": (1, 1)}[case]
    if case == "qty_nil":
        # nil quantities: sums and averages skip them (the oracle's Q1 counts
        # the non-nil values per group for aggr.subavg), count(*) does not
        op = gdk.q1_fused(cols, ora.mkdate(1998, 9, 2), fused=False)
        assert _q1_rows(got) == _q1_rows(op)
    want = ora.q1(host, 4)
    assert _q1_rows(got) == _q1_rows(want)


@pytest.mark.parametrize("n", [255, 256, 70_001, 2_000_129])
def test_q6_variants(gdk, ora, n):
    """Every fused-Q6 launch variant (full read k_q6 / k_q6c, predicate
    cascade k_q6s) gives the oracle's revenue, with nils in every column; the
    cascade reads fewer column lines than the full read."""
    r = rng(61)
    host = ora.tpch_lineitem(17, 0, n, 20_000)
    for k, nilv in (("shipdate", np.iinfo(np.int32).min), ("discount", np.iinfo(np.int64).min),
                    ("quantity", np.iinfo(np.int64).min), ("extendedprice", np.iinfo(np.int64).min)):
        host[k][r.random(n) < 0.01] = nilv
    cols = {k: gdk.BAT.from_numpy(gdk.TYPE_int if k == "shipdate" else gdk.TYPE_lng, host[k])
            for k in ("shipdate", "discount", "quantity", "extendedprice")}
    d0, d1 = ora.mkdate(1994, 1, 1), ora.mkdate(1995, 1, 1)
    want = ora.q6(host, 4)
    try:
        for v, b in ((14, 12), (5, 8), (2, 8), (16, 16), (17, 16), (18, 8), (19, 16), (20, 8)):
            gdk.q6_set_variant(v, b)
            got = gdk.q6_fused(cols["shipdate"], cols["discount"], cols["quantity"],
                               cols["extendedprice"], d0, d1, 5, 7, 2400)
            assert got == want, (v, b)
            lines = gdk.q6_last_lines()
            if v >= 16 and n >= 70_000:
                assert 0 < lines * 128 < 3 * 8 * n, lines
            elif v < 16:
                assert lines == 0
    finally:
        gdk.q6_set_variant(19, 16)


@pytest.mark.parametrize("case", ["none", "price_huge", "price_neg_nil"])
def test_q6_value_ranges(gdk, ora, case):
    """Q6 accumulates revenue in 128 bits: prices near 2^60 (products beyond
    64 bits), negative prices and nil prices agree with the oracle."""
    n = 400_009
    cols = gdk.tpch_lineitem(13, 0, n, 20_000)
    host = ora.tpch_lineitem(13, 0, n, 20_000)
    if case == "price_huge":
        host["extendedprice"][::61] = (1 << 60) + 7
        host["extendedprice"][1::67] = -(1 << 60) - 3
    elif case == "price_neg_nil":
        host["extendedprice"][::13] *= -1
        host["extendedprice"][5::29] = np.iinfo(np.int64).min
    cols["extendedprice"] = gdk.BAT.from_numpy(gdk.TYPE_lng, host["extendedprice"])
    d0, d1 = ora.mkdate(1994, 1, 1), ora.mkdate(1995, 1, 1)
    got = gdk.q6_fused(cols["shipdate"], cols["discount"], cols["quantity"],
                       cols["extendedprice"], d0, d1, 5, 7, 2400)
    assert got == ora.q6(host, 4)


@pytest.mark.parametrize("tname", ["dbl", "flt"])
def test_fsum_exact(gdk, ora, tname):
    """BATsum of flt / dbl (dofsum, gdk_aggr.c:183): bit-exact with the
    oracle's msum restatement on wide ranges, cancellation, nils,
    candidates, subnormal and intermediate-overflow cases."""
    r = rng(92)
    tp = getattr(gdk, "TYPE_" + tname)
    dt = np.float64 if tname == "dbl" else np.float32
    cases = []
    for scale in ((1, 5, 20, 60) if tname == "dbl" else (1, 5, 20, 30)):
        v = (r.standard_normal(300_000) * 10.0 ** r.integers(-scale, scale, 300_000)).astype(dt)
        cases.append(v)
    v = r.standard_normal(200_000).astype(dt)
    cases.append(np.concatenate([v, -v[::-1], np.array([1e-3], dt)]))      # cancels to 1e-3
    cases.append(np.array([2.0 ** -1070, 2.0 ** -1074, -(2.0 ** -1073)], np.float64).astype(dt))
    cases.append(np.array([0.0, -0.0], dt))
    if tname == "dbl":
        cases.append(np.array([1e308, 1e308, -1e308, 1.0], np.float64))    # finite despite overflow
        cases.append(np.array([1e16, 1.0, -1e16] * 1000, np.float64))
    for v in cases:
        B, OB = gdk.BAT.from_numpy(tp, v), ora.Bat.from_array(tp, v)
        for rt in ((gdk.TYPE_dbl,) if tname == "dbl" else (gdk.TYPE_dbl, gdk.TYPE_flt)):
            try:
                want = ora.BATsum(rt, OB)
            except ora.OracleError as e:
                with pytest.raises(gdk.GDKError) as ei:
                    gdk.BATsum(rt, B)
                assert str(ei.value) == str(e)
                continue
            got = gdk.BATsum(rt, B)
            assert np.array(got, np.float64).tobytes() == np.array(want, np.float64).tobytes(), (v[:4], rt)
    # nils, empty, candidates
    v = r.standard_normal(100_000).astype(dt)
    v[::37] = np.nan
    s = np.sort(r.choice(100_000, 50_000, replace=False)).astype(np.uint64)
    B, OB = gdk.BAT.from_numpy(tp, v), ora.Bat.from_array(tp, v)
    S, OS = gdk.BAT.from_numpy(gdk.TYPE_oid, s), ora.Bat.from_array(ora.TYPE_oid, s)
    assert gdk.BATsum(gdk.TYPE_dbl, B, S) == ora.BATsum(ora.TYPE_dbl, OB, OS)
    assert np.isnan(gdk.BATsum(gdk.TYPE_dbl, B, skip_nils=False))
    E = gdk.BAT.from_numpy(tp, np.array([np.nan, np.nan], dt))
    assert np.isnan(gdk.BATsum(gdk.TYPE_dbl, E)) and gdk.BATsum(gdk.TYPE_dbl, E, nil_if_empty=False) == 0.0


def test_fsum_overflow(gdk):
    with pytest.raises(gdk.GDKError, match="22003!overflow in sum aggregate"):
        gdk.BATsum(gdk.TYPE_dbl, gdk.BAT.from_numpy(gdk.TYPE_dbl, np.array([1e308, 1e308])))
    with pytest.raises(gdk.GDKError, match="22003!overflow in sum aggregate"):
        gdk.BATsum(gdk.TYPE_flt, gdk.BAT.from_numpy(gdk.TYPE_flt, np.array([3e38, 3e38], np.float32)))


@pytest.mark.parametrize("ng", [1, 4, 300, 20_000])
def test_fgroupsum_exact(gdk, ora, ng):
    """BATgroupsum of dbl / flt (dofsum with gids): bit-exact per group with
    the oracle's msum restatement; nils, empty groups, candidates."""
    r = rng(93)
    n = 200_000
    v = r.standard_normal(n) * 10.0 ** r.integers(-8, 8, n)
    v[r.random(n) < 0.01] = np.nan
    gid = r.integers(0, ng, n).astype(np.uint64)
    if ng > 1:
        gid[gid == ng - 1] = 0                      # one empty group
    for tname, rt in (("dbl", "dbl"), ("flt", "flt"), ("flt", "dbl")):
        tp, tr = getattr(gdk, "TYPE_" + tname), getattr(gdk, "TYPE_" + rt)
        vv = v.astype(np.float64 if tname == "dbl" else np.float32)
        B, OB = gdk.BAT.from_numpy(tp, vv), ora.Bat.from_array(tp, vv)
        G, OG = gdk.BAT.from_numpy(gdk.TYPE_oid, gid), ora.Bat.from_array(ora.TYPE_oid, gid)
        for skip in (True, False):
            got = np.asarray(gdk.BATgroupsum(B, G, None, tr, skip).values())
            want = np.asarray(ora.BATgroupsum(OB, OG, None, tr, skip).values())
            assert got.tobytes() == want.tobytes(), (tname, rt, skip)
        # with a dense candidate slice: g aligned with the candidates
        # (BATgroupaggrinit, gdk_aggr.c:65-146)
        m = n // 2
        S, OS = gdk.BAT.dense(1000, m), ora.Bat.dense(1000, m)
        Gs = gdk.BAT.from_numpy(gdk.TYPE_oid, gid[:m], hseqbase=1000)
        OGs = ora.Bat.from_array(ora.TYPE_oid, gid[:m], hseqbase=1000)
        got = np.asarray(gdk.BATgroupsum(B, Gs, None, tr, True, s=S).values())
        want = np.asarray(ora.BATgroupsum(OB, OGs, None, tr, True, s=OS).values())
        assert got.tobytes() == want.tobytes()


def _hge_pairs(v):
    """int64 values (INT64_MIN = nil) as hge (lo, hi) uint64 pairs"""
    lo = v.astype(np.uint64)
    hi = np.where(v < 0, np.uint64(2**64 - 1), np.uint64(0)).astype(np.uint64)
    nil = v == -(2**63)
    lo[nil], hi[nil] = 0, np.uint64(1 << 63)
    return np.stack([lo, hi], 1).reshape(-1)


@pytest.mark.parametrize("tname", ["bte", "sht", "int", "lng", "hge", "flt", "dbl"])
def test_groupavg(gdk, ora, tname):
    """BATgroupavg (gdk_aggr.c:1801): integer averages from the exact floor
    average + remainder, flt/dbl from the order-dependent AVERAGE_ITER_FLOAT
    replay; bit-exact dbl results and counts against the oracle."""
    r = rng(57)
    n = 120_000
    tp = getattr(gdk, "TYPE_" + tname)
    if tname in ("flt", "dbl"):
        v = r.standard_normal(n) * 10.0 ** r.integers(-3, 6, n)
        v[r.random(n) < 0.002] = np.nan
        v = v.astype(np.float32 if tname == "flt" else np.float64)
        data = v
    else:
        bits = {"bte": 8, "sht": 16, "int": 32, "lng": 64, "hge": 64}[tname]
        v = r.integers(-(2**(bits - 1)) + 1, 2**(bits - 1), n, dtype=np.int64)
        v[r.random(n) < 0.002] = -(2**(bits - 1)) if bits < 64 else -(2**63)
        data = _hge_pairs(v) if tname == "hge" else v.astype(gdk.NP[tp])
    B = gdk.BAT.from_numpy(tp, data, nonil=False)
    OB = ora.Bat.from_array(tp, data, nonil=False)
    for ng in (1, 5, 700, 5000):
        gid = r.integers(0, ng, n).astype(np.uint64)
        if ng > 2:
            gid[gid == 2] = 1                       # an empty group
        G, OG = gdk.BAT.from_numpy(gdk.TYPE_oid, gid, key=False), ora.Bat.from_array(ora.TYPE_oid, gid)
        for skip in (True, False):
            for scale in (0, 2):
                a, c = gdk.BATgroupavg(B, G, None, skip, scale=scale)
                oa, oc = ora.BATgroupavg(OB, OG, None, skip, scale=scale)
                assert np.asarray(a.values()).tobytes() == np.asarray(oa.values()).tobytes(), \
                    (ng, skip, scale)
                assert np.array_equal(c.to_numpy(), oc.values())
    # dense candidate slice, g aligned with it
    m = n // 3
    S, OS = gdk.BAT.dense(500, m), ora.Bat.dense(500, m)
    gid = r.integers(0, 9, m).astype(np.uint64)
    G = gdk.BAT.from_numpy(gdk.TYPE_oid, gid, hseqbase=500, key=False)
    OG = ora.Bat.from_array(ora.TYPE_oid, gid, hseqbase=500)
    a, c = gdk.BATgroupavg(B, G, None, True, s=S)
    oa, oc = ora.BATgroupavg(OB, OG, None, True, s=OS)
    assert np.asarray(a.values()).tobytes() == np.asarray(oa.values()).tobytes()
    assert np.array_equal(c.to_numpy(), oc.values())


def test_groupavg_trivial_paths(gdk, ora):
    """Singleton groups (g key + nonil) return the values converted to dbl
    with counts 1 and no scale; no candidates -> nil averages, counts 0."""
    r = rng(58)
    n = 5000
    v = r.integers(-2**62, 2**62, n).astype(np.int64)
    v[::97] = gdk.NIL[gdk.TYPE_lng]
    perm = r.permutation(n).astype(np.uint64)
    B, OB = gdk.BAT.from_numpy(gdk.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_lng, v)
    G = gdk.BAT.from_numpy(gdk.TYPE_oid, perm, key=True, nonil=True)
    OG = ora.Bat.from_array(ora.TYPE_oid, perm, key=True, nonil=True)
    for skip, want_counts in ((False, True), (True, False)):
        a, c = gdk.BATgroupavg(B, G, None, skip, scale=3, want_counts=want_counts)
        oa, oc = ora.BATgroupavg(OB, OG, None, skip, scale=3, want_counts=want_counts)
        assert np.asarray(a.values()).tobytes() == np.asarray(oa.values()).tobytes()
        if want_counts:
            assert np.array_equal(c.to_numpy(), oc.values())
    f = r.standard_normal(n).astype(np.float32)
    a, _ = gdk.BATgroupavg(gdk.BAT.from_numpy(gdk.TYPE_flt, f), G, None, False)
    assert np.asarray(a.values()).tobytes() == f.astype(np.float64).tobytes()
    S, OS = gdk.BAT.dense(0, 0), ora.Bat.dense(0, 0)
    G0 = gdk.BAT.from_numpy(gdk.TYPE_oid, np.zeros(0, np.uint64))
    a, c = gdk.BATgroupavg(B, G0, None, True, s=S)
    assert a.count() == 0 and c.count() == 0


def test_complex_candidate_lists(gdk, ora):
    """cand_except / cand_mask candidate lists (gdk/gdk_cand.h:23-38,
    gdk_cand.c:455-560): a void BAT whose vheap holds the exceptions or the
    mask.  Every operator must see exactly the candidates the equivalent
    materialised list holds -- checked on select, thetaselect, calc, sum,
    groupsum and join against the oracle with the materialised list."""
    r = rng(61)
    n = 50_000
    v = r.integers(-1000, 1000, n).astype(np.int32)
    v[::53] = gdk.NIL[gdk.TYPE_int]
    B, OB = gdk.BAT.from_numpy(gdk.TYPE_int, v, hseqbase=100), ora.Bat.from_array(ora.TYPE_int, v, hseqbase=100)
    # except list over [150, 150 + 30000 + nexc) -- reaches past b's end
    exc = np.sort(r.choice(np.arange(150, 150 + 30_000), 700, replace=False)).astype(np.uint64)
    exc = np.unique(np.concatenate([exc, [150, 151]])).astype(np.uint64)   # pruned at the front
    NEG = gdk.BAT.negoid_cand(150, 30_000, exc)
    neg_oids = np.setdiff1d(np.arange(150, 150 + 30_000 + len(exc), dtype=np.uint64), exc)
    # mask over rows 20..60000 (partly before and after b)
    bits = r.random(60_000) < 0.3
    MSK = gdk.BAT.mask_cand(20, bits)
    msk_oids = (20 + np.flatnonzero(bits)).astype(np.uint64)
    for S, oids in ((NEG, neg_oids), (MSK, msk_oids)):
        OS = ora.Bat.from_array(ora.TYPE_oid, oids, sorted_=True, key=True, nonil=True)
        got = gdk.BATselect(B, S, -100, 300, True, False, False).to_numpy()
        want = np.asarray(ora.BATselect(OB, OS, -100, 300, True, False, False).values())
        assert np.array_equal(got, want)
        got = gdk.BATthetaselect(B, S, 0, ">=").to_numpy()
        want = np.asarray(ora.BATthetaselect(OB, OS, 0, ">=").values())
        assert np.array_equal(got, want)
        assert gdk.BATsum(gdk.TYPE_lng, B, s=S) == ora.BATsum(ora.TYPE_lng, OB, s=OS)
        c = gdk.BATcalcaddcst(B, 7, gdk.TYPE_int, gdk.TYPE_lng, s=S).to_numpy()
        lo = np.clip(oids, 100, 100 + n).astype(np.int64)
        keep = oids[(oids >= 100) & (oids < 100 + n)].astype(np.int64) - 100
        want = np.where(v[keep] == gdk.NIL[gdk.TYPE_int], gdk.NIL[gdk.TYPE_lng], v[keep].astype(np.int64) + 7)
        assert np.array_equal(c, want), lo.size
        # join with a complex left candidate list
        rk = r.permutation(2000).astype(np.int32) - 1000
        R = gdk.BAT.from_numpy(gdk.TYPE_int, rk)
        OR = ora.Bat.from_array(ora.TYPE_int, rk, key=True, nonil=True)
        r1, r2 = gdk.BATjoin(B, R, sl=S)
        o1, o2 = ora.BATjoin(OB, OR, sl=OS)
        assert np.array_equal(r1.to_numpy(), np.asarray(o1.values()))
        assert np.array_equal(r2.to_numpy(), np.asarray(o2.values()))


def _same(got, want):
    g, w = got.values(), want.values()
    if isinstance(g, list) or isinstance(w, list):
        return list(g) == list(w)
    return np.asarray(g).tobytes() == np.asarray(w).tobytes()


@pytest.mark.parametrize("tname", ["int", "lng", "hge", "dbl", "oid"])
def test_projectchain_and_project2(gdk, ora, tname):
    """BATprojectchain (gdk_project.c:879) = the sequence of BATproject calls
    it stands for (its own definition), fused on the device; BATproject2
    (gdk_project.c:590) = BATproject over r1 ++ r2.  Checked against the
    oracle's BATproject; nil oids, dense steps, complex candidate lists and
    the "does not match always" error included."""
    r = rng(71)
    tp = getattr(gdk, "TYPE_" + tname)
    n3 = 40_000
    if tname == "hge":
        vals = r.integers(-2**62, 2**62, 2 * n3).astype(np.uint64)
    elif tname == "dbl":
        vals = r.standard_normal(n3)
    elif tname == "oid":
        vals = r.integers(0, 2**40, n3).astype(np.uint64)
    else:
        vals = r.integers(-10**6, 10**6, n3).astype(gdk.NP[tp])
    V = gdk.BAT.from_numpy(tp, vals, hseqbase=1000)
    OV = ora.Bat.from_array(tp, vals, hseqbase=1000)
    # chain: a (oid into b's heads) . b (oid into V's heads) . V
    b = (1000 + r.integers(0, n3, 30_000)).astype(np.uint64)
    b[::97] = gdk.OID_NIL
    a = r.integers(0, 30_000, 25_000).astype(np.uint64) + 50
    A, B = gdk.BAT.from_numpy(gdk.TYPE_oid, a), gdk.BAT.from_numpy(gdk.TYPE_oid, b, hseqbase=50)
    OA, OBb = ora.Bat.from_array(ora.TYPE_oid, a), ora.Bat.from_array(ora.TYPE_oid, b, hseqbase=50)
    got = gdk.BATprojectchain([A, B, V])
    want = ora.BATproject(ora.BATproject(OA, OBb), OV)
    assert _same(got, want)
    assert got.s.tnil
    # an identity (dense) step is skipped; a dense first step
    D = gdk.BAT.dense(50, 30_000, hseqbase=50)
    got2 = gdk.BATprojectchain([A, D, B, V])
    assert _same(got2, want)
    C0 = gdk.BAT.dense(60, 1000)
    got3 = gdk.BATprojectchain([C0, B, V])
    want3 = ora.BATproject(ora.BATproject(ora.Bat.from_array(ora.TYPE_oid, np.arange(60, 1060, dtype=np.uint64)),
                                          OBb), OV)
    assert _same(got3, want3)
    # complex candidate list as the first step
    M = gdk.BAT.negoid_cand(60, 900, np.array([70, 500, 999], np.uint64))
    keep = np.setdiff1d(np.arange(60, 963, dtype=np.uint64), [70, 500, 999])
    got4 = gdk.BATprojectchain([M, B, V])
    want4 = ora.BATproject(ora.BATproject(ora.Bat.from_array(ora.TYPE_oid, keep), OBb), OV)
    assert _same(got4, want4)
    bad = a.copy()
    bad[7] = 10**9
    with pytest.raises(gdk.GDKError, match="does not match always"):
        gdk.BATprojectchain([gdk.BAT.from_numpy(gdk.TYPE_oid, bad), B, V])
    # BATproject2: r1 = V[:m], r2 = V[m:]
    m = n3 // 3
    if tname == "hge":
        v1, v2 = vals[:2 * m], vals[2 * m:]
    else:
        v1, v2 = vals[:m], vals[m:]
    R1 = gdk.BAT.from_numpy(tp, v1, hseqbase=1000)
    R2 = gdk.BAT.from_numpy(tp, v2, hseqbase=1000 + m)
    got5 = gdk.BATproject2(B, R1, R2)
    want5 = ora.BATproject(OBb, OV)
    assert _same(got5, want5)
    # dense l across the r1 / r2 boundary, and inside r2 (slice)
    for lo, cnt in ((1000 + m - 5, 10), (1000 + m + 3, 100)):
        L = gdk.BAT.dense(lo, cnt)
        got6 = gdk.BATproject2(L, R1, R2)
        want6 = ora.BATproject(ora.Bat.from_array(ora.TYPE_oid, np.arange(lo, lo + cnt, dtype=np.uint64)), OV)
        assert _same(got6, want6)


@pytest.mark.parametrize("tname", ["bte", "sht", "int", "lng", "hge"])
@pytest.mark.parametrize("skip", [True, False])
def test_groupavg3combine(gdk, ora, tname, skip):
    """BATgroupavg3combine (gdk_aggr.c:2634) bit-exact against the oracle's
    row-by-row combine_averages replay: partials from BATgroupavg3 over
    shards (negative remainders after rounding, empty and nil groups)."""
    r = rng(81)
    tp = getattr(gdk, "TYPE_" + tname)
    bits = {"bte": 8, "sht": 16, "int": 32, "lng": 40, "hge": 40}[tname]
    n, ng = 30_000, 700
    v = r.integers(-(2**(bits - 1)) + 1, 2**(bits - 1), n, dtype=np.int64)
    nilv = -(2**(bits - 1)) if tname in ("bte", "sht", "int") else -(2**63)
    v[r.random(n) < 0.01] = nilv
    gid = r.integers(0, ng, n).astype(np.uint64)
    gid[gid == 5] = 6
    dt = gdk.NP.get(tp, np.int64)
    parts = []
    for sh in np.array_split(np.arange(n), 5):
        vv = v[sh]
        data = _hge_pairs(vv) if tname == "hge" else vv.astype(dt)
        a, rm, c = gdk.BATgroupavg3(gdk.BAT.from_numpy(tp, data, nonil=False),
                                    gdk.BAT.from_numpy(gdk.TYPE_oid, gid[sh], key=False), None, skip)
        parts.append((a.to_numpy(), rm.to_numpy(), c.to_numpy(), a.count()))
    A = np.concatenate([p[0] for p in parts])
    R = np.concatenate([p[1] for p in parts])
    K = np.concatenate([p[2] for p in parts])
    G = np.concatenate([np.arange(p[3], dtype=np.uint64) for p in parts])
    Ad = A.reshape(-1) if tname == "hge" else A
    got = gdk.BATgroupavg3combine(gdk.BAT.from_numpy(tp, Ad, nonil=False), gdk.BAT.from_numpy(gdk.TYPE_lng, R),
                                  gdk.BAT.from_numpy(gdk.TYPE_lng, K), gdk.BAT.from_numpy(gdk.TYPE_oid, G, key=False),
                                  None, skip)
    want = ora.BATgroupavg3combine(ora.Bat.from_array(tp, Ad), ora.Bat.from_array(ora.TYPE_lng, R),
                                   ora.Bat.from_array(ora.TYPE_lng, K), ora.Bat.from_array(ora.TYPE_oid, G),
                                   None, skip)
    assert _same(got, want)


def test_grouped_aggregates_candidate_lists(gdk, ora):
    """BATgroupsum / count / min / max / avg3 / avg with a materialised (and a
    cand_except) candidate list: g has one group id per candidate and its
    head starts at the first candidate (BATgroupaggrinit, gdk_aggr.c:65)."""
    r = rng(91)
    n = 60_000
    v = r.integers(-10**9, 10**9, n).astype(np.int64)
    v[::41] = gdk.NIL[gdk.TYPE_lng]
    B, OB = gdk.BAT.from_numpy(gdk.TYPE_lng, v, hseqbase=10), ora.Bat.from_array(ora.TYPE_lng, v, hseqbase=10)
    oids = np.sort(r.choice(np.arange(10, 10 + n), 25_000, replace=False)).astype(np.uint64)
    S = gdk.BAT.from_numpy(gdk.TYPE_oid, oids, sorted_=True, key=True, nonil=True)
    OS = ora.Bat.from_array(ora.TYPE_oid, oids, sorted_=True, key=True, nonil=True)
    gid = r.integers(0, 300, len(oids)).astype(np.uint64)
    G = gdk.BAT.from_numpy(gdk.TYPE_oid, gid, hseqbase=int(oids[0]), key=False)
    OG = ora.Bat.from_array(ora.TYPE_oid, gid, hseqbase=int(oids[0]))
    for skip in (True, False):
        assert _same(gdk.BATgroupsum(B, G, None, gdk.TYPE_hge, skip, s=S),
                     ora.BATgroupsum(OB, OG, None, ora.TYPE_hge, skip, s=OS))
        assert np.array_equal(gdk.BATgroupcount(B, G, None, skip, s=S).to_numpy(),
                              np.asarray(ora.BATgroupcount(OB, OG, None, skip, s=OS).values()))
        a, rm, c = gdk.BATgroupavg3(B, G, None, skip, s=S)
        oa, orm, oc = ora.BATgroupavg3(OB, OG, None, skip, s=OS)
        assert _same(a, oa) and _same(rm, orm) and _same(c, oc)
        av, cn = gdk.BATgroupavg(B, G, None, skip, s=S)
        oav, ocn = ora.BATgroupavg(OB, OG, None, skip, s=OS)
        assert _same(av, oav) and _same(cn, ocn)
    assert _same(gdk.BATgroupmin(B, G, None, s=S), ora.BATgroupminmax(OB, OG, None, False, s=OS))
    assert _same(gdk.BATgroupmax(B, G, None, s=S), ora.BATgroupminmax(OB, OG, None, True, s=OS))
    # cand_except list over the same BAT
    exc = np.sort(r.choice(np.arange(100, 30_000), 500, replace=False)).astype(np.uint64)
    NEG = gdk.BAT.negoid_cand(100, 29_900 - 500, exc)
    keep = np.setdiff1d(np.arange(100, 30_000, dtype=np.uint64), exc)
    gid2 = r.integers(0, 50, len(keep)).astype(np.uint64)
    G2 = gdk.BAT.from_numpy(gdk.TYPE_oid, gid2, hseqbase=int(keep[0]), key=False)
    OG2 = ora.Bat.from_array(ora.TYPE_oid, gid2, hseqbase=int(keep[0]))
    OK = ora.Bat.from_array(ora.TYPE_oid, keep, sorted_=True, key=True, nonil=True)
    assert _same(gdk.BATgroupsum(B, G2, None, gdk.TYPE_hge, True, s=NEG),
                 ora.BATgroupsum(OB, OG2, None, ora.TYPE_hge, True, s=OK))


@pytest.mark.parametrize("sel_t", ["int", "lng", "bte"])
@pytest.mark.parametrize("sel", [0.98, 0.5, 0.02])
def test_project_through_select_bitmap(gdk, sel_t, sel):
    """A select result of >= 1M oids keeps its scan bitmap (Priv::smap) and
    BATproject through it streams the projected column: same values as the
    oid gather, for every value width (1, 2, 4, 8, 16 B and str offsets),
    unaligned scan starts (a sliced column), candidate oids offset by the
    head base, and an r that does not cover the list (the error)."""
    r = rng(91)
    n = 3_000_017
    dt = {"int": np.int32, "lng": np.int64, "bte": np.int8}[sel_t]
    tp = getattr(gdk, "TYPE_" + sel_t)
    lim = {"bte": 100, "int": 1_000_000, "lng": 1_000_000}[sel_t]
    col = r.integers(0, lim, n).astype(dt)
    thr = int(lim * sel)
    B = gdk.BAT.from_numpy(tp, col, hseqbase=77)
    for lo in (0, 3):                       # 3: a view whose data is not 16-B aligned
        S = gdk.BATslice(B, lo, n) if lo else B
        c = gdk.BATthetaselect(S, None, thr, "<")
        want_idx = np.flatnonzero(col[lo:] < thr) + lo
        assert np.array_equal(c.to_numpy().astype(np.int64), want_idx + 77)
        for vt, vals in ((gdk.TYPE_lng, r.integers(-2**62, 2**62, n)),
                         (gdk.TYPE_int, r.integers(-2**30, 2**30, n).astype(np.int32)),
                         (gdk.TYPE_sht, r.integers(-2**14, 2**14, n).astype(np.int16)),
                         (gdk.TYPE_bte, r.integers(-100, 100, n).astype(np.int8)),
                         (gdk.TYPE_dbl, r.standard_normal(n)),
                         (gdk.TYPE_hge, r.integers(0, 2**63, 2 * n).astype(np.uint64))):
            V = gdk.BAT.from_numpy(vt, vals, hseqbase=77)
            got = gdk.BATproject(c, V).to_numpy()
            want = vals.reshape(n, 2)[want_idx] if vt == gdk.TYPE_hge else vals[want_idx]
            assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8)), vt
        # r longer than the scanned range (its last rows are no candidate
        # slot; the 16-byte vector path must not take them for tail hits)
        for vt, dtv in ((gdk.TYPE_lng, np.int64), (gdk.TYPE_bte, np.int8)):
            vals = r.integers(-100, 100, n + 29).astype(dtv)
            got = gdk.BATproject(c, gdk.BAT.from_numpy(vt, vals, hseqbase=77)).to_numpy()
            assert np.array_equal(got, vals[want_idx]), vt
    # r shorter than the list's range: "does not match always" as with the gather
    c = gdk.BATthetaselect(B, None, thr, "<")
    short = gdk.BAT.from_numpy(gdk.TYPE_lng, np.arange(n - 5, dtype=np.int64), hseqbase=77)
    if want_idx[-1] >= n - 5:
        with pytest.raises(gdk.GDKError, match="does not match always"):
            gdk.BATproject(c, short)
