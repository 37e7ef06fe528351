"""The oracle (oracle/liboracle.so, CPU restatement) against the reference's own
known-answer fixtures (tests/golden/maltest_fixtures.json, extracted from
monetdb5/modules/kernel/Tests/select.maltest, monetdb5/mal/Tests/tst1500.maltest,
tst1503.maltest and monetdb5/modules/mal/Tests/bigsum.maltest)."""
import math

import numpy as np
import pytest

from helpers import FIX, replay_project, replay_select


def test_select_maltest(ora):
    def mk(tp, vals):
        return ora.Bat.from_array(tp, vals)
    bad = replay_select(ora, mk, ora.TYPE_int, ora.NIL[ora.TYPE_int])
    assert not bad, bad[:3]
    assert len(FIX["select"]["cases"]) == 192


@pytest.mark.parametrize("name", ["group_tst1500", "group_tst1503"])
def test_group_maltest(ora, name):
    fx = FIX[name]
    b = ora.Bat.from_array(ora.TYPE_bte, fx["values"])
    g, e, h = ora.BATgroup(b)
    assert list(g.values()) == fx["expected"]["g1"]
    assert list(e.values()) == fx["expected"]["e1"]
    assert list(h.values()) == fx["expected"]["h1"]


def test_bigsum_maltest(ora):
    fx = FIX["bigsum"]
    vals = np.full(fx["repeat_count"] + 1, fx["repeat_value"], np.int64)
    vals[0] = fx["first"]
    b = ora.Bat.from_array(ora.TYPE_lng, vals)
    s = ora.BATsum(ora.TYPE_dbl, b)
    assert "%.10g" % s == fx["expected"]


def test_thetaselect_ops(ora):
    vals = np.array([5, 1, -3, ora.NIL[ora.TYPE_int], 5, 9], np.int32)
    b = ora.Bat.from_array(ora.TYPE_int, vals)
    exp = {"<": [1, 2], "<=": [0, 1, 2, 4], ">": [5], ">=": [0, 4, 5], "=": [0, 4],
           "==": [0, 4], "!=": [1, 2, 5], "<>": [1, 2, 5], "ne": [1, 2, 3, 5], "eq": [0, 4]}
    for op, want in exp.items():
        assert list(ora.BATthetaselect(b, None, 5, op).values()) == want, op
    # nil value: empty except eq/ne
    assert ora.BATthetaselect(b, None, ora.NIL[ora.TYPE_int], "<").count() == 0
    assert list(ora.BATthetaselect(b, None, ora.NIL[ora.TYPE_int], "eq").values()) == [3]
    with pytest.raises(ora.OracleError, match="unknown operator"):
        ora.BATthetaselect(b, None, 5, "~")


def test_calc_overflow_message(ora):
    b = ora.Bat.from_array(ora.TYPE_int, np.array([1, 2**30, 3], np.int32))
    with pytest.raises(ora.OracleError, match=r"22003!overflow in calculation 1073741824\*4\."):
        ora.BATcalc("*", b, None, ora.TYPE_int, c2=4, t2=ora.TYPE_int)
    r = ora.BATcalc("*", b, None, ora.TYPE_lng, c2=4, t2=ora.TYPE_int)
    assert list(r.values()) == [4, 2**32, 12]


def test_groupsum_nil_rules(ora):
    # two groups: a nil before the group's first value is forgotten
    # (gdk_aggr.c:497-527), a nil after it makes the sum nil
    L = ora.NIL[ora.TYPE_lng]
    b = ora.Bat.from_array(ora.TYPE_lng, np.array([L, 1, 2, 3, L, 4], np.int64))
    g = ora.Bat.from_array(ora.TYPE_oid, np.array([0, 0, 1, 1, 1, 0], np.uint64))
    s = ora.BATgroupsum(b, g, None, ora.TYPE_lng, skip_nils=False)
    assert list(s.values()) == [5, L]
    s = ora.BATgroupsum(b, g, None, ora.TYPE_lng, skip_nils=True)
    assert list(s.values()) == [5, 5]


def test_avg3_rounding(ora):
    b = ora.Bat.from_array(ora.TYPE_lng, np.array([1, 2, -1, -2, 7, 8, 8], np.int64))
    g = ora.Bat.from_array(ora.TYPE_oid, np.array([0, 0, 1, 1, 2, 2, 2], np.uint64))
    a, r, c = ora.BATgroupavg3(b, g, None)
    # 3/2 = 1.5 -> 2 (rem -1); -3/2 = -1.5 -> -2 (floor -2 rem 1, 2*1 > 2 false);
    # 23/3 = 7.67 -> 8 (rem -1)
    assert list(a.values()) == [2, -2, 8]
    assert list(r.values()) == [-1, 1, -1]
    assert list(c.values()) == [2, 2, 3]


def test_q6_threads_agree(ora):
    cols = ora.tpch_lineitem(7, 0, 200_000, 2000)
    r1 = ora.q6(cols, 1)
    r4 = ora.q6(cols, 4)
    assert r1 == r4 and r1 > 0


def test_q1_threads_agree(ora):
    cols = ora.tpch_lineitem(7, 0, 200_000, 2000)
    a = ora.q1(cols, 1)
    b = ora.q1(cols, 3)
    assert a == b and len(a) == 4
    assert sum(r["count_order"] for r in a) <= 200_000


def _avg3(s, n):
    """BATgroupavg3's average / remainder of an exact sum (floor, then half
    away from zero; gdk_aggr.c:2070-2095)"""
    q, r = divmod(s, n)
    if r > 0:
        if q < 0:
            if 2 * r > n:
                q, r = q + 1, r - n
        elif 2 * r >= n:
            q, r = q + 1, r - n
    return q, r


def test_q1_nils_numpy(ora):
    """The oracle's Q1 with nil quantities / prices / discounts: sums skip
    nils, the three averages divide by each column's non-nil count, count(*)
    counts every row -- checked against Python integers."""
    n = 60_013
    cols = ora.tpch_lineitem(23, 0, n, 2000)
    nil = np.iinfo(np.int64).min
    cols["quantity"][3::97] = nil
    cols["extendedprice"][5::101] = nil
    cols["discount"][7::89] = nil
    got = {(r["returnflag"], r["linestatus"]): r for r in ora.q1(cols, 2)}
    sel = cols["shipdate"] <= ora.mkdate(1998, 9, 2)
    keys = set(zip(cols["returnflag"][sel].tolist(), cols["linestatus"][sel].tolist()))
    assert set(got) == keys
    for rf, ls in keys:
        m = sel & (cols["returnflag"] == rf) & (cols["linestatus"] == ls)
        r = got[(rf, ls)]
        assert r["count_order"] == int(m.sum())
        for col, sk, ak, rk in (("quantity", "sum_qty", "avg_qty", "rem_qty"),
                                ("extendedprice", "sum_base_price", "avg_price", "rem_price"),
                                ("discount", None, "avg_disc", "rem_disc")):
            v = [int(x) for x in cols[col][m] if x != nil]
            if sk:
                assert r[sk] == sum(v), sk
            assert (r[ak], r[rk]) == _avg3(sum(v), len(v)), ak


def test_rangebounds_small(ora):
    b = ora.Bat.from_array(ora.TYPE_lng, np.array([1, 2, 4, 8, 9, 1, 3], np.int64))
    p = ora.Bat.from_array(ora.TYPE_bit, np.array([1, 0, 0, 0, 0, 1, 0], np.int8))
    pre = ora.rangebounds(b, p, 2, True)
    fol = ora.rangebounds(b, p, 2, False)
    assert list(pre.values()) == [0, 0, 1, 3, 3, 5, 5]
    assert list(fol.values()) == [2, 3, 3, 5, 5, 7, 7]


def test_analytical_sum_oracle_small(ora):
    # hand-checked: partitions {0,1,2} {3..6}; peers {0,1} {2} {3} {4,5} {6}
    v = np.array([1, 2, 3, -(2**63), 5, 6, 7], np.int64)
    p = np.array([0, 0, 0, 1, 0, 0, 0], np.int8)
    o = np.array([1, 0, 1, 1, 1, 0, 1], np.int8)
    B, P, O = (ora.Bat.from_array(ora.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_bit, p),
               ora.Bat.from_array(ora.TYPE_bit, o))
    NIL = -(2**127)
    assert ora.analyticalsum(B, P, O, None, None, ora.TYPE_hge, 3).values() == [3, 3, 6, NIL, 11, 11, 18]
    assert ora.analyticalsum(B, P, O, None, None, ora.TYPE_hge, 4).values() == [6, 6, 3, 18, 18, 18, 7]
    assert list(ora.analyticalcount(B, P, O, None, None, True, 3).values()) == [2, 2, 3, 0, 2, 2, 3]
    s = ora.Bat.from_array(ora.TYPE_oid, np.array([0, 0, 1, 3, 3, 4, 5], np.uint64))
    e = ora.Bat.from_array(ora.TYPE_oid, np.array([2, 3, 3, 4, 6, 7, 7], np.uint64))
    assert list(ora.analyticalsum(B, P, O, s, e, ora.TYPE_lng, 1).values()) == [3, 6, 5, -(2**63), 11, 18, 13]


def test_firstn_maltest(ora):
    """Plain top-n (no group ids): the rows the reference's heap keeps,
    including its choice among tied rows (pqueue*.maltest)."""
    from helpers import firstn_cases
    n_checked = 0
    for src, c in firstn_cases(plain_only=True):
        b = ora.Bat.from_array(ora.TYPE_int, np.array(c["values"], np.int32))
        s = g = None
        if c["s"]:
            s = ora.Bat.from_array(ora.TYPE_oid, np.array(c["s_values"], np.uint64))
            g = ora.Bat.from_array(ora.TYPE_oid, np.array(c["g_values"], np.uint64))
        t = ora.BATfirstn(b, c["n"], s=s, g=g, asc=c["asc"], nilslast=c["nilslast"])
        assert [int(v) for v in t.values()] == c["expected"]["topn"], (src, c)
        n_checked += 1
    assert n_checked >= 27


def test_firstn_oracle_sets(ora):
    """Heap restatement: strictly-better rows always in, right count, the
    rest tied with the n-th value; sorted inputs take the reference's slices."""
    r = np.random.default_rng(11)
    for trial in range(40):
        N = int(r.integers(2, 400))
        v = r.integers(-5, 5, N).astype(np.int32)
        v[r.random(N) < 0.1] = -(1 << 31)
        if trial % 5 == 0:
            v = np.sort(v)
        elif trial % 5 == 1:
            v = np.sort(v)[::-1].copy()
        for asc in (True, False):
            for nilslast in (True, False):
                n = int(r.integers(1, N + 1))
                t = np.array(ora.BATfirstn(ora.Bat.from_array(ora.TYPE_int, v), n, asc=asc,
                                           nilslast=nilslast).values(), np.int64)
                assert len(t) == min(n, N)
                assert np.all(np.diff(t) > 0)
                if trial % 5 == 1 and nilslast == asc and (v == -(1 << 31)).any():
                    continue        # reverse-sorted with nils: the reference's slice (see oracle)
                x = v.astype(np.float64)
                x[v == -(1 << 31)] = np.inf if nilslast else -np.inf
                key = x if asc else -x
                if not asc:
                    key[v == -(1 << 31)] = np.inf if nilslast else -np.inf
                kth = np.sort(key)[min(n, N) - 1]
                assert np.all(np.isin(np.flatnonzero(key < kth), t))
                assert np.all(key[t] <= kth)


def test_sort_maltest(ora):
    """algebra.sort of orderidx00 / orderidx04.maltest: sorted values and
    (stable) order oids."""
    from helpers import FIX
    for fx in FIX["sort"]:
        for c in fx["cases"]:
            b = ora.Bat.from_array(ora.TYPE_int, np.array(c["values"], np.int32))
            srt, order = ora.BATsort(b, reverse=c["reverse"], nilslast=c["nilslast"])
            assert [int(v) for v in srt.values()] == c["sorted"]
            if c["order"]:
                assert [int(v) for v in order.values()] == c["order_oids"]


def test_window_frames_sqltest(ora):
    """analytics03.test windowed SUM / COUNT with peer-closed frames."""
    from helpers import replay_window_frames
    bad = replay_window_frames(
        lambda b, p, o, tp2, f: ora.analyticalsum(b, p, o, None, None, tp2, f).values(),
        lambda b, p, o, ign, f: ora.analyticalcount(b, p, o, None, None, ign, f).values(),
        lambda tp, a: ora.Bat.from_array(tp, a), ora.TYPE_int, ora.TYPE_bit, ora.TYPE_lng)
    assert not bad, bad


def test_fsum_oracle(ora):
    """dofsum restatement (gdk_aggr.c:183-427) = the correctly rounded sum
    (msum), checked against math.fsum; flt results are that double cast."""
    r = np.random.default_rng(91)
    for trial in range(30):
        n = int(r.integers(1, 3000))
        v = r.standard_normal(n) * 10.0 ** r.integers(-20, 20, n)
        if trial % 3 == 0:
            v = np.concatenate([v, -v[: n // 2]])
        B = ora.Bat.from_array(ora.TYPE_dbl, v)
        assert ora.BATsum(ora.TYPE_dbl, B) == math.fsum(v)
        f = v.astype(np.float32)
        assert np.float32(ora.BATsum(ora.TYPE_flt, ora.Bat.from_array(ora.TYPE_flt, f))) == \
            np.float32(math.fsum(f.astype(np.float64)))
    big = np.array([1e308, 1e308, -1e308], np.float64)         # intermediate overflow, finite result
    assert ora.BATsum(ora.TYPE_dbl, ora.Bat.from_array(ora.TYPE_dbl, big)) == 1e308
    with pytest.raises(ora.OracleError, match="overflow"):
        ora.BATsum(ora.TYPE_dbl, ora.Bat.from_array(ora.TYPE_dbl, np.array([1e308, 1e308])))


def test_groupavg_oracle(ora):
    """BATgroupavg (gdk_aggr.c:1801): integer averages are floor + remainder
    (exact, checked against Fractions), flt/dbl replay AVERAGE_ITER_FLOAT
    in row order (checked against the same recurrence in Python)."""
    from fractions import Fraction
    r = np.random.default_rng(5)
    n, ng = 3000, 7
    gid = r.integers(0, ng, n).astype(np.uint64)
    G = ora.Bat.from_array(ora.TYPE_oid, gid)
    v = r.integers(-2**62, 2**62, n).astype(np.int64)
    v[r.random(n) < 0.05] = -(2**63)
    for skip in (True, False):
        a, c = ora.BATgroupavg(ora.Bat.from_array(ora.TYPE_lng, v), G, None, skip_nils=skip)
        for k in range(ng):
            x = v[gid == k]
            if not skip and (x == -(2**63)).any():
                assert math.isnan(a.values()[k]) and c.values()[k] == 0
                continue
            x = [int(t) for t in x if t != -(2**63)]
            q, m = divmod(sum(x), len(x))
            assert a.values()[k] == float(q) + float(m) / len(x)
            assert c.values()[k] == len(x)
    f = r.standard_normal(n) * 1e3
    f[r.random(n) < 0.05] = np.nan
    a, c = ora.BATgroupavg(ora.Bat.from_array(ora.TYPE_dbl, f), G, None, skip_nils=True, scale=2)
    for k in range(ng):
        av, cnt = 0.0, 0
        for x in f[gid == k]:
            if math.isnan(x):
                continue
            cnt += 1
            av = av + (x - av) / cnt if (av > 0) == (x > 0) else av - av / cnt + x / cnt
        assert a.values()[k] == av / 100.0 and c.values()[k] == cnt
    # singleton groups: converted values, counts 1, no scale
    Gd = ora.Bat.from_array(ora.TYPE_oid, np.arange(n, dtype=np.uint64)[::-1], key=True, nonil=True)
    a, c = ora.BATgroupavg(ora.Bat.from_array(ora.TYPE_lng, v), Gd, None, skip_nils=False, scale=3)
    want = np.where(v == -(2**63), np.nan, v.astype(np.float64))
    np.testing.assert_array_equal(np.array(a.values()), want)
    assert set(c.values()) == {1}


def test_window_avg_sqltest(ora):
    """analytics03.test's windowed AVG answers (int and real inputs)."""
    from helpers import replay_window_avg
    bad = replay_window_avg(
        lambda b, p, o, f: ora.analyticalavg(b, p, o, None, None, f).values(),
        lambda tp, a: ora.Bat.from_array(tp, np.asarray(a)), ora.TYPE_int, ora.TYPE_flt, ora.TYPE_bit)
    assert not bad, bad


def _cdiv(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _avg_iter(x, st):
    """AVERAGE_ITER (gdk_calc_private.h:231-275) with C integer division"""
    a, rr, n = st
    n += 1
    an, xn = _cdiv(a, n), _cdiv(x, n)
    z1 = xn - an
    xn, an = x - xn * n, a - an * n
    if xn >= an:
        z2 = xn - an
        while z2 >= n:
            z2 -= n
            z1 += 1
    else:
        z2 = an - xn
        while True:
            z1 -= 1
            if z2 < n:
                z2 = n - z2
                break
            z2 -= n
    a, rr = a + z1, rr + z2
    if rr >= n:
        rr, a = rr - n, a + 1
    return [a, rr, n]


def _tree_avg(vals, s, e, fin=None):
    """segment-tree AVG of one partition (gdk_analytic.h:63-130): nodes
    [a, rr, n], inner nodes fold their non-empty children's a"""
    levels = [[[v, 0, 1] if v is not None else [0, 0, 0] for v in vals]]
    while len(levels[-1]) > 1 or len(levels) == 1:
        prev, nxt = levels[-1], []
        for pos in range(0, len(prev), 16):
            acc = [0, 0, 0]
            for c in prev[pos:pos + 16]:
                if c[2]:
                    acc = _avg_iter(c[0], acc)
            nxt.append(acc)
        levels.append(nxt)
    out = []
    for b, t in zip(s, e):
        acc = [0, 0, 0]
        if b < t:
            for lv in levels:
                pb, pe = b // 16, t // 16
                if pb == pe:
                    for x in lv[b:t]:
                        if x[2]:
                            acc = _avg_iter(x[0], acc)
                    break
                if b != pb * 16:
                    for x in lv[b:pb * 16 + 16]:
                        if x[2]:
                            acc = _avg_iter(x[0], acc)
                    pb += 1
                for x in lv[pe * 16:t]:
                    if x[2]:
                        acc = _avg_iter(x[0], acc)
                b, t = pb, pe
        if fin is not None:
            out.append(fin(acc))
            continue
        out.append(math.nan if acc[2] == 0 else acc[0] + acc[1] / acc[2])
    return out


def test_window_avg_tree_oracle(ora):
    """The oracle's general-frame AVG replays the reference's segment tree
    (average of child averages, not the exact frame average), checked against
    an independent Python restatement on two partitions."""
    r = np.random.default_rng(11)
    sizes = [700, 300]
    n = sum(sizes)
    v = r.integers(-10**12, 10**12, n).astype(np.int64)
    v[r.random(n) < 0.05] = -(2**63)
    p = np.zeros(n, np.int8)
    p[0] = 1
    p[sizes[0]] = 1
    s = np.empty(n, np.uint64)
    e = np.empty(n, np.uint64)
    k = 0
    for sz in sizes:
        for i in range(sz):
            s[k + i] = k + max(0, i - int(r.integers(0, 300)))
            e[k + i] = k + min(sz, i + 1 + int(r.integers(0, 300)))
        k += sz
    got = ora.analyticalavg(ora.Bat.from_array(ora.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_bit, p), None,
                            ora.Bat.from_array(ora.TYPE_oid, s), ora.Bat.from_array(ora.TYPE_oid, e), 1).values()
    k = 0
    for sz in sizes:
        vals = [None if x == -(2**63) else int(x) for x in v[k:k + sz]]
        want = _tree_avg(vals, [int(x) - k for x in s[k:k + sz]], [int(x) - k for x in e[k:k + sz]])
        np.testing.assert_array_equal(np.array(got[k:k + sz]), np.array(want))
        k += sz


def test_groupavg3combine_oracle(ora):
    """BATgroupavg3combine (gdk_aggr.c:2634) of per-shard BATgroupavg3
    partials equals BATgroupavg3 over the whole input (its purpose in the
    mitosis/mergetable plan), here checked on exact integers."""
    r = np.random.default_rng(17)
    n, ng, shards = 6000, 9, 4
    v = r.integers(-10**9, 10**9, n).astype(np.int64)
    v[r.random(n) < 0.03] = -(2**63)
    gid = r.integers(0, ng, n).astype(np.uint64)
    A, R, K, G = [], [], [], []
    for sh in np.array_split(np.arange(n), shards):
        a, rm, c = ora.BATgroupavg3(ora.Bat.from_array(ora.TYPE_lng, v[sh]),
                                    ora.Bat.from_array(ora.TYPE_oid, gid[sh]), None, True)
        A += list(a.values())
        R += list(rm.values())
        K += list(c.values())
        G += list(range(ng))
    comb = ora.BATgroupavg3combine(ora.Bat.from_array(ora.TYPE_lng, np.array(A, np.int64)),
                                   ora.Bat.from_array(ora.TYPE_lng, np.array(R, np.int64)),
                                   ora.Bat.from_array(ora.TYPE_lng, np.array(K, np.int64)),
                                   ora.Bat.from_array(ora.TYPE_oid, np.array(G, np.uint64)), None, True)
    full, _, _ = ora.BATgroupavg3(ora.Bat.from_array(ora.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_oid, gid),
                                  None, True)
    assert list(comb.values()) == list(full.values())


def _round_avg(a, rr, n):
    """ANALYTICAL_AVERAGE_INT_CALC_FINALIZE: half away from zero"""
    if rr > 0 and (2 * rr > n if a < 0 else 2 * rr >= n):
        a += 1
    return a


def test_window_avginteger_oracle(ora):
    """GDKanalyticalavginteger (gdk_analytic_statistics.c:428-700): running
    frames give the exact average rounded half away from zero (checked with
    Python integers); general frames the segment tree's folded state,
    rounded the same way (checked with the Python tree restatement)."""
    r = np.random.default_rng(13)
    sizes = [500, 300, 1]
    n = sum(sizes)
    v = r.integers(-10**6, 10**6, n).astype(np.int32)
    v[r.random(n) < 0.05] = -(2**31)
    p = np.zeros(n, np.int8)
    p[np.cumsum([0] + sizes[:-1])] = 1
    ob = np.concatenate([np.sort(r.integers(0, sz // 4 + 1, sz)) for sz in sizes])
    o = p.copy()
    o[1:] |= (ob[1:] != ob[:-1]).astype(np.int8)
    B, P, O = (ora.Bat.from_array(ora.TYPE_int, v), ora.Bat.from_array(ora.TYPE_bit, p),
               ora.Bat.from_array(ora.TYPE_bit, o))
    NIL = -(2**31)

    def exact(xs):
        xs = [int(x) for x in xs if x != NIL]
        if not xs:
            return NIL
        q, m = divmod(sum(xs), len(xs))
        return _round_avg(q, m, len(xs))
    got5 = ora.analyticalavginteger(B, P, O, None, None, 5).values()
    got3 = ora.analyticalavginteger(B, P, O, None, None, 3).values()
    got4 = ora.analyticalavginteger(B, P, O, None, None, 4).values()
    k = 0
    for sz in sizes:
        part = v[k:k + sz]
        pstart = np.flatnonzero(o[k:k + sz])
        pend = np.append(pstart[1:], sz)
        for a, b_ in zip(pstart, pend):
            assert all(got5[k + i] == exact(part) for i in range(a, b_))
            assert all(got3[k + i] == exact(part[:b_]) for i in range(a, b_))
            assert all(got4[k + i] == exact(part[a:]) for i in range(a, b_))
        k += sz
    s = np.empty(n, np.uint64)
    e = np.empty(n, np.uint64)
    k = 0
    for sz in sizes:
        for i in range(sz):
            s[k + i] = k + max(0, i - int(r.integers(0, 200)))
            e[k + i] = k + min(sz, i + 1 + int(r.integers(0, 200)))
        k += sz
    got = ora.analyticalavginteger(B, P, None, ora.Bat.from_array(ora.TYPE_oid, s),
                                   ora.Bat.from_array(ora.TYPE_oid, e), 1).values()
    k = 0
    for sz in sizes:
        vals = [None if x == NIL else int(x) for x in v[k:k + sz]]
        want = _tree_avg(vals, [int(x) - k for x in s[k:k + sz]], [int(x) - k for x in e[k:k + sz]],
                         fin=lambda acc: NIL if acc[2] == 0 else _round_avg(acc[0], acc[1], acc[2]))
        assert list(got[k:k + sz]) == want
        k += sz


# ---- window frame bounds pinned on the reference's SQL fixtures ------------
def _ora_bounds(ora):
    def f(b, p, l, lim, tp1, tp2, unit, pre, sh):
        return ora.windowbounds(b, p, l, lim, tp1, tp2, unit, pre, sh).values()
    return f


def _ora_make(ora):
    return lambda tp, a: ora.Bat.from_array(tp, a)


def test_windowbounds_employee_fixture(ora):
    """window_functions.test: SUM(salary) over ROWS / GROUPS / RANGE frames."""
    from helpers import replay_employee
    assert replay_employee(_ora_bounds(ora), _ora_make(ora)) == []


def test_windowbounds_interval_fixture(ora):
    """analytics07.test: RANGE frames with month / second intervals on
    date, timestamp and time columns (asc and desc)."""
    from helpers import replay_intervals
    assert replay_intervals(_ora_bounds(ora), _ora_make(ora)) == []


def test_windowbounds_interval_errors(ora):
    from helpers import bound_args, interval_cases
    n = 0
    for c, tp, v in interval_cases(errors=True):
        b = ora.Bat.from_array(tp, v)
        with pytest.raises(ora.OracleError, match="42000!"):
            for bnd, st in ((c["start"], True), (c["end"], False)):
                pre, sh, tp2, lim = bound_args(1, bnd, st, tp)
                ora.windowbounds(b, None, None, lim, tp, tp2, 1, pre, sh)
        n += 1
    assert n == 2


def test_project_maltest(ora):
    """algebra.projection of algebra.select results: tst033 / tst034 /
    orderidx02.maltest (20 cases)"""
    mk = lambda tp, v: ora.Bat.from_array(tp, np.array(v, np.int32))
    assert sum(len(f["cases"]) for f in FIX["project"]) == 20
    bad = replay_project(ora, mk, ora.TYPE_int, ora.NIL[ora.TYPE_int])
    assert not bad, bad[:3]


def test_window_sqltests_oracle(ora):
    """analytics00 / 01 / 02 / 14 / 15.test (the reference's own answers):
    ntile, first_value, last_value, nth_value, lag, lead, min, max, sum,
    count, avg, prod, stddev / variance / covariance (samp, pop) and corr over
    PARTITION BY / ORDER BY / ROWS frames, replayed through the oracle's
    restatement of gdk_analytic_func.c / gdk_analytic_statistics.c /
    gdk_analytic_bounds.c."""
    from helpers import replay_window_sqltests, sqlwin_api_ora
    ran, bad = replay_window_sqltests(sqlwin_api_ora(ora))
    assert ran >= 346
    assert not bad, bad[:3]
