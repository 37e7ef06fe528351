"""The oracle (oracle/liboracle.so, CPU restatement) against the reference's own
known-answer fixtures (tests/golden/maltest_fixtures.json, extracted from
monetdb5/modules/kernel/Tests/select.maltest, monetdb5/mal/Tests/tst1500.maltest,
tst1503.maltest and monetdb5/modules/mal/Tests/bigsum.maltest)."""
import math

import numpy as np
import pytest

from helpers import FIX, replay_select


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
