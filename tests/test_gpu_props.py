"""Result properties of the device operators against the oracle's restatement
of the reference's rules (tsorted / trevsorted / tkey /
tnonil / tnil / tseqbase, void results, and BATgroup's tmaxpos and
tunique_est).  Every case compares the values too."""
import numpy as np
import pytest

from helpers import rng

pytestmark = pytest.mark.gpu

NIL32 = -(1 << 31)


def dprops(b, extra=False):
    s = b.s
    p = dict(type="void" if s.ttype == 0 else s.ttype, count=s.count, sorted=bool(s.tsorted),
             revsorted=bool(s.trevsorted), key=bool(s.tkey), nonil=bool(s.tnonil), nil=bool(s.tnil))
    if s.ttype in (0, 6):
        p["tseqbase"] = s.tseqbase
    if extra:
        p["maxpos"] = s.tmaxpos
        p["unique_est"] = s.tunique_est
    return p


def oprops(b, extra=False):
    s = b.s
    p = dict(type="void" if s.type == 0 else s.type, count=s.count, sorted=bool(s.sorted),
             revsorted=bool(s.revsorted), key=bool(s.key), nonil=bool(s.nonil), nil=bool(s.nil))
    if s.type in (0, 6):
        p["tseqbase"] = s.tseqbase
    if extra:
        p["maxpos"] = s.maxpos
        p["unique_est"] = s.unique_est
    return p


def same(d, o, extra=False, what=""):
    assert np.array_equal(np.asarray(d.values()), np.asarray(o.values())), what
    assert dprops(d, extra) == oprops(o, extra), what


def pair(gdk, ora, tp, vals, hseq=0, **flags):
    """the same BAT on both sides with the same known flags"""
    kw = dict(sorted_=flags.get("sorted", False), revsorted=flags.get("revsorted", False),
              key=flags.get("key", False), nonil=flags.get("nonil", False))
    a = np.asarray(vals)
    d = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tp), a, hseqbase=hseq, **kw)
    o = ora.Bat.from_array(getattr(ora, "TYPE_" + tp), a, hseqbase=hseq, **kw)
    o.s.nil = d.s.tnil          # both know whether a nil is present
    return d, o


def cands(gdk, ora, oids):
    oids = np.asarray(oids, np.uint64)
    return pair(gdk, ora, "oid", oids, sorted=True, key=True, nonil=True, revsorted=len(oids) <= 1)


@pytest.mark.parametrize("case", ["unsorted", "sorted", "cand", "all", "none", "one", "nil"])
def test_select_props(gdk, ora, case):
    r = rng(301)
    v = r.integers(0, 1000, 50_000).astype(np.int32)
    flags = {}
    if case == "sorted":
        v = np.sort(v)
        flags = dict(sorted=True, nonil=True)
    if case == "nil":
        v[::31] = NIL32
    D, O = pair(gdk, ora, "int", v, hseq=7, **flags)
    lo, hi = {"all": (-10, 2000), "none": (5000, 6000), "one": (int(v[123]), int(v[123]))}.get(case, (100, 300))
    s = (None, None)
    if case == "cand":
        s = cands(gdk, ora, np.sort(r.choice(50_000, 20_000, replace=False)) + 7)
    d = gdk.BATselect(D, s[0], lo, hi, True, True, False)
    o = ora.BATselect(O, s[1], lo, hi, True, True, False)
    same(d, o, what=case)
    d = gdk.BATthetaselect(D, s[0], 500, "<")
    o = ora.BATthetaselect(O, s[1], 500, "<")
    same(d, o, what=case + " theta")


@pytest.mark.parametrize("case", ["dense_l", "sorted_l", "random_l", "nil_oids", "sorted_key_r"])
def test_project_props(gdk, ora, case):
    r = rng(302)
    n = 30_000
    rv = r.integers(-500, 500, n).astype(np.int64)
    rflags = {}
    if case == "sorted_key_r":
        rv = np.arange(n, dtype=np.int64) * 3
        rflags = dict(sorted=True, key=True, nonil=True)
    R, OR = pair(gdk, ora, "lng", rv, hseq=5, **rflags)
    if case == "dense_l":
        L, OL = gdk.BAT.dense(105, 2000), ora.Bat.dense(105, 2000)
    elif case in ("sorted_l", "sorted_key_r"):
        L, OL = cands(gdk, ora, np.sort(r.choice(n, 9000, replace=False)) + 5)
    else:
        lo = r.integers(5, n + 5, 9000).astype(np.uint64)
        if case == "nil_oids":
            lo[::17] = 1 << 63
        L, OL = pair(gdk, ora, "oid", lo)
    same(gdk.BATproject(L, R), ora.BATproject(OL, OR), what=case)


@pytest.mark.parametrize("op", ["+", "-", "*"])
@pytest.mark.parametrize("shape", ["bb", "bc_pos", "bc_neg", "cb", "sorted_bb", "nil"])
def test_calc_props(gdk, ora, op, shape):
    r = rng(303)
    n = 20_000
    a = r.integers(-1000, 1000, n).astype(np.int32)
    b = r.integers(-1000, 1000, n).astype(np.int32)
    fa = fb = {}
    if shape.startswith("sorted") or shape in ("bc_pos", "bc_neg", "cb"):
        a, b = np.sort(a), np.sort(b)
        fa = fb = dict(sorted=True, nonil=True)
    if shape == "nil":
        a[::13] = NIL32
    A, OA = pair(gdk, ora, "int", a, **fa)
    B, OB = pair(gdk, ora, "int", b, **fb)
    fn = {"+": "add", "-": "sub", "*": "mul"}[op]
    if shape in ("bb", "sorted_bb", "nil"):
        d = getattr(gdk, "BATcalc" + fn)(A, B, gdk.TYPE_lng)
        o = ora.BATcalc(op, OA, OB, ora.TYPE_lng)
    elif shape in ("bc_pos", "bc_neg"):
        c = 7 if shape == "bc_pos" else -7
        d = getattr(gdk, "BATcalc" + fn + "cst")(A, c, gdk.TYPE_int, gdk.TYPE_lng)
        o = ora.BATcalc(op, OA, None, ora.TYPE_lng, c2=c, t2=ora.TYPE_int)
    else:
        d = getattr(gdk, "BATcalccst" + fn)(-3, gdk.TYPE_int, A, gdk.TYPE_lng)
        o = ora.BATcalc(op, None, OA, ora.TYPE_lng, c1=-3, t1=ora.TYPE_int)
    same(d, o, what=(op, shape))


@pytest.mark.parametrize("case", ["general", "cand", "subgroup", "key", "single", "nils", "contiguous",
                                  "wide"])
def test_group_props(gdk, ora, case):
    r = rng(304)
    n = 40_000
    v = r.integers(0, 50, n).astype(np.int32)
    flags, s, g = {}, (None, None), (None, None)
    if case == "nils":
        v[::7] = NIL32
    if case == "key":
        v = r.permutation(n).astype(np.int32)
        flags = dict(key=True, nonil=True)
    if case == "single":
        v = np.full(n, 3, np.int32)
        flags = dict(sorted=True, revsorted=True, nonil=True)
    if case == "contiguous":
        v = np.sort(v)
    if case == "wide":
        v = r.integers(0, 20_000, n).astype(np.int32)
    D, O = pair(gdk, ora, "int", v, hseq=3, **flags)
    if case == "cand":
        s = cands(gdk, ora, np.sort(r.choice(n, 15_000, replace=False)) + 3)
    if case == "subgroup":
        g0d, _, _ = gdk.BATgroup(gdk.BAT.from_numpy(gdk.TYPE_int, (v % 3).astype(np.int32), hseqbase=3))
        g0o, _, _ = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, (v % 3).astype(np.int32), hseqbase=3))
        g = (g0d, g0o)
    gd, ed, hd = gdk.BATgroup(D, s[0], g[0])
    go, eo, ho = ora.BATgroup(O, s[1], g[1])
    same(gd, go, extra=True, what="groups")
    same(ed, eo, what="extents")
    assert dprops(ed)["count"] == oprops(eo)["count"]
    if ed.s.ttype == 6:
        assert ed.s.tunique_est == eo.s.unique_est
    same(hd, ho, what="histo")
    # the estimate BATgroup leaves on its input (gdk_group.c:1316-1317)
    assert D.s.tunique_est == O.s.unique_est


@pytest.mark.parametrize("agg", ["sum", "count", "min", "max"])
def test_grouped_aggregate_props(gdk, ora, agg):
    r = rng(305)
    n = 30_000
    v = r.integers(-100, 100, n).astype(np.int64)
    v[::11] = -(1 << 63)
    k = r.integers(0, 9, n).astype(np.int32)
    gd, ed, _ = gdk.BATgroup(gdk.BAT.from_numpy(gdk.TYPE_int, k))
    go, eo, _ = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, k))
    D, O = pair(gdk, ora, "lng", v)
    if agg == "sum":
        d, o = gdk.BATgroupsum(D, gd, ed, gdk.TYPE_hge), ora.BATgroupsum(O, go, eo, ora.TYPE_hge)
    elif agg == "count":
        d, o = gdk.BATgroupcount(D, gd, ed), ora.BATgroupcount(O, go, eo)
    elif agg == "min":
        d, o = gdk.BATgroupmin(D, gd, ed), ora.BATgroupminmax(O, go, eo, False)
    else:
        d, o = gdk.BATgroupmax(D, gd, ed), ora.BATgroupminmax(O, go, eo, True)
    same(d, o, what=agg)


@pytest.mark.parametrize("reverse", [False, True])
def test_sort_props(gdk, ora, reverse):
    r = rng(306)
    v = r.integers(-500, 500, 30_000).astype(np.int32)
    v[::29] = NIL32
    D, O = pair(gdk, ora, "int", v)
    sd, od_, _ = gdk.BATsort(D, reverse=reverse, nilslast=reverse)
    so, oo = ora.BATsort(O, reverse=reverse, nilslast=reverse)
    same(sd, so, what="sorted")
    same(od_, oo, what="order")
