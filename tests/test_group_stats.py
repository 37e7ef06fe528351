"""Grouped and whole-column statistics: BATgroupstdev_* / BATgroupvariance_*
(dogroupstdev, gdk/gdk_aggr.c:4612), BATgroupcovariance_* (:4851),
BATgroupcorrelation (:5057), BATcalcstdev_* / BATcalcvariance_*
(calcvariance :4276), BATcalccovariance_* (:4404), BATcalccorrelation
(:4503), and BATgroupmedian / BATgroupquantile / _avg (doBATgroupquantile
:3881).

Pinning: the reference's own SQL tests -- sql/test/quantiles/Tests/
quantiles.test (10000 DECIMAL(15,2) prices, quantiles whole and per
l_returnflag, p outside [0,1] an error), sql/test/Tests/median_stdev.test,
sql/test/BugTracker-2013/Tests/stddev-group.Bug-3257.test and
median-null.Bug-3280.test -- replayed through the oracle and the device
(tests/golden/stats_fixtures.json, made by make_maltest_fixtures.py).  The
oracle's Welford loops are further checked bit for bit against a pure-Python
restatement (Python floats are IEEE doubles, the same operations in the same
order), and the device against the oracle bit for bit on every value type,
group count, candidate form and nil rule."""
import json
import math
import os

import numpy as np
import pytest

from helpers import rng

HERE = os.path.dirname(os.path.abspath(__file__))
SFX = json.load(open(os.path.join(HERE, "golden", "stats_fixtures.json")))
I64N = -(1 << 63)
NILS = {"bte": -(1 << 7), "sht": -(1 << 15), "int": -(1 << 31), "lng": I64N}
NPT = {"bte": np.int8, "sht": np.int16, "int": np.int32, "lng": np.int64, "flt": np.float32, "dbl": np.float64}


def _hge_words(v):
    v = np.asarray(v, np.int64)
    w = np.empty((len(v), 2), np.uint64)
    w[:, 0] = v.view(np.uint64)
    w[:, 1] = np.where(v < 0, np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64(0))
    nil = v == I64N
    w[nil, 0] = 0
    w[nil, 1] = np.uint64(1 << 63)
    return w


def _col(mod, tname, v):
    """a BAT of type tname from int64 / float64 values (I64N / NaN = nil)"""
    tp = getattr(mod, "TYPE_" + tname)
    if tname == "hge":
        a = _hge_words(v)
    elif tname in ("flt", "dbl"):
        a = np.asarray(v, NPT[tname])
    else:
        a = np.asarray(v, np.int64)
        a = np.where(a == I64N, NILS[tname], a).astype(NPT[tname])
    if hasattr(mod, "Bat"):
        return mod.Bat.from_array(tp, a)
    return mod.BAT.from_numpy(tp, a, sorted_=False, revsorted=False, key=False)


def _oids(mod, v, hseq=0, dense=None):
    if dense is not None:
        return mod.Bat.dense(dense, len(v)) if hasattr(mod, "Bat") else mod.BAT.dense(dense, len(v))
    a = np.asarray(v, np.uint64)
    if hasattr(mod, "Bat"):
        return mod.Bat.from_array(mod.TYPE_oid, a, hseqbase=hseq)
    return mod.BAT.from_numpy(mod.TYPE_oid, a, hseqbase=hseq, sorted_=False, revsorted=False, key=False)


def _vals(b):
    return np.asarray(b.values() if hasattr(b, "values") and not hasattr(b, "to_numpy") else b.to_numpy())


class OraAPI:
    def __init__(self, ora):
        self.m = ora

    def group(self, name, b1, b2, g, e, skip_nils, s, sample):
        return np.asarray(self.m.BATgroupstat(name, b1, b2, g, e, skip_nils, s, sample).values(), np.float64)

    def calc(self, name, b1, b2, sample):
        return self.m.BATcalcstat(name, b1, b2, sample)

    def quantile(self, b, g, e, q, skip_nils=True, s=None, average=False):
        r = self.m.BATgroupquantile(b, g, e, q, skip_nils, s, average)
        return r, np.asarray(r.values())


class GdkAPI:
    def __init__(self, gdk):
        self.m = gdk

    def group(self, name, b1, b2, g, e, skip_nils, s, sample):
        G = self.m
        if name in ("stdev", "variance"):
            f = getattr(G, "BATgroup%s_%s" % (name, "sample" if sample else "population"))
            r = f(b1, g, e, skip_nils, s)
        elif name == "covariance":
            r = getattr(G, "BATgroupcovariance_%s" % ("sample" if sample else "population"))(b1, b2, g, e,
                                                                                             skip_nils, s)
        else:
            r = G.BATgroupcorrelation(b1, b2, g, e, skip_nils, s)
        return r.to_numpy().astype(np.float64)

    def calc(self, name, b1, b2, sample):
        G = self.m
        if name in ("stdev", "variance"):
            return G.BATcalcvariance(b1, sample, stdev=name == "stdev")
        if name == "covariance":
            return G.BATcalccovariance(b1, b2, sample), math.nan
        return G.BATcalccorrelation(b1, b2), math.nan

    def quantile(self, b, g, e, q, skip_nils=True, s=None, average=False):
        r = self.m.BATgroupquantile(b, g, e, q, skip_nils, s, average)
        return r, r.to_numpy()


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f" or b.dtype.kind == "f":
        a, b = a.astype(np.float64), b.astype(np.float64)
        return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))) and
                    np.array_equal(np.signbit(a[~np.isnan(a)]), np.signbit(b[~np.isnan(b)])))
    return np.array_equal(a, b)


# ---- the reference's SQL tests --------------------------------------------------

def _fmt3(x):
    return "%.3f" % x


def _cents(v):
    v = int(v)
    return "%s%d.%02d0" % ("-" if v < 0 else "", abs(v) // 100, abs(v) % 100)


def _groups(keys):
    """group ids in order of first appearance (BATgroup's numbering) and count"""
    ids, out = {}, []
    for k in keys:
        out.append(ids.setdefault(k, len(ids)))
    return np.asarray(out, np.uint64), len(ids)


def replay_stats_sqltests(api, mod):
    """every query of the four reference tests; returns the number checked"""
    done = 0
    fx = SFX["quantiles"]
    price = np.asarray(fx["price_cents"], np.int64)
    gid, ng = _groups(fx["flag"])
    b = _col(mod, "lng", price)
    for qy in fx["queries"]:
        g = _oids(mod, gid) if qy["grouped"] else None
        e = _oids(mod, np.zeros(ng), dense=0) if qy["grouped"] else None
        if qy["error"]:
            for _, p in qy["items"]:
                with pytest.raises(Exception, match="quantile"):
                    api.quantile(b, g, e, p)
            done += 1
            continue
        cols = [[_cents(v) for v in api.quantile(b, g, e, p)[1]] for _, p in qy["items"]]
        rows = sorted(zip(*cols))
        assert [x for r in rows for x in r] == qy["expected"], qy
        done += 1
    fx = SFX["median_stdev"]
    for qy in fx["queries"]:
        v = np.asarray(fx[qy["column"]], np.int64)
        if qy["grouped"]:
            gid, ng = _groups(fx["groupID"])
            r = api.quantile(_col(mod, "int", v), _oids(mod, gid), _oids(mod, np.zeros(ng), dense=0), 0.5)[1]
            keys = list(dict.fromkeys(fx["groupID"]))
            got = [str(x) for k, m in sorted(zip(keys, r)) for x in (k, int(m))]
        else:
            got = [str(int(api.quantile(_col(mod, "int", v), None, None, 0.5)[1][0]))]
        assert got == qy["expected"], qy
        done += 1
    fx = SFX["stddev_group"]
    i = _col(mod, "int", fx["i"])
    for qy in fx["queries"]:
        name = "stdev" if qy["func"] == "stddev_pop" else "variance"
        if qy["grouped"]:
            gid, ng = _groups(fx["j"])
            r = api.group(name, i, None, _oids(mod, gid), _oids(mod, np.zeros(ng), dense=0), True, None, False)
            got = sorted(_fmt3(x) for x in r)
        else:
            got = [_fmt3(api.calc(name, i, None, False)[0])]
        assert got == qy["expected"], qy
        done += 1
    fx = SFX["median_null"]
    mpg = np.asarray([math.nan if x is None else x for x in fx["mpg"]], np.float64)
    r = api.quantile(_col(mod, "dbl", mpg), None, None, 0.5)[1]
    assert [_fmt3(r[0])] == fx["expected"]
    return done + 1


def test_stats_sqltests_oracle(ora):
    assert replay_stats_sqltests(OraAPI(ora), ora) == 30


@pytest.mark.gpu
def test_gpu_stats_sqltests(gdk):
    assert replay_stats_sqltests(GdkAPI(gdk), gdk) == 30


# ---- the oracle against a pure-Python restatement -----------------------------------

def _py_moments(kind, xs, ys, gids, ng, skip_nils, issample, variance):
    """AGGR_STDEV / AGGR_COVARIANCE / AGGR_CORRELATION and their result steps,
    in Python floats (IEEE doubles: the same roundings)"""
    st = [[0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0] for _ in range(ng)]   # cnt mean1 mean2 m2 up down1 down2
    NONE = -1
    for x, y, g in zip(xs, ys, gids):
        s = st[g]
        if x is None or (kind != "var" and y is None):
            if not skip_nils:
                s[0] = NONE
            continue
        if s[0] == NONE:
            continue
        s[0] += 1
        n = float(s[0])
        d1 = x - s[1]
        s[1] += d1 / n
        if kind == "var":
            s[3] += d1 * (x - s[1])
            continue
        d2 = y - s[2]
        s[2] += d2 / n
        if kind == "cov":
            s[3] += d1 * (y - s[2])
        else:
            aux = y - s[2]
            s[4] += d1 * aux
            s[5] += d1 * (x - s[1])
            s[6] += d2 * aux
    out = []
    for c, m1, m2_, m2, up, dn1, dn2 in st:
        if kind == "cor":
            if c <= 1 or dn1 == 0 or dn2 == 0:
                out.append(math.nan)
            else:
                out.append((up / c) / (math.sqrt(dn1 / c) * math.sqrt(dn2 / c)))
        elif c in (0, NONE):
            out.append(math.nan)
        elif c == 1:
            out.append(math.nan if issample else 0.0)
        else:
            v = m2 / (c - issample)
            out.append(v if (kind != "var" or variance) else math.sqrt(v))
    return np.asarray(out)


def _random_case(r, n, ng, tname, nil_frac=0.05):
    if tname in ("flt", "dbl"):
        v = r.normal(100.0, 40.0, n)
        v[r.random(n) < nil_frac] = np.nan
        if tname == "flt":
            v = v.astype(np.float32).astype(np.float64)
        return v
    hi = {"bte": 100, "sht": 30000, "int": 1 << 30, "lng": 1 << 40, "hge": 1 << 40}[tname]
    v = r.integers(-hi, hi, n).astype(np.int64)
    v[r.random(n) < nil_frac] = I64N
    return v


def _pyvals(v):
    return [None if (isinstance(x, float) and math.isnan(x)) or x == I64N else float(x) for x in v.tolist()]


@pytest.mark.parametrize("tname", ["bte", "int", "lng", "flt", "dbl"])
@pytest.mark.parametrize("kind", ["var", "cov", "cor"])
def test_oracle_moments_model(ora, tname, kind):
    r = rng(1401)
    n, ng = 3000, 37
    x, y = _random_case(r, n, ng, tname), _random_case(r, n, ng, tname)
    gids = r.integers(0, ng, n).astype(np.uint64)
    g = _oids(ora, gids)
    e = _oids(ora, np.zeros(ng), dense=0)
    bx, by = _col(ora, tname, x), _col(ora, tname, y)
    name = {"var": "variance", "cov": "covariance", "cor": "correlation"}[kind]
    for skip_nils in (True, False):
        for sample in ((True, False) if kind != "cor" else (False,)):
            for variance in ((True, False) if kind == "var" else (False,)):
                nm = name if kind != "var" else ("variance" if variance else "stdev")
                got = OraAPI(ora).group(nm, bx, by if kind != "var" else None, g, e, skip_nils, None, sample)
                want = _py_moments(kind, _pyvals(x), _pyvals(y), gids.tolist(), ng, skip_nils, sample, variance)
                assert _same(got, want), (nm, skip_nils, sample)


def test_oracle_calc_and_quantile_model(ora):
    r = rng(1402)
    v = _random_case(r, 5000, 1, "dbl")
    b = _col(ora, "dbl", v)
    val, avg = ora.BATcalcstat("stdev", b, None, True)
    want = _py_moments("var", _pyvals(v), _pyvals(v), [0] * len(v), 1, True, True, False)[0]
    assert val == want
    vals = sorted(x for x in _pyvals(v) if x is not None)
    for q in (0.0, 0.05, 0.3, 0.5, 0.77, 1.0):
        p = len(vals)
        f = (p - 1) * q
        qi = p - int(p + 0.5 - f)
        got = ora.BATgroupquantile(b, None, None, q).values()[0]
        assert got == vals[qi]
        lo, hi = math.floor(f), math.ceil(f)
        got = ora.BATgroupquantile(b, None, None, q, average=True).values()[0]
        assert got == (f - lo) * vals[hi] + (lo + 1 - f) * vals[lo]
    with pytest.raises(Exception, match="overflow"):
        ora.BATcalcstat("variance", _col(ora, "dbl", np.array([1e300, -1e300, 1e300])), None, False)


# ---- the device against the oracle -----------------------------------------------

MOMENT_TYPES = ["bte", "sht", "int", "lng", "hge", "flt", "dbl"]


@pytest.mark.gpu
@pytest.mark.parametrize("tname", MOMENT_TYPES)
@pytest.mark.parametrize("ng", [1, 6, 2000, 60000])
def test_gpu_group_moments(gdk, ora, tname, ng):
    r = rng(1403 + ng)
    n = 150_000
    x, y = _random_case(r, n, ng, tname), _random_case(r, n, ng, tname)
    gids = r.integers(0, ng, n).astype(np.uint64)
    if ng == 6:
        gids = np.sort(gids)                       # clustered groups
    G, O = GdkAPI(gdk), OraAPI(ora)
    gx, gy, ox, oy = _col(gdk, tname, x), _col(gdk, tname, y), _col(ora, tname, x), _col(ora, tname, y)
    for cand in ("none", "dense", "oids"):
        if cand == "none":
            sel = np.arange(n)
            gs = os_ = None
        elif cand == "dense":
            sel = np.arange(1000, n - 777)
            gs, os_ = gdk.BAT.dense(1000, len(sel)), ora.Bat.dense(1000, len(sel))
        else:
            sel = np.sort(r.choice(n, n // 3, replace=False))
            gs = gdk.BAT.from_numpy(gdk.TYPE_oid, sel.astype(np.uint64), sorted_=True, key=True, nonil=True)
            os_ = ora.Bat.from_array(ora.TYPE_oid, sel.astype(np.uint64), sorted_=True, key=True, nonil=True)
        gg = _oids(gdk, gids[sel], hseq=int(sel[0]))
        og = _oids(ora, gids[sel], hseq=int(sel[0]))
        ge, oe = gdk.BAT.dense(0, ng), ora.Bat.dense(0, ng)
        for name in ("stdev", "variance", "covariance", "correlation"):
            for skip_nils in (True, False):
                for sample in ((True, False) if name != "correlation" else (False,)):
                    two = name in ("covariance", "correlation")
                    want = O.group(name, ox, oy if two else None, og, oe, skip_nils, os_, sample)
                    got = G.group(name, gx, gy if two else None, gg, ge, skip_nils, gs, sample)
                    assert _same(got, want), (name, cand, skip_nils, sample)


@pytest.mark.gpu
def test_gpu_group_moments_trivial(gdk, ora):
    """singleton groups, empty inputs, no extents, overflow"""
    G, O = GdkAPI(gdk), OraAPI(ora)
    r = rng(1404)
    v = _random_case(r, 500, 1, "int", nil_frac=0)
    gx, ox = _col(gdk, "int", v), _col(ora, "int", v)
    for name in ("stdev", "variance", "covariance", "correlation"):
        two = name in ("covariance", "correlation")
        for sample in (True, False):
            # dense g: every group a single row
            want = O.group(name, ox, ox if two else None, ora.Bat.dense(0, 500), None, True, None, sample)
            got = G.group(name, gx, gx if two else None, gdk.BAT.dense(0, 500), None, True, None, sample)
            assert _same(got, want)
            # g with a few ids, no extents (the range comes from g)
            gi = (np.arange(500) % 7 + 3).astype(np.uint64)
            want = O.group(name, ox, ox if two else None, _oids(ora, gi), None, True, None, sample)
            got = G.group(name, gx, gx if two else None, _oids(gdk, gi), None, True, None, sample)
            assert _same(got, want) and len(got) == 7
    e0g, e0o = _col(gdk, "int", np.zeros(0, np.int64)), _col(ora, "int", np.zeros(0, np.int64))
    assert _same(G.group("stdev", e0g, None, _oids(gdk, []), None, True, None, True),
                 O.group("stdev", e0o, None, _oids(ora, []), None, True, None, True))
    big = np.array([1e300, -1e300, 1e300, 2.0])
    with pytest.raises(gdk.GDKError, match="overflow"):
        G.group("variance", _col(gdk, "dbl", big), None, _oids(gdk, [0, 0, 0, 1]), None, True, None, False)


@pytest.mark.gpu
@pytest.mark.parametrize("tname", MOMENT_TYPES)
def test_gpu_calc_moments(gdk, ora, tname):
    r = rng(1405)
    for n in (0, 1, 2, 20_000):
        x, y = _random_case(r, n, 1, tname), _random_case(r, n, 1, tname)
        gx, gy, ox, oy = _col(gdk, tname, x), _col(gdk, tname, y), _col(ora, tname, x), _col(ora, tname, y)
        for name in ("stdev", "variance", "covariance", "correlation"):
            for sample in (True, False):
                two = name in ("covariance", "correlation")
                w = OraAPI(ora).calc(name, ox, oy if two else None, sample)
                g = GdkAPI(gdk).calc(name, gx, gy if two else None, sample)
                assert _same([g[0]], [w[0]]), (name, n, sample)
                if not two:
                    assert _same([g[1]], [w[1]])
    with pytest.raises(gdk.GDKError, match="overflow"):
        gdk.BATcalcvariance(_col(gdk, "dbl", np.array([1e300, -1e300, 1e300, 2.0])), False)


QTYPES = ["bte", "sht", "int", "lng", "flt", "dbl"]


@pytest.mark.gpu
@pytest.mark.parametrize("tname", QTYPES)
@pytest.mark.parametrize("ng", [0, 1, 9, 5000])
def test_gpu_quantile(gdk, ora, tname, ng):
    r = rng(1406 + ng)
    n = 100_000
    v = _random_case(r, n, 1, tname, nil_frac=0.1)
    G, O = GdkAPI(gdk), OraAPI(ora)
    gb, ob = _col(gdk, tname, v), _col(ora, tname, v)
    if ng:
        gids = r.integers(0, ng, n).astype(np.uint64)
        gg, og = _oids(gdk, gids), _oids(ora, gids)
        ge, oe = gdk.BAT.dense(0, ng), ora.Bat.dense(0, ng)
    else:
        gg = og = ge = oe = None
    for q in (0.0, 0.05, 0.5, 0.95, 1.0, math.nan):
        for skip_nils in (True, False):
            for average in (False, True):
                wb, want = O.quantile(ob, og, oe, q, skip_nils, None, average)
                gbat, got = G.quantile(gb, gg, ge, q, skip_nils, None, average)
                assert _same(got, want), (q, skip_nils, average)
                assert gbat.hseqbase == wb.s.hseqbase
    for q in (-0.5, 1.5):
        with pytest.raises(gdk.GDKError, match="quantile"):
            G.quantile(gb, gg, ge, q)


@pytest.mark.gpu
def test_gpu_quantile_forms(gdk, ora):
    """candidates (dense: fine; with gaps and groups: BATproject's error),
    dense g (a copy of b), fewer runs than groups (nil padded)"""
    r = rng(1407)
    n = 20_000
    v = _random_case(r, n, 1, "int")
    gb, ob = _col(gdk, "int", v), _col(ora, "int", v)
    gids = r.integers(0, 40, n).astype(np.uint64)
    sel = np.arange(300, 15_000)
    gg, og = _oids(gdk, gids[sel], hseq=300), _oids(ora, gids[sel], hseq=300)
    for average in (False, True):
        want = OraAPI(ora).quantile(ob, og, ora.Bat.dense(0, 50), 0.3, True, ora.Bat.dense(300, len(sel)), average)
        got = GdkAPI(gdk).quantile(gb, gg, gdk.BAT.dense(0, 50), 0.3, True, gdk.BAT.dense(300, len(sel)), average)
        assert _same(got[1], want[1]) and len(got[1]) == 50
        # dense g
        want = OraAPI(ora).quantile(ob, ora.Bat.dense(5, n), None, 0.3, True, None, average)
        got = GdkAPI(gdk).quantile(gb, gdk.BAT.dense(5, n), None, 0.3, True, None, average)
        assert _same(got[1], want[1]) and got[0].hseqbase == 5
        # ungrouped with an oid list
        cl = np.sort(r.choice(n, 5000, replace=False)).astype(np.uint64)
        want = OraAPI(ora).quantile(ob, None, None, 0.7, True,
                                    ora.Bat.from_array(ora.TYPE_oid, cl, sorted_=True, key=True, nonil=True), average)
        got = GdkAPI(gdk).quantile(gb, None, None, 0.7, True,
                                   gdk.BAT.from_numpy(gdk.TYPE_oid, cl, sorted_=True, key=True, nonil=True), average)
        assert _same(got[1], want[1])
    cl = np.sort(r.choice(n, 5000, replace=False)).astype(np.uint64)
    with pytest.raises(gdk.GDKError, match="does not match always"):
        gdk.BATgroupquantile(gb, _oids(gdk, gids[cl.astype(np.int64)], hseq=int(cl[0])), None, 0.5, True,
                             gdk.BAT.from_numpy(gdk.TYPE_oid, cl, sorted_=True, key=True, nonil=True))
