"""Windowed statistics and products: GDKanalytical_stddev_samp / _pop,
_variance_samp / _pop, _covariance_samp / _pop, _correlation
(gdk/gdk_analytic_statistics.c:689-1443) and GDKanalyticalprod
(gdk/gdk_analytic_func.c:2024-2560).

Pinning: the reference's analytics00 / 02 / 14 / 15.test answers (prod,
stddev_samp / _pop, var_samp / _pop, covar_samp / _pop, corr over PARTITION BY
/ ORDER BY / ROWS frames) are replayed through the oracle
(test_oracle.py::test_window_sqltests_oracle) and the device
(test_gpu_window_funcs.py::test_window_sqltests).  Here the device is
checked against the oracle bit for bit on random columns: every frame kind
(3, 4, 5, 6 and segment-tree frames from ROWS bounds), partitions of every
size, nils, every value type, and the overflow rules (an infinite
accumulator; an integer product past the result type, which depends on
whether a zero comes first)."""
import numpy as np
import pytest

from helpers import rng

I64N = -(1 << 63)
STATS = ["stddev_samp", "stddev_pop", "variance_samp", "variance_pop", "covariance_samp", "covariance_pop",
         "correlation"]
NPT = {"bte": np.int8, "sht": np.int16, "int": np.int32, "lng": np.int64, "flt": np.float32, "dbl": np.float64}
NILS = {"bte": -(1 << 7), "sht": -(1 << 15), "int": -(1 << 31), "lng": I64N}


def _vals(r, n, tname, nil_frac=0.08, lo=-1000, hi=1000):
    if tname in ("flt", "dbl"):
        v = r.normal(0.0, 50.0, n)
        v[r.random(n) < nil_frac] = np.nan
        return v.astype(NPT[tname])
    v = r.integers(lo, hi, n).astype(np.int64)
    v[r.random(n) < nil_frac] = I64N
    if tname == "hge":
        w = np.empty((n, 2), np.uint64)
        w[:, 0] = v.view(np.uint64)
        w[:, 1] = np.where(v < 0, np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64(0))
        w[v == I64N, 0] = 0
        w[v == I64N, 1] = np.uint64(1 << 63)
        return w
    return np.where(v == I64N, NILS[tname], v).astype(NPT[tname])


def _layout(r, n, nparts):
    """partition and peer bits (ORDER BY runs) and ROWS bounds of a random
    frame per query"""
    p = np.zeros(n, np.int8)
    if nparts > 1:
        p[np.sort(r.choice(np.arange(1, n), nparts - 1, replace=False))] = 1
    o = p.copy()
    o[0] = 1
    o[r.random(n) < 0.3] = 1
    return p, o


def _rows_bounds(p, before, after):
    n = len(p)
    starts = np.flatnonzero(np.r_[1, p[1:]])
    pid = np.cumsum(np.r_[1, p[1:]]) - 1
    ps = starts[pid]
    pe = np.r_[starts[1:], n][pid]
    i = np.arange(n)
    s = np.maximum(ps, i - before).astype(np.uint64)
    e = np.minimum(pe, i + after + 1).astype(np.uint64)
    return s, e


def _mk(mod, tp, a):
    if hasattr(mod, "Bat"):
        return mod.Bat.from_array(tp, a)
    return mod.BAT.from_numpy(tp, a)


def _same(g, w):
    g, w = np.asarray(g), np.asarray(w)
    if g.dtype.kind == "f":
        return bool(np.all((g == w) | (np.isnan(g) & np.isnan(w))))
    return np.array_equal(g, w)


def _frames(r, n, p):
    yield 3, None, None
    yield 4, None, None
    yield 5, None, None
    yield 6, None, None
    for before, after in ((5, 0), (2, 2), (40, 3), (300, 700)):
        s, e = _rows_bounds(p, before, after)
        yield 0, s, e


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["bte", "sht", "int", "lng", "hge", "flt", "dbl"])
@pytest.mark.parametrize("nparts", [1, 7, 900])
def test_gpu_window_stats(gdk, ora, tname, nparts):
    r = rng(1501 + nparts)
    n = 20_000
    x, y = _vals(r, n, tname), _vals(r, n, tname)
    p, o = _layout(r, n, nparts)
    tp_g, tp_o = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
    gx, gy, ox, oy = _mk(gdk, tp_g, x), _mk(gdk, tp_g, y), _mk(ora, tp_o, x), _mk(ora, tp_o, y)
    gp, op_ = (_mk(gdk, gdk.TYPE_bit, p), _mk(ora, ora.TYPE_bit, p)) if nparts > 1 else (None, None)
    go, oo = _mk(gdk, gdk.TYPE_bit, o), _mk(ora, ora.TYPE_bit, o)
    for ft, s, e in _frames(r, n, p):
        gs = ge = os_ = oe = None
        if s is not None:
            gs, ge = _mk(gdk, gdk.TYPE_oid, s), _mk(gdk, gdk.TYPE_oid, e)
            os_, oe = _mk(ora, ora.TYPE_oid, s), _mk(ora, ora.TYPE_oid, e)
        for name in STATS:
            two = name.startswith("cov") or name == "correlation"
            want = ora.analyticalstat(name, ox, oy if two else None, op_, oo, os_, oe, ft)
            got = gdk.GDKanalytical_stat(name, gx, gy if two else None, gp, go, gs, ge, ft)
            assert _same(got.to_numpy(), want.values()), (name, ft)
            assert bool(got.s.tnil) == bool(want.s.nil), (name, ft)


PROD_TYPES = [("bte", "bte"), ("bte", "sht"), ("sht", "int"), ("int", "lng"), ("lng", "lng"), ("int", "hge"),
              ("lng", "hge"), ("flt", "flt"), ("flt", "dbl"), ("dbl", "dbl")]


@pytest.mark.gpu
@pytest.mark.parametrize("t1,t2", PROD_TYPES)
@pytest.mark.parametrize("nparts", [1, 50, 3000])
def test_gpu_window_prod(gdk, ora, t1, t2, nparts):
    r = rng(1502 + nparts)
    n = 12_000
    # small magnitudes (mostly +-1, 2) so that long frames stay in range
    if t1 in ("flt", "dbl"):
        v = r.choice([-1.5, -1.0, -0.5, 0.5, 1.0, 1.25, 2.0], n)
        v[r.random(n) < 0.05] = np.nan
        x = v.astype(NPT[t1])
    else:
        v = r.choice([-1, 1, 1, -1, 2, -2, 1, 3], n).astype(np.int64)
        v[r.random(n) < 0.05] = I64N
        x = np.where(v == I64N, NILS[t1], v).astype(NPT[t1])
    p, o = _layout(r, n, nparts)
    tg1, to1 = getattr(gdk, "TYPE_" + t1), getattr(ora, "TYPE_" + t1)
    tg2, to2 = getattr(gdk, "TYPE_" + t2), getattr(ora, "TYPE_" + t2)
    gx, ox = _mk(gdk, tg1, x), _mk(ora, to1, x)
    gp, op_ = (_mk(gdk, gdk.TYPE_bit, p), _mk(ora, ora.TYPE_bit, p)) if nparts > 1 else (None, None)
    go, oo = _mk(gdk, gdk.TYPE_bit, o), _mk(ora, ora.TYPE_bit, o)
    for ft, s, e in _frames(r, n, p):
        gs = ge = os_ = oe = None
        if s is not None:
            gs, ge = _mk(gdk, gdk.TYPE_oid, s), _mk(gdk, gdk.TYPE_oid, e)
            os_, oe = _mk(ora, ora.TYPE_oid, s), _mk(ora, ora.TYPE_oid, e)
        try:
            want = ora.analyticalprod(ox, op_, oo, os_, oe, to2, ft)
        except Exception as ex:                       # noqa: BLE001
            assert "overflow" in str(ex)
            with pytest.raises(gdk.GDKError, match="overflow"):
                gdk.GDKanalyticalprod(gx, gp, go, gs, ge, tg2, ft)
            continue
        got = gdk.GDKanalyticalprod(gx, gp, go, gs, ge, tg2, ft)
        if t2 == "hge":
            assert got.values() == want.values(), ft
        else:
            assert _same(got.to_numpy(), want.values()), ft


@pytest.mark.gpu
def test_gpu_window_overflow(gdk, ora):
    """overflow: a zero before a huge run hides it in running frames but not
    in the segment tree; an infinite variance accumulator is an error"""
    n = 64
    x = np.full(n, 1 << 20, np.int64)
    x[0] = 0
    gx, ox = _mk(gdk, gdk.TYPE_lng, x), _mk(ora, ora.TYPE_lng, x)
    o = np.ones(n, np.int8)
    go, oo = _mk(gdk, gdk.TYPE_bit, o), _mk(ora, ora.TYPE_bit, o)
    for ft in (3, 4, 5):
        try:
            want = ora.analyticalprod(ox, None, oo, None, None, ora.TYPE_lng, ft).values()
            got = gdk.GDKanalyticalprod(gx, None, go, None, None, gdk.TYPE_lng, ft).to_numpy()
            assert _same(got, want), ft
        except Exception as ex:                       # noqa: BLE001
            assert "overflow" in str(ex)
            with pytest.raises(gdk.GDKError, match="overflow"):
                gdk.GDKanalyticalprod(gx, None, go, None, None, gdk.TYPE_lng, ft)
    s, e = _rows_bounds(np.zeros(n, np.int8), 2, 0)
    with pytest.raises(Exception, match="overflow"):
        ora.analyticalprod(ox, None, oo, _mk(ora, ora.TYPE_oid, s), _mk(ora, ora.TYPE_oid, e), ora.TYPE_lng, 0)
    with pytest.raises(gdk.GDKError, match="overflow"):
        gdk.GDKanalyticalprod(gx, None, go, _mk(gdk, gdk.TYPE_oid, s), _mk(gdk, gdk.TYPE_oid, e), gdk.TYPE_lng, 0)
    big = np.array([1e300, -1e300] * 8)
    with pytest.raises(gdk.GDKError, match="overflow"):
        gdk.GDKanalytical_stat("variance_pop", _mk(gdk, gdk.TYPE_dbl, big), None, None, None, None, None, 5)
    with pytest.raises(Exception, match="overflow"):
        ora.analyticalstat("variance_pop", _mk(ora, ora.TYPE_dbl, big), None, None, None, None, None, 5)


def test_oracle_window_stats_small(ora):
    """the oracle's running frames against a direct restatement on a tiny
    column (Python floats: the same IEEE operations in the same order)"""
    import math
    x = [3.0, None, 5.0, 8.0, 8.0, None, 1.0]
    a = np.array([np.nan if v is None else v for v in x])
    b = ora.Bat.from_array(ora.TYPE_dbl, a)
    o = ora.Bat.from_array(ora.TYPE_bit, np.array([1, 0, 1, 1, 0, 1, 1], np.int8))
    got = ora.analyticalstat("stddev_samp", b, None, None, o, None, None, 3).values()
    n = mean = m2 = 0.0
    want = []
    groups = [[0, 1], [2], [3, 4], [5], [6]]
    for g in groups:
        for i in g:
            if x[i] is None:
                continue
            n += 1
            d = x[i] - mean
            mean += d / n
            m2 += d * (x[i] - mean)
        v = math.sqrt(m2 / (n - 1)) if n > 1 else math.nan
        want += [v] * len(g)
    assert _same(got, want)
