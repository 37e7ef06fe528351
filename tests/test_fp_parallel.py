"""The parallel form of order-dependent float folds (mgdk_set_fp_parallel_min).

The reference folds flt/dbl moments (AGGR_STDEV / AGGR_COVARIANCE /
AGGR_CORRELATION, gdk_aggr.c:4561-5013; calcvariance :4276), the running
mean of a float average (AVERAGE_ITER_FLOAT, gdk_calc_private.h:277) and a
running float SUM (frames 3 / 4, gdk_analytic_func.c:1959) one row after the
other; the device replays that order bit for bit, one lane per group or
partition.  A single group or partition of at least fp_parallel_min rows
takes a blocked, pairwise-combined form instead.  Its results differ from
the sequential ones by rounding only; the bounds asserted here are the ones
DESIGN.md states (u = 2^-53 for dbl, 2^-24 for a flt accumulator):

  running SUM, every row:  |par - seq| <= 2 n u sum|x|
  mean of one group:       |par - seq| <= 4 n u max|x|
  variance (and M2):       |par - seq| <= 4 n u sum(x^2) / (n - s)
  stdev:                   |par - seq| <= that / (2 stdev) + 2 ulp
  covariance:              |par - seq| <= 4 n u sqrt(sum x^2 sum y^2) / (n - s)
  correlation:             |par - seq| <= 8 n u (kx + ky + kxy)

(kx = sum x^2 / sum (x - mx)^2, kxy = sqrt(sum x^2 sum y^2) / |sum (x - mx)(y - my)|:
forward-error bounds of both evaluations, which each stay within half of
it of the exact value).  Below the threshold the device equals the oracle
bit for bit; the observed differences are printed."""
import math

import numpy as np
import pytest

from helpers import rng

U = 2.0 ** -53


@pytest.fixture
def par(gdk):
    prev = gdk.set_fp_parallel_min(1000)
    yield
    gdk.set_fp_parallel_min(prev)


def _vals(seed, n, nan_every=0):
    r = rng(seed)
    v = r.standard_normal(n) * 100.0 + 50.0
    if nan_every:
        v[::nan_every] = np.nan
    return v


@pytest.mark.gpu
def test_gpu_knob(gdk):
    prev = gdk.set_fp_parallel_min(12345)
    assert gdk.set_fp_parallel_min(prev) == 12345
    assert prev == 1 << 20


@pytest.mark.gpu
@pytest.mark.parametrize("sample", [False, True])
def test_gpu_moments_parallel(gdk, ora, par, sample):
    n = 300_000
    x = _vals(1801, n, nan_every=211)
    y = 0.5 * np.nan_to_num(x) + _vals(1802, n) * 0.3
    y[::307] = np.nan
    ok = ~(np.isnan(x) | np.isnan(y))
    X, Y = gdk.BAT.from_numpy(gdk.TYPE_dbl, x), gdk.BAT.from_numpy(gdk.TYPE_dbl, y)
    OX, OY = ora.Bat.from_array(ora.TYPE_dbl, x), ora.Bat.from_array(ora.TYPE_dbl, y)
    s = 1 if sample else 0
    xv = x[~np.isnan(x)]
    nx = len(xv)
    var_b = 4 * nx * U * float(np.sum(xv * xv)) / (nx - s)
    v, a = gdk.BATcalcvariance(X, sample)
    ov, oa = ora.BATcalcstat("variance", OX, None, sample)
    print("variance", v, ov, abs(v - ov) / math.ulp(ov), "ulp")
    assert abs(v - ov) <= var_b
    assert abs(a - oa) <= 4 * nx * U * float(np.max(np.abs(xv)))
    sd, _ = gdk.BATcalcvariance(X, sample, stdev=True)
    osd, _ = ora.BATcalcstat("stdev", OX, None, sample)
    assert abs(sd - osd) <= var_b / (2 * osd) + 2 * math.ulp(osd)
    # covariance / correlation skip a row where either value is nil
    xx, yy = x[ok], y[ok]
    m = len(xx)
    cov_b = 4 * m * U * math.sqrt(float(np.sum(xx * xx)) * float(np.sum(yy * yy))) / (m - s)
    c = gdk.BATcalccovariance(X, Y, sample)
    oc, _ = ora.BATcalcstat("covariance", OX, OY, sample)
    print("covariance", c, oc, abs(c - oc) / math.ulp(oc), "ulp")
    assert abs(c - oc) <= cov_b
    r = gdk.BATcalccorrelation(X, Y)
    orr, _ = ora.BATcalcstat("correlation", OX, OY)
    dx, dy = xx - xx.mean(), yy - yy.mean()
    kx = float(np.sum(xx * xx) / np.sum(dx * dx))
    ky = float(np.sum(yy * yy) / np.sum(dy * dy))
    kxy = math.sqrt(float(np.sum(xx * xx)) * float(np.sum(yy * yy))) / abs(float(np.sum(dx * dy)))
    print("correlation", r, orr, abs(r - orr) / math.ulp(orr), "ulp")
    assert abs(r - orr) <= 8 * m * U * (kx + ky + kxy)


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["int", "flt"])
def test_gpu_moments_parallel_types(gdk, ora, par, tname):
    r = rng(1803)
    n = 200_000
    if tname == "int":
        x = r.integers(-10**6, 10**6, n).astype(np.int32)
        x[::97] = -(1 << 31)
        xv = x[x != -(1 << 31)].astype(np.float64)
    else:
        x = (r.standard_normal(n) * 1e3).astype(np.float32)
        x[::97] = np.nan
        xv = x[~np.isnan(x)].astype(np.float64)
    tp = getattr(gdk, "TYPE_" + tname)
    v, _ = gdk.BATcalcvariance(gdk.BAT.from_numpy(tp, x), False)
    ov, _ = ora.BATcalcstat("variance", ora.Bat.from_array(getattr(ora, "TYPE_" + tname), x), None, False)
    assert abs(v - ov) <= 4 * len(xv) * U * float(np.sum(xv * xv)) / len(xv)


@pytest.mark.gpu
def test_gpu_moments_below_threshold_exact(gdk, ora):
    x = _vals(1804, 50_000, nan_every=101)
    prev = gdk.set_fp_parallel_min(None)
    try:
        v, a = gdk.BATcalcvariance(gdk.BAT.from_numpy(gdk.TYPE_dbl, x), True)
    finally:
        gdk.set_fp_parallel_min(prev)
    ov, oa = ora.BATcalcstat("variance", ora.Bat.from_array(ora.TYPE_dbl, x), None, True)
    assert v == ov and a == oa


@pytest.mark.gpu
def test_gpu_moments_overflow(gdk, par):
    x = np.full(5000, 1e300)
    x[::2] = -1e300
    with pytest.raises(gdk.GDKError, match="overflow in calculation"):
        gdk.BATcalcvariance(gdk.BAT.from_numpy(gdk.TYPE_dbl, x), False)


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["flt", "dbl"])
@pytest.mark.parametrize("skip", [True, False])
def test_gpu_groupavg_one_group_parallel(gdk, ora, par, tname, skip):
    n = 250_000
    x = _vals(1805, n, nan_every=0 if not skip else 401)
    if tname == "flt":
        x = x.astype(np.float32)
    g = np.zeros(n, np.uint64)
    g[::1000] = 1            # rows of another group id: outside the group range [0, 1)
    tp = getattr(gdk, "TYPE_" + tname)
    otp = getattr(ora, "TYPE_" + tname)
    e = gdk.BAT.dense(0, 1)
    a, c = gdk.BATgroupavg(gdk.BAT.from_numpy(tp, x), gdk.BAT.from_numpy(gdk.TYPE_oid, g), e, skip)
    oa, oc = ora.BATgroupavg(ora.Bat.from_array(otp, x), ora.Bat.from_array(ora.TYPE_oid, g), ora.Bat.dense(0, 1),
                             skip)
    got, want = a.to_numpy()[0], np.asarray(oa.values())[0]
    assert c.to_numpy()[0] == np.asarray(oc.values())[0]
    xs = x[(g == 0) & ~np.isnan(x)].astype(np.float64)
    print("avg", got, want, abs(got - want) / math.ulp(want), "ulp")
    assert abs(got - want) <= 4 * len(xs) * U * float(np.max(np.abs(xs)))
    if not skip:
        x2 = x.copy()
        x2[5] = np.nan
        a, c = gdk.BATgroupavg(gdk.BAT.from_numpy(tp, x2), gdk.BAT.from_numpy(gdk.TYPE_oid, g), e, False)
        assert np.isnan(a.to_numpy()[0]) and c.to_numpy()[0] == 0


def _peers(r, n, maxrun):
    o = np.zeros(n, np.int8)
    i = 0
    while i < n:
        o[i] = 1
        i += int(r.integers(1, maxrun + 1))
    return o


@pytest.mark.gpu
@pytest.mark.parametrize("frame", [3, 4])
@pytest.mark.parametrize("types", [("dbl", "dbl"), ("flt", "dbl"), ("flt", "flt")])
@pytest.mark.parametrize("maxrun", [1, 50, 9000, 0])
def test_gpu_running_sum_parallel(gdk, ora, par, frame, types, maxrun):
    r = rng(1806 + maxrun)
    n = 120_000
    x = r.standard_normal(n) * 10.0
    x[:37] = np.nan          # the running sum stays nil until the first value
    x[1000:1100] = np.nan
    t1, t2 = types
    if t1 == "flt":
        x = x.astype(np.float32)
    if maxrun:
        o = _peers(r, n, maxrun)
    else:
        o = np.zeros(n, np.int8)    # one peer group: every row gets the total
        o[0] = 1
    tp1, tp2 = getattr(gdk, "TYPE_" + t1), getattr(gdk, "TYPE_" + t2)
    got = gdk.GDKanalyticalsum(gdk.BAT.from_numpy(tp1, x), None, gdk.BAT.from_numpy(gdk.TYPE_bit, o), None, None,
                               tp2, frame).to_numpy().astype(np.float64)
    want = np.asarray(ora.analyticalsum(ora.Bat.from_array(getattr(ora, "TYPE_" + t1), x), None,
                                        ora.Bat.from_array(ora.TYPE_bit, o), None, None,
                                        getattr(ora, "TYPE_" + t2), frame).values()).astype(np.float64)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    u = 2.0 ** -24 if t2 == "flt" else U
    bound = 2 * n * u * float(np.nansum(np.abs(x.astype(np.float64))))
    d = np.nan_to_num(np.abs(got - want))
    print("running sum max diff", float(d.max()), "bound", bound)
    assert float(d.max()) <= bound


@pytest.mark.gpu
def test_gpu_running_sum_parallel_overflow(gdk, par):
    x = np.full(10_000, 1e308)
    o = np.ones(10_000, np.int8)
    with pytest.raises(gdk.GDKError, match="overflow"):
        gdk.GDKanalyticalsum(gdk.BAT.from_numpy(gdk.TYPE_dbl, x), None, gdk.BAT.from_numpy(gdk.TYPE_bit, o), None,
                             None, gdk.TYPE_dbl, 3)
