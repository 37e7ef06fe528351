"""Windowed SUM / COUNT over frames (GDKanalyticalsum / GDKanalyticalcount,
gdk/gdk_analytic_func.c:1959 / :1626) against the oracle restatement, with
frames from GDKanalyticalwindowbounds (the RANGE bounds of §8 a10)."""
import numpy as np
import pytest

from helpers import rng

pytestmark = pytest.mark.gpu

NIL64 = np.iinfo(np.int64).min


def _data(r, nparts=23, plen=517, nil_frac=0.05, tname="lng", lo=-10**6, hi=10**6):
    dt = {"int": np.int32, "lng": np.int64, "sht": np.int16}[tname]
    vals, bits, order = [], [], []
    for _ in range(nparts):
        n = int(r.integers(1, 2 * plen))
        ob = np.sort(r.integers(0, n // 3 + 1, n))               # ORDER BY values -> peers
        v = r.integers(lo, hi, n).astype(dt)
        v[r.random(n) < nil_frac] = np.iinfo(dt).min
        vals.append(v)
        b = np.zeros(n, np.int8)
        b[0] = 1
        bits.append(b)
        order.append(ob)
    v = np.concatenate(vals)
    p = np.concatenate(bits)
    ob = np.concatenate(order).astype(np.int64)
    o = np.ones(len(v), np.int8)
    o[1:] = (ob[1:] != ob[:-1]) | (p[1:] != 0)
    return v, p, o, ob


def _bounds(gdk, ob, p, limit):
    OB = gdk.BAT.from_numpy(gdk.TYPE_lng, ob)
    P = gdk.BAT.from_numpy(gdk.TYPE_bit, p)
    s = gdk.GDKanalyticalwindowbounds(OB, P, limit, True)
    e = gdk.GDKanalyticalwindowbounds(OB, P, limit, False)
    return s, e


@pytest.mark.parametrize("tname", ["int", "lng"])
@pytest.mark.parametrize("tp2", ["lng", "hge"])
@pytest.mark.parametrize("frame", [3, 4, 5, 6, 1])
def test_analytical_sum(gdk, ora, tname, tp2, frame):
    r = rng(301)
    v, p, o, ob = _data(r, tname=tname)
    tp1 = getattr(gdk, "TYPE_" + tname)
    T2 = getattr(gdk, "TYPE_" + tp2)
    s = e = None
    if frame == 1:
        s, e = _bounds(gdk, ob, p, 3)
    got = gdk.GDKanalyticalsum(gdk.BAT.from_numpy(tp1, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                               gdk.BAT.from_numpy(gdk.TYPE_bit, o), s, e, T2, frame)
    os_ = ora.Bat.from_array(ora.TYPE_oid, s.to_numpy()) if s else None
    oe = ora.Bat.from_array(ora.TYPE_oid, e.to_numpy()) if e else None
    want = ora.analyticalsum(ora.Bat.from_array(tp1, v), ora.Bat.from_array(ora.TYPE_bit, p),
                             ora.Bat.from_array(ora.TYPE_bit, o), os_, oe, T2, frame)
    g = got.values()
    w = want.values()
    assert list(g) == list(w)


@pytest.mark.parametrize("ignore_nils", [True, False])
@pytest.mark.parametrize("frame", [3, 4, 5, 6, 1])
def test_analytical_count(gdk, ora, ignore_nils, frame):
    r = rng(302)
    v, p, o, ob = _data(r)
    s = e = None
    if frame == 1:
        s, e = _bounds(gdk, ob, p, 5)
    got = gdk.GDKanalyticalcount(gdk.BAT.from_numpy(gdk.TYPE_lng, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                                 gdk.BAT.from_numpy(gdk.TYPE_bit, o), s, e, ignore_nils, frame)
    os_ = ora.Bat.from_array(ora.TYPE_oid, s.to_numpy()) if s else None
    oe = ora.Bat.from_array(ora.TYPE_oid, e.to_numpy()) if e else None
    want = ora.analyticalcount(ora.Bat.from_array(ora.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_bit, p),
                               ora.Bat.from_array(ora.TYPE_bit, o), os_, oe, ignore_nils, frame)
    assert np.array_equal(got.to_numpy(), want.values())


@pytest.mark.parametrize("frame", [3, 4, 5])
def test_analytical_sum_lng_overflow(gdk, ora, frame):
    # running partials overflow lng in one partition: the reference's error
    v = np.array([2**62, 2**62, 5, 7, 2**62, -(2**62), 1], np.int64)
    p = np.array([0, 0, 0, 1, 1, 0, 0], np.int8)
    o = np.ones(7, np.int8)
    args = (gdk.BAT.from_numpy(gdk.TYPE_lng, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
            gdk.BAT.from_numpy(gdk.TYPE_bit, o), None, None)
    with pytest.raises(ora.OracleError, match="22003!overflow in calculation"):
        ora.analyticalsum(ora.Bat.from_array(ora.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_bit, p),
                          ora.Bat.from_array(ora.TYPE_bit, o), None, None, ora.TYPE_lng, frame)
    with pytest.raises(gdk.GDKError, match="22003!overflow in calculation"):
        gdk.GDKanalyticalsum(*args, gdk.TYPE_lng, frame)
    # the same sums in hge are exact
    got = gdk.GDKanalyticalsum(*args, gdk.TYPE_hge, frame).values()
    want = ora.analyticalsum(ora.Bat.from_array(ora.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_bit, p),
                             ora.Bat.from_array(ora.TYPE_bit, o), None, None, ora.TYPE_hge, frame).values()
    assert list(got) == list(want)


def test_analytical_sum_frames_large_magnitude(gdk):
    # |values| summing past lng in a partition: lng frame sums depend on the
    # reference's segment-tree order -> refused loudly, hge is exact
    v = np.array([2**62, -(2**62), 2**62, -(2**62), 3], np.int64)
    V = gdk.BAT.from_numpy(gdk.TYPE_lng, v)
    s = gdk.BAT.from_numpy(gdk.TYPE_oid, np.array([0, 0, 1, 2, 3], np.uint64))
    e = gdk.BAT.from_numpy(gdk.TYPE_oid, np.array([1, 2, 3, 4, 5], np.uint64))
    with pytest.raises(gdk.GDKError, match="not supported on the device path"):
        gdk.GDKanalyticalsum(V, None, None, s, e, gdk.TYPE_lng, 1)
    got = gdk.GDKanalyticalsum(V, None, None, s, e, gdk.TYPE_hge, 1).values()
    assert list(got) == [2**62, 0, 0, 0, -(2**62) + 3]


def test_analytical_sum_large(gdk, ora):
    # multi-tile prefix scan (several 2048-row tiles and a ragged tail)
    r = rng(303)
    v, p, o, ob = _data(r, nparts=60, plen=3000)
    got = gdk.GDKanalyticalsum(gdk.BAT.from_numpy(gdk.TYPE_lng, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                               gdk.BAT.from_numpy(gdk.TYPE_bit, o), None, None, gdk.TYPE_hge, 3).values()
    want = ora.analyticalsum(ora.Bat.from_array(ora.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_bit, p),
                             ora.Bat.from_array(ora.TYPE_bit, o), None, None, ora.TYPE_hge, 3).values()
    assert list(got) == list(want)


def test_window_frames_sqltest(gdk):
    """analytics03.test (the reference's own answers): windowed SUM / COUNT
    over RANGE frames closed at the current row's peers, and whole partitions."""
    from helpers import replay_window_frames
    bad = replay_window_frames(
        lambda b, p, o, tp2, f: gdk.GDKanalyticalsum(b, p, o, None, None, tp2, f).to_numpy(),
        lambda b, p, o, ign, f: gdk.GDKanalyticalcount(b, p, o, None, None, ign, f).to_numpy(),
        lambda tp, a: gdk.BAT.from_numpy(tp, a), gdk.TYPE_int, gdk.TYPE_bit, gdk.TYPE_lng)
    assert not bad, bad


@pytest.mark.parametrize("limit", [0, 40, 3000, 10**9])
@pytest.mark.parametrize("tname", ["int", "lng"])
def test_analytical_sum_general_frames_hge(gdk, ora, limit, tname):
    """RANGE frames [s, e) into hge: short frames take the fused tile kernel
    (values staged in LDS), frames longer than a tile's window fall back to
    the global prefix path; both equal the oracle, nils included."""
    r = rng(304)
    v, p, o, ob = _data(r, nparts=40, plen=4000, tname=tname)
    s, e = _bounds(gdk, ob, p, limit)
    tp1 = getattr(gdk, "TYPE_" + tname)
    got = gdk.GDKanalyticalsum(gdk.BAT.from_numpy(tp1, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p), None, s, e,
                               gdk.TYPE_hge, 1).values()
    want = ora.analyticalsum(ora.Bat.from_array(tp1, v), ora.Bat.from_array(ora.TYPE_bit, p), None,
                             ora.Bat.from_array(ora.TYPE_oid, s.to_numpy()),
                             ora.Bat.from_array(ora.TYPE_oid, e.to_numpy()), ora.TYPE_hge, 1).values()
    assert list(got) == list(want)


def _avg_input(r, tname, n):
    if tname in ("flt", "dbl"):
        v = (r.standard_normal(n) * 10.0 ** r.integers(-2, 5, n)).astype(np.float32 if tname == "flt" else np.float64)
        v[r.random(n) < 0.05] = np.nan
        return v
    dt = {"bte": np.int8, "sht": np.int16, "int": np.int32, "lng": np.int64}[tname]
    info = np.iinfo(dt)
    v = r.integers(info.min + 1, info.max, n, dtype=np.int64).astype(dt)
    v[r.random(n) < 0.05] = info.min
    return v


@pytest.mark.parametrize("tname", ["bte", "sht", "int", "lng", "flt", "dbl"])
@pytest.mark.parametrize("frame", [3, 4, 5, 6, 1])
def test_analytical_avg(gdk, ora, tname, frame):
    """GDKanalyticalavg (gdk_analytic_statistics.c:364) bit-exact against the
    oracle: exact integer running frames, AVERAGE_ITER_FLOAT replay for
    flt/dbl, and the reference's segment tree (averages of child averages)
    for general frames."""
    r = rng(311)
    _, p, o, ob = _data(r, nparts=31, plen=900)
    n = len(p)
    v = _avg_input(r, tname, n)
    tp = getattr(gdk, "TYPE_" + tname)
    s = e = None
    if frame == 1:
        s, e = _bounds(gdk, ob, p, 40)
    got = gdk.GDKanalyticalavg(gdk.BAT.from_numpy(tp, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                               gdk.BAT.from_numpy(gdk.TYPE_bit, o), s, e, frame)
    os_ = ora.Bat.from_array(ora.TYPE_oid, s.to_numpy()) if s else None
    oe = ora.Bat.from_array(ora.TYPE_oid, e.to_numpy()) if e else None
    want = ora.analyticalavg(ora.Bat.from_array(tp, v), ora.Bat.from_array(ora.TYPE_bit, p),
                             ora.Bat.from_array(ora.TYPE_bit, o), os_, oe, frame)
    assert np.asarray(got.values()).tobytes() == np.asarray(want.values()).tobytes()
    assert bool(got.s.tnil) == bool(np.isnan(np.asarray(want.values())).any())


@pytest.mark.parametrize("tname", ["int", "lng", "dbl"])
def test_analytical_avg_deep_trees(gdk, ora, tname):
    """General frames over long partitions (4-level trees, frames up to the
    whole partition) and a single partition without p."""
    r = rng(312)
    n = 150_000
    tp = getattr(gdk, "TYPE_" + tname)
    v = _avg_input(r, tname, n)
    for parts in (True, False):
        p = np.zeros(n, np.int8)
        p[0] = 1
        if parts:
            p[r.choice(n, 3, replace=False)] = 1
        starts = np.flatnonzero(p)
        ends = np.append(starts[1:], n)
        pid = np.cumsum(p) - 1
        i = np.arange(n)
        s = np.maximum(starts[pid], i - r.integers(0, 70_000, n)).astype(np.uint64)
        e = np.minimum(ends[pid], i + 1 + r.integers(0, 70_000, n)).astype(np.uint64)
        P = gdk.BAT.from_numpy(gdk.TYPE_bit, p) if parts else None
        OP = ora.Bat.from_array(ora.TYPE_bit, p) if parts else None
        got = gdk.GDKanalyticalavg(gdk.BAT.from_numpy(tp, v), P, None, gdk.BAT.from_numpy(gdk.TYPE_oid, s),
                                   gdk.BAT.from_numpy(gdk.TYPE_oid, e), 1)
        want = ora.analyticalavg(ora.Bat.from_array(tp, v), OP, None, ora.Bat.from_array(ora.TYPE_oid, s),
                                 ora.Bat.from_array(ora.TYPE_oid, e), 1)
        assert np.asarray(got.values()).tobytes() == np.asarray(want.values()).tobytes()


def test_window_avg_sqltest(gdk):
    """analytics03.test's windowed AVG answers on the device."""
    from helpers import replay_window_avg
    bad = replay_window_avg(
        lambda b, p, o, f: gdk.GDKanalyticalavg(b, p, o, None, None, f).values(),
        lambda tp, a: gdk.BAT.from_numpy(tp, np.asarray(a)), gdk.TYPE_int, gdk.TYPE_flt, gdk.TYPE_bit)
    assert not bad, bad


def test_analytical_avg_edges(gdk):
    """empty input; hge refused loudly; a frame with only nils is nil."""
    E = gdk.BAT.from_numpy(gdk.TYPE_lng, np.zeros(0, np.int64))
    assert gdk.GDKanalyticalavg(E, None, None, None, None, 5).count() == 0
    H = gdk.BAT.from_numpy(gdk.TYPE_hge, np.zeros(8, np.uint64))
    with pytest.raises(gdk.GDKError, match="not supported on the device path"):
        gdk.GDKanalyticalavg(H, None, None, None, None, 5)
    v = np.array([NIL64, NIL64, 4, NIL64], np.int64)
    s = gdk.BAT.from_numpy(gdk.TYPE_oid, np.array([0, 0, 1, 3], np.uint64))
    e = gdk.BAT.from_numpy(gdk.TYPE_oid, np.array([1, 2, 3, 4], np.uint64))
    got = gdk.GDKanalyticalavg(gdk.BAT.from_numpy(gdk.TYPE_lng, v), None, None, s, e, 1).values()
    assert np.isnan(got[0]) and np.isnan(got[1]) and got[2] == 4.0 and np.isnan(got[3])


@pytest.mark.parametrize("tname", ["bte", "sht", "int", "lng"])
@pytest.mark.parametrize("frame", [3, 4, 5, 6, 1])
def test_analytical_avginteger(gdk, ora, tname, frame):
    """GDKanalyticalavginteger (gdk_analytic_statistics.c:631) bit-exact
    against the oracle's AVERAGE_ITER replay: rounded exact averages over
    the running frames, the segment tree's state over general frames."""
    r = rng(313)
    _, p, o, ob = _data(r, nparts=31, plen=900)
    n = len(p)
    v = _avg_input(r, tname, n)
    tp = getattr(gdk, "TYPE_" + tname)
    s = e = None
    if frame == 1:
        s, e = _bounds(gdk, ob, p, 40)
    got = gdk.GDKanalyticalavginteger(gdk.BAT.from_numpy(tp, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                                      gdk.BAT.from_numpy(gdk.TYPE_bit, o), s, e, frame)
    os_ = ora.Bat.from_array(ora.TYPE_oid, s.to_numpy()) if s else None
    oe = ora.Bat.from_array(ora.TYPE_oid, e.to_numpy()) if e else None
    want = ora.analyticalavginteger(ora.Bat.from_array(tp, v), ora.Bat.from_array(ora.TYPE_bit, p),
                                    ora.Bat.from_array(ora.TYPE_bit, o), os_, oe, frame)
    assert np.array_equal(got.to_numpy(), np.asarray(want.values()))
    assert bool(got.s.tnil) == bool(want.s.nil)


def test_analytical_avginteger_deep_tree(gdk, ora):
    r = rng(314)
    n = 120_000
    v = _avg_input(r, "lng", n)
    i = np.arange(n)
    s = np.maximum(0, i - r.integers(0, 60_000, n)).astype(np.uint64)
    e = np.minimum(n, i + 1 + r.integers(0, 60_000, n)).astype(np.uint64)
    got = gdk.GDKanalyticalavginteger(gdk.BAT.from_numpy(gdk.TYPE_lng, v), None, None,
                                      gdk.BAT.from_numpy(gdk.TYPE_oid, s), gdk.BAT.from_numpy(gdk.TYPE_oid, e), 1)
    want = ora.analyticalavginteger(ora.Bat.from_array(ora.TYPE_lng, v), None, None,
                                    ora.Bat.from_array(ora.TYPE_oid, s), ora.Bat.from_array(ora.TYPE_oid, e), 1)
    assert np.array_equal(got.to_numpy(), np.asarray(want.values()))


def _fdata(r, tname, nparts=23, plen=517, nil_frac=0.05):
    dt = np.float32 if tname == "flt" else np.float64
    v, p, o, ob = _data(r, nparts=nparts, plen=plen, nil_frac=0.0)
    x = (r.standard_normal(len(v)) * 10.0 ** r.integers(-3, 6, len(v))).astype(dt)
    x[r.random(len(v)) < nil_frac] = np.nan
    return x, p, o, ob


@pytest.mark.parametrize("t1,t2", [("flt", "flt"), ("flt", "dbl"), ("dbl", "dbl")])
@pytest.mark.parametrize("frame", [3, 4, 5, 6, 1, 2])
def test_analytical_sum_float(gdk, ora, t1, t2, frame):
    """GDKanalyticalsum over flt / dbl: frames 3 / 4 add in row order, frame 5
    is the partition's dofsum, frames from the bounds walk the reference's
    segment tree -- all bit-identical to the oracle's restatement."""
    r = rng(311 + frame)
    v, p, o, ob = _fdata(r, t1)
    tp1, T2 = getattr(gdk, "TYPE_" + t1), getattr(gdk, "TYPE_" + t2)
    s = e = None
    if frame in (1, 2):
        s, e = _bounds(gdk, ob, p, 3 if frame == 1 else 40)
    got = gdk.GDKanalyticalsum(gdk.BAT.from_numpy(tp1, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                               gdk.BAT.from_numpy(gdk.TYPE_bit, o), s, e, T2, frame)
    os_ = ora.Bat.from_array(ora.TYPE_oid, s.to_numpy()) if s else None
    oe = ora.Bat.from_array(ora.TYPE_oid, e.to_numpy()) if e else None
    want = ora.analyticalsum(ora.Bat.from_array(tp1, v), ora.Bat.from_array(ora.TYPE_bit, p),
                             ora.Bat.from_array(ora.TYPE_bit, o), os_, oe, T2, frame)
    g, w = got.to_numpy(), want.values()
    assert g.dtype == w.dtype
    assert np.array_equal(g.view(np.uint32 if g.dtype == np.float32 else np.uint64),
                          w.view(np.uint32 if w.dtype == np.float32 else np.uint64))
    assert bool(got.s.tnil) == bool(want.s.nil)


@pytest.mark.parametrize("frame", [3, 4, 5, 1])
def test_analytical_sum_float_overflow(gdk, ora, frame):
    r = rng(5)
    v, p, o, ob = _fdata(r, "flt", nparts=3, plen=40, nil_frac=0.0)
    v[5:9] = 3e38
    s = e = None
    if frame == 1:
        s, e = _bounds(gdk, ob, p, 10)
    os_ = ora.Bat.from_array(ora.TYPE_oid, s.to_numpy()) if s else None
    oe = ora.Bat.from_array(ora.TYPE_oid, e.to_numpy()) if e else None
    with pytest.raises(ora.OracleError) as we:
        ora.analyticalsum(ora.Bat.from_array(ora.TYPE_flt, v), ora.Bat.from_array(ora.TYPE_bit, p),
                          ora.Bat.from_array(ora.TYPE_bit, o), os_, oe, ora.TYPE_flt, frame)
    with pytest.raises(gdk.GDKError) as ge:
        gdk.GDKanalyticalsum(gdk.BAT.from_numpy(gdk.TYPE_flt, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                             gdk.BAT.from_numpy(gdk.TYPE_bit, o), s, e, gdk.TYPE_flt, frame)
    assert str(ge.value) == str(we.value)
