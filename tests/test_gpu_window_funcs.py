"""Window functions beyond the frame aggregates -- GDKanalyticalntile,
first, last, nth_value, lag, lead, min and max (gdk_analytic_func.c:124,
:230, :312, :421, :671, :823, :1264) -- on the device against the oracle's
restatement (oracle/gdk_oracle_window.c) on the same inputs: partitions,
peer groups, ROWS / RANGE frames from GDKanalyticalwindowbounds on both
sides, nils, every fixed-width type, all frame kinds of min / max, nil
arguments and the reference's errors.  Results and nil properties are
compared; flt / dbl compare with == (a general frame whose extreme is both
-0.0 and +0.0 may differ in the zero's sign)."""
import numpy as np
import pytest

from helpers import rng

TYPES = [("bte", np.int8), ("sht", np.int16), ("int", np.int32), ("lng", np.int64), ("flt", np.float32),
         ("dbl", np.float64), ("hge", None), ("date", np.int32)]


def _vals(r, tname, dt, n, nils=0.05):
    if tname == "hge":
        v = [int(x) * (1 << 70) + 3 for x in r.integers(-1000, 1000, n)]
        for i in np.flatnonzero(r.random(n) < nils):
            v[i] = -(1 << 127)
        return v
    if dt in (np.float32, np.float64):
        v = (r.integers(-1000, 1000, n) / 8).astype(dt)
        v[r.random(n) < nils] = np.nan
        return v
    info = np.iinfo(dt)
    v = r.integers(max(info.min + 1, -1000), min(info.max, 1000), n).astype(dt)
    v[r.random(n) < nils] = info.min
    return v


def _pair(gdk, ora, tname, v, hseq=0):
    if tname == "hge":
        words = np.array([gdk.int_to_hge_words(x) for x in v], np.uint64)
        return (gdk.BAT.from_numpy(gdk.TYPE_hge, words, hseqbase=hseq),
                ora.Bat.from_array(ora.TYPE_hge, words, hseqbase=hseq))
    tg, to = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
    return gdk.BAT.from_numpy(tg, v, hseqbase=hseq), ora.Bat.from_array(to, v, hseqbase=hseq)


def _bits(gdk, ora, f):
    f = np.asarray(f, np.int8)
    return gdk.BAT.from_numpy(gdk.TYPE_bit, f), ora.Bat.from_array(ora.TYPE_bit, f)


def _same(got, want, tname):
    g, w = got.values(), want.values()
    if tname == "hge":
        assert list(g) == list(w)
    elif tname in ("flt", "dbl"):
        g, w = np.asarray(g), np.asarray(w)
        assert np.array_equal(np.isnan(g), np.isnan(w))
        assert np.array_equal(g[~np.isnan(g)], w[~np.isnan(w)])
    else:
        assert np.array_equal(np.asarray(g), np.asarray(w))
    assert bool(got.s.tnil) == bool(want.s.nil) and bool(got.s.tnonil) == bool(want.s.nonil)


def _layout(r, n, kind):
    """partition and peer-start bits (p[0] = 0 as the reference's plans)"""
    if kind == "one":
        p = np.zeros(n, np.int8)
    elif kind == "small":
        p = (r.random(n) < 0.2).astype(np.int8)
    else:
        p = (r.random(n) < 0.002).astype(np.int8)
    p[0] = 0
    o = np.maximum(p, (r.random(n) < 0.4).astype(np.int8))
    o[0] = 0
    return p, o


def _rows_bounds(gdk, ora, n, p_g, p_o, lo, hi):
    """ROWS BETWEEN lo PRECEDING AND hi FOLLOWING on both sides"""
    col = np.arange(n, dtype=np.int64)
    bg, bo = gdk.BAT.from_numpy(gdk.TYPE_lng, col), ora.Bat.from_array(ora.TYPE_lng, col)
    s = gdk.GDKanalyticalwindowbounds(bg, p_g, lo, True, tp2=gdk.TYPE_lng, unit=0)
    e = gdk.GDKanalyticalwindowbounds(bg, p_g, hi, False, tp2=gdk.TYPE_lng, unit=0)
    os_ = ora.windowbounds(bo, p_o, None, lo, ora.TYPE_lng, ora.TYPE_lng, 0, True)
    oe = ora.windowbounds(bo, p_o, None, hi, ora.TYPE_lng, ora.TYPE_lng, 0, False)
    return s, e, os_, oe


@pytest.mark.gpu
@pytest.mark.parametrize("tname,dt", TYPES)
@pytest.mark.parametrize("layout", ["one", "small", "large"])
def test_lag_lead(gdk, ora, tname, dt, layout):
    r = rng(len(tname) * 31 + len(layout))
    n = 40_003
    v = _vals(r, tname, dt, n)
    b, ob = _pair(gdk, ora, tname, v)
    pf, _ = _layout(r, n, layout)
    p, op = _bits(gdk, ora, pf)
    dflt = 7 if tname != "hge" else 5 << 80
    for off in (0, 1, 3, 1000):
        _same(gdk.GDKanalyticallag(b, p, off, dflt), ora.analyticallag(ob, op, off, dflt), tname)
        _same(gdk.GDKanalyticallead(b, p, off, dflt), ora.analyticallead(ob, op, off, dflt), tname)
    nil = gdk.NIL[getattr(gdk, "TYPE_" + tname)]
    _same(gdk.GDKanalyticallag(b, None, 2, nil), ora.analyticallag(ob, None, 2, nil), tname)
    _same(gdk.GDKanalyticallead(b, p, gdk.BUN_NONE, dflt), ora.analyticallead(ob, op, ora.BUN_NONE, dflt), tname)


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["bte", "sht", "int", "lng", "hge"])
@pytest.mark.parametrize("layout", ["one", "small", "large"])
def test_ntile(gdk, ora, tname, layout):
    r = rng(len(tname) + 7 * len(layout))
    n = 30_011
    pf, _ = _layout(r, n, layout)
    p, op = _bits(gdk, ora, pf)
    b, ob = _pair(gdk, ora, "int", np.zeros(n, np.int32))
    tg, to = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
    for k in (1, 3, 7, 100, 120 if tname == "bte" else 30_000):
        _same(gdk.GDKanalyticalntile(b, p, ntile=k, tpe=tg), ora.analyticalntile(ob, op, ntile=k, tpe=to), tname)
    # per-row n with nils
    if tname == "hge":
        nv = [int(x) for x in r.integers(1, 20, n)]
        nv[5] = -(1 << 127)
    else:
        dt = {"bte": np.int8, "sht": np.int16, "int": np.int32, "lng": np.int64}[tname]
        nv = r.integers(1, 20, n).astype(dt)
        nv[5] = np.iinfo(dt).min
    nb, onb = _pair(gdk, ora, tname, nv)
    _same(gdk.GDKanalyticalntile(b, p, n=nb), ora.analyticalntile(ob, op, n=onb), tname)
    with pytest.raises(gdk.GDKError, match="ntile must be greater than zero"):
        gdk.GDKanalyticalntile(b, p, ntile=0, tpe=tg)


@pytest.mark.gpu
@pytest.mark.parametrize("tname,dt", TYPES)
def test_first_last_nth(gdk, ora, tname, dt):
    r = rng(len(tname) * 3)
    n = 50_021
    v = _vals(r, tname, dt, n)
    b, ob = _pair(gdk, ora, tname, v)
    pf, _ = _layout(r, n, "small")
    p, op = _bits(gdk, ora, pf)
    for lo, hi in ((0, 0), (3, 2), (100, 0), (0, 50)):
        s, e, os_, oe = _rows_bounds(gdk, ora, n, p, op, lo, hi)
        _same(gdk.GDKanalyticalfirst(b, s, e), ora.analyticalfirst(ob, os_, oe), tname)
        _same(gdk.GDKanalyticallast(b, s, e), ora.analyticallast(ob, os_, oe), tname)
        for nth in (1, 2, 5, -(1 << 63)):
            _same(gdk.GDKanalyticalnthvalue(b, s, e, nth=nth), ora.analyticalnthvalue(ob, os_, oe, nth=nth), tname)
        t = r.integers(1, 8, n).astype(np.int64)
        t[::97] = np.iinfo(np.int64).min
        tb, otb = gdk.BAT.from_numpy(gdk.TYPE_lng, t), ora.Bat.from_array(ora.TYPE_lng, t)
        _same(gdk.GDKanalyticalnthvalue(b, s, e, t=tb), ora.analyticalnthvalue(ob, os_, oe, t=otb), tname)
    with pytest.raises(gdk.GDKError, match="nth_value must be greater than zero"):
        gdk.GDKanalyticalnthvalue(b, s, e, nth=0)


@pytest.mark.gpu
@pytest.mark.parametrize("tname,dt", TYPES)
@pytest.mark.parametrize("frame", [3, 4, 5, 6, "rows_small", "rows_wide", "range"])
@pytest.mark.parametrize("layout", ["one", "small", "large"])
def test_min_max(gdk, ora, tname, dt, frame, layout):
    r = rng(len(tname) * 13 + len(str(frame)) + len(layout))
    n = 20_011
    v = _vals(r, tname, dt, n, nils=0.1)
    if tname in ("flt", "dbl"):
        v = np.abs(v)                     # no -0.0 / +0.0 mixes (see the module docstring)
    b, ob = _pair(gdk, ora, tname, v)
    pf, of = _layout(r, n, layout)
    p, op = _bits(gdk, ora, pf)
    o, oo = _bits(gdk, ora, of)
    s = e = os_ = oe = None
    ft = frame
    if frame == "rows_small":
        s, e, os_, oe = _rows_bounds(gdk, ora, n, p, op, 2, 3)
        ft = 0
    elif frame == "rows_wide":
        s, e, os_, oe = _rows_bounds(gdk, ora, n, p, op, 700, 40)
        ft = 0
    elif frame == "range":
        col = np.sort(r.integers(0, n // 4, n)).astype(np.int64)
        bg, bo = gdk.BAT.from_numpy(gdk.TYPE_lng, col), ora.Bat.from_array(ora.TYPE_lng, col)
        s = gdk.GDKanalyticalwindowbounds(bg, p, 30, True, tp2=gdk.TYPE_lng, unit=1)
        e = gdk.GDKanalyticalwindowbounds(bg, p, 10, False, tp2=gdk.TYPE_lng, unit=1)
        os_ = ora.windowbounds(bo, op, None, 30, ora.TYPE_lng, ora.TYPE_lng, 1, True)
        oe = ora.windowbounds(bo, op, None, 10, ora.TYPE_lng, ora.TYPE_lng, 1, False)
        ft = 0
    _same(gdk.GDKanalyticalmin(b, p, o, s, e, ft), ora.analyticalmin(ob, op, oo, os_, oe, ft), tname)
    _same(gdk.GDKanalyticalmax(b, p, o, s, e, ft), ora.analyticalmax(ob, op, oo, os_, oe, ft), tname)


@pytest.mark.gpu
def test_min_max_zero_ties_running_frames(gdk, ora):
    """-0.0 / +0.0 ties in the running frames resolve as the reference's
    scans do: frames 3 / 5 keep the earlier zero, frame 4 the later one --
    compared bit for bit."""
    v = np.array([1.0, 0.0, -0.0, 2.0, -0.0, 0.0, 3.0, 0.0], np.float64)
    b, ob = _pair(gdk, ora, "dbl", v)
    p, op = _bits(gdk, ora, [0, 0, 0, 0, 1, 0, 0, 0])
    o, oo = _bits(gdk, ora, [0, 1, 1, 1, 1, 1, 0, 1])
    for ft in (3, 4, 5):
        for fn, ofn in ((gdk.GDKanalyticalmin, ora.analyticalmin), (gdk.GDKanalyticalmax, ora.analyticalmax)):
            got = np.asarray(fn(b, p, o, None, None, ft).values())
            want = np.asarray(ofn(ob, op, oo, None, None, ft).values())
            assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), (ft, fn.__name__)


def test_oracle_window_small_cases(ora):
    """Hand-checked cases of the restatement (the reference's loops on a
    6-row column with partitions [0, 3) and [3, 6))."""
    b = ora.Bat.from_array(ora.TYPE_int, np.array([5, 3, 7, 1, 9, 2], np.int32))
    p = ora.Bat.from_array(ora.TYPE_bit, np.array([0, 0, 0, 1, 0, 0], np.int8))
    assert list(ora.analyticallag(b, p, 1, -1).values()) == [-1, 5, 3, -1, 1, 9]
    assert list(ora.analyticallead(b, p, 2, 0).values()) == [7, 0, 0, 2, 0, 0]
    assert list(ora.analyticalntile(b, p, ntile=2, tpe=ora.TYPE_int).values()) == [1, 1, 2, 1, 1, 2]
    assert list(ora.analyticalmin(b, p, None, None, None, 5).values()) == [3, 3, 3, 1, 1, 1]
    assert list(ora.analyticalmax(b, p, None, None, None, 5).values()) == [7, 7, 7, 9, 9, 9]
    o = ora.Bat.from_array(ora.TYPE_bit, np.array([0, 1, 0, 1, 1, 1], np.int8))
    assert list(ora.analyticalmin(b, p, o, None, None, 3).values()) == [5, 3, 3, 1, 1, 1]
    assert list(ora.analyticalmax(b, p, o, None, None, 4).values()) == [7, 7, 7, 9, 9, 2]
    s = ora.Bat.from_array(ora.TYPE_oid, np.array([0, 0, 1, 3, 3, 4], np.uint64))
    e = ora.Bat.from_array(ora.TYPE_oid, np.array([1, 2, 3, 4, 5, 6], np.uint64))
    assert list(ora.analyticalfirst(b, s, e).values()) == [5, 5, 3, 1, 1, 9]
    assert list(ora.analyticallast(b, s, e).values()) == [5, 3, 7, 1, 9, 2]
    assert list(ora.analyticalnthvalue(b, s, e, nth=2).values()) == [np.iinfo(np.int32).min, 3, 7,
                                                                   np.iinfo(np.int32).min, 9, 2]
    assert list(ora.analyticalmin(b, p, None, s, e, 0).values()) == [5, 3, 3, 1, 1, 2]


@pytest.mark.gpu
@pytest.mark.parametrize("tname,dt", TYPES + [("str", None)])
@pytest.mark.parametrize("mode", ["none", "p", "npbit"])
def test_diff(gdk, ora, tname, dt, mode):
    """GDKanalyticaldiff over sorted runs with nils (NaN runs for floats,
    -0.0 next to +0.0), with a partition column, a constant npbit or neither."""
    r = rng(len(tname) * 5 + len(mode))
    n = 30_007
    if tname == "str":
        from strheap import sample
        t, heap, _ = sample(r, n, 4)
        t = np.sort(t)
        b = gdk.BAT.from_numpy(gdk.TYPE_str, t, vheap=heap, sorted_=False, revsorted=False, key=False, nonil=False)
        ob = ora.Bat.from_array(ora.TYPE_str, t, vheap=heap)
    else:
        v = _vals(r, tname, dt, n, nils=0.0)
        if tname == "hge":
            v = sorted(v)
            v[:50] = [-(1 << 127)] * 50
        else:
            v = np.sort(v)
            if tname in ("flt", "dbl"):
                v[:50] = np.nan
                v[100:103] = [-0.0, 0.0, -0.0]
            else:
                v[:50] = np.iinfo(dt).min
        b, ob = _pair(gdk, ora, tname, v)
        b.s.tnonil = 0
        ob.s.nonil = 0
    pf, _ = _layout(r, n, "small")
    p, op = _bits(gdk, ora, pf)
    if mode == "p":
        got, want = gdk.GDKanalyticaldiff(b, p=p), ora.analyticaldiff(ob, p=op)
    elif mode == "npbit":
        got, want = gdk.GDKanalyticaldiff(b, npbit=1), ora.analyticaldiff(ob, npbit=1)
    else:
        got, want = gdk.GDKanalyticaldiff(b), ora.analyticaldiff(ob)
    assert np.array_equal(got.to_numpy(), np.asarray(want.values()))


@pytest.mark.gpu
def test_window_sqltests(gdk):
    """analytics00 / 01 / 02 / 14 / 15.test (the reference's own answers) on
    the device: the same 346 window queries the oracle replays
    (tests/test_oracle.py::test_window_sqltests_oracle)."""
    from helpers import replay_window_sqltests, sqlwin_api_gdk
    ran, bad = replay_window_sqltests(sqlwin_api_gdk(gdk))
    assert ran >= 346
    assert not bad, bad[:3]
