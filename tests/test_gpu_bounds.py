"""GDKanalyticalwindowbounds on the device (gdk/gdk_analytic_bounds.c:1440):
ROWS / RANGE / GROUPS, every value and limit type, static and per-row
limits, pinned on the reference's SQL fixtures and compared with the oracle
(values, errors and result properties)."""
import numpy as np
import pytest

from helpers import (TYPE_DATE, TYPE_DAYTIME, TYPE_TIMESTAMP, bound_args, interval_cases, mkdate,
                     mktimestamp, replay_employee, replay_intervals)

pytestmark = pytest.mark.gpu

BTE, SHT, INT, LNG, HGE, FLT, DBL, BIT = 3, 4, 5, 10, 11, 8, 9, 2
NILS = {BTE: -(1 << 7), SHT: -(1 << 15), INT: -(1 << 31), LNG: -(1 << 63), HGE: -(1 << 127),
        TYPE_DATE: -(1 << 31), TYPE_DAYTIME: -(1 << 63), TYPE_TIMESTAMP: -(1 << 63)}
NPT = {BTE: np.int8, SHT: np.int16, INT: np.int32, LNG: np.int64, FLT: np.float32, DBL: np.float64,
       TYPE_DATE: np.int32, TYPE_DAYTIME: np.int64, TYPE_TIMESTAMP: np.int64, BIT: np.int8}


def hge_pairs(vals):
    out = np.empty((len(vals), 2), np.uint64)
    for i, v in enumerate(vals):
        v = int(v) & ((1 << 128) - 1)
        out[i, 0], out[i, 1] = v & ((1 << 64) - 1), v >> 64
    return out


def both(gdk, ora, tp, vals):
    """(device BAT, oracle Bat) of the same values (Python list / array)."""
    if tp == HGE:
        a = hge_pairs(vals)
    else:
        a = np.asarray(vals, NPT[tp])
    return gdk.BAT.from_numpy(tp, a), ora.Bat.from_array(tp, a)


def dev_bounds(gdk):
    def f(b, p, l, lim, tp1, tp2, unit, pre, sh):
        return gdk.GDKanalyticalwindowbounds(b, p, lim, pre, tp1=tp1, tp2=tp2, unit=unit, l=l,
                                             second_half=sh).to_numpy()
    return f


def test_employee_fixture(gdk):
    """window_functions.test: SUM(salary) over ROWS 'unbounded preceding ..
    current row' and '2 preceding .. current row', GROUPS '1 preceding ..
    1 following', RANGE '100.0 preceding .. 50.0 following' on
    DECIMAL(7,2) (int at scale 2)."""
    assert replay_employee(dev_bounds(gdk), lambda tp, a: gdk.BAT.from_numpy(tp, a)) == []


def test_interval_fixture(gdk):
    """analytics07.test: RANGE frames of month / second / minute / hour
    intervals over date, timestamp and time columns, asc and desc."""
    assert replay_intervals(dev_bounds(gdk), lambda tp, a: gdk.BAT.from_numpy(tp, a)) == []


def test_interval_errors(gdk):
    n = 0
    for c, tp, v in interval_cases(errors=True):
        b = gdk.BAT.from_numpy(tp, v)
        with pytest.raises(gdk.GDKError, match="42000!"):
            for bnd, st in ((c["start"], True), (c["end"], False)):
                pre, sh, tp2, lim = bound_args(1, bnd, st, tp)
                gdk.GDKanalyticalwindowbounds(b, None, lim, pre, tp1=tp, tp2=tp2, unit=1, second_half=sh)
        n += 1
    assert n == 2


# ---- random parity against the oracle ------------------------------------------
def rand_values(r, tp, n, nil_frac):
    if tp == FLT or tp == DBL:
        v = np.round(r.normal(0, 50, n), 1).astype(NPT[tp])
        v[r.random(n) < nil_frac] = np.nan
        return list(v)
    if tp == TYPE_DATE:
        v = [mkdate(int(y), int(m), int(d)) for y, m, d in
             zip(r.integers(1990, 2000, n), r.integers(1, 13, n), r.integers(1, 29, n))]
    elif tp == TYPE_DAYTIME:
        v = [int(x) for x in r.integers(0, 86_400_000_000, n)]
    elif tp == TYPE_TIMESTAMP:
        v = [mktimestamp(mkdate(int(y), int(m), int(d)), int(t)) for y, m, d, t in
             zip(r.integers(1995, 1997, n), r.integers(1, 13, n), r.integers(1, 29, n),
                 r.integers(0, 86_400_000_000, n))]
    else:
        span = {BTE: 120, SHT: 30000, INT: 2_000_000_000, LNG: 1 << 62, HGE: 1 << 120}[tp]
        if r.random() < 0.5:         # small values: frames of several rows
            span = min(span, 60)
        if tp == HGE and span > 60:
            # values beyond lng: a high word plus a low word
            v = [int(h) * (1 << 64) + int(lo) for h, lo in
                 zip(r.integers(-(1 << 40), 1 << 40, n), r.integers(0, 1 << 62, n))]
        else:
            v = [int(x) for x in r.integers(-span, span, n)]
    nil = NILS[tp]
    return [nil if r.random() < nil_frac else x for x in v]


def order_partitions(vals, parts, tp, how):
    """sort each partition asc (nils first) / desc (nils last) / leave it"""
    if how == "none":
        return vals
    isnil = (lambda x: x != x) if tp in (FLT, DBL) else (lambda x: x == NILS[tp])
    out = []
    starts = list(np.flatnonzero(parts)) + [len(vals)]
    if starts[0] != 0:
        starts = [0] + starts
    for a, e in zip(starts[:-1], starts[1:]):
        seg = vals[a:e]
        nn = sorted(x for x in seg if not isnil(x))
        nl = [x for x in seg if isnil(x)]
        out += nl + nn if how == "asc" else nn[::-1] + nl
    return out


def rand_limit(r, tp1, tp2, small):
    if tp2 in (FLT, DBL):
        return float(np.float32(r.choice([0.5, 3.0, 25.0, 80.0])))
    if tp1 in (TYPE_DATE, TYPE_TIMESTAMP) and tp2 == INT:
        return int(r.integers(1, 5))             # months
    if tp1 in (TYPE_DATE, TYPE_DAYTIME, TYPE_TIMESTAMP):
        return int(r.choice([1, 30, 3600, 86400 * 3, 86400 * 40])) * 1000    # msec
    if small:
        return int(r.integers(1, 40))
    hi = {BTE: 120, SHT: 30000, INT: 1 << 31, LNG: 1 << 62, HGE: 1 << 100}[tp2]
    return int(r.integers(1, min(hi, 1 << 62)))


def compare(gdk, ora, b, ob, p, op, l, ol, lim, tp1, tp2, unit, pre, sh):
    try:
        want = ora.windowbounds(ob, op, ol, lim, tp1, tp2, unit, pre, sh)
        werr = None
    except ora.OracleError as e:
        werr = str(e)
    try:
        got = gdk.GDKanalyticalwindowbounds(b, p, lim, pre, tp1=tp1, tp2=tp2, unit=unit, l=l, second_half=sh)
        gerr = None
    except gdk.GDKError as e:
        gerr = str(e)
    assert werr == gerr, (werr, gerr)
    if werr is None:
        assert np.array_equal(got.to_numpy(), want.values())
        assert (got.s.tnonil, got.s.tnil) == (want.s.nonil, want.s.nil)
    return werr


@pytest.mark.parametrize("tp", [BTE, SHT, INT, LNG, HGE, FLT, DBL, TYPE_DATE, TYPE_DAYTIME, TYPE_TIMESTAMP])
def test_range_random(gdk, ora, tp):
    r = np.random.default_rng(1000 + tp)
    errors = 0
    for trial in range(24):
        n = int(r.integers(1, 3000))
        nparts = int(r.integers(1, 6))
        parts = np.zeros(n, np.int8)
        parts[r.choice(n, min(n, nparts), replace=False)] = 1
        how = ["asc", "desc", "none"][trial % 3]
        vals = order_partitions(rand_values(r, tp, n, 0.05 if trial % 2 else 0.0), parts, tp, how)
        b, ob = both(gdk, ora, tp, vals)
        P, OP = both(gdk, ora, BIT, parts) if trial % 4 else (None, None)
        if tp in (TYPE_DATE, TYPE_TIMESTAMP):
            tp2 = [INT, LNG][trial % 2]
        elif tp == TYPE_DAYTIME:
            tp2 = LNG
        elif tp in (FLT, DBL):
            tp2 = tp
        elif tp == HGE:
            tp2 = HGE
        else:
            tp2 = [BTE, SHT, INT, LNG, HGE][trial % 5]
            if tp2 in (BTE, SHT) and tp2 > tp:
                tp2 = tp
        dynamic = trial % 3 == 1
        small = trial % 2 == 0
        for pre in (True, False):
            if dynamic:
                lims = [rand_limit(r, tp, tp2, small) for _ in range(n)]
                l, ol = both(gdk, ora, tp2, lims)
                lim = None
            else:
                lim = rand_limit(r, tp, tp2, small)
                if tp2 in (BTE, SHT, INT) and lim >= {BTE: 127, SHT: 32767, INT: (1 << 31) - 1}[tp2]:
                    lim = 5
                l = ol = None
            if compare(gdk, ora, b, ob, P, OP, l, ol, lim, tp, tp2, 1, pre, 0) is not None:
                errors += 1
    assert errors < 24        # overflow cases occur, but most trials compute bounds


@pytest.mark.parametrize("unit", [0, 2])
def test_rows_groups_random(gdk, ora, unit):
    r = np.random.default_rng(77 + unit)
    for trial in range(30):
        n = int(r.integers(1, 4000))
        parts = np.zeros(n, np.int8)
        parts[r.choice(n, min(n, int(r.integers(1, 8))), replace=False)] = 1
        P, OP = both(gdk, ora, BIT, parts) if trial % 3 else (None, None)
        if unit == 2:
            peers = (r.random(n) < 0.3).astype(np.int8)
            peers[parts == 1] = 1
            b, ob = both(gdk, ora, BIT, peers)
            tp1 = BIT
        else:
            b, ob = both(gdk, ora, INT, r.integers(0, 100, n))
            tp1 = INT
        tp2 = [BTE, SHT, INT, LNG, HGE][trial % 5]
        for pre in (True, False):
            for sh in (0, 1):
                if trial % 2:
                    lims = [int(x) for x in r.integers(0, 20, n)]
                    l, ol = both(gdk, ora, tp2, lims)
                    compare(gdk, ora, b, ob, P, OP, l, ol, None, tp1, tp2, unit, pre, sh)
                else:
                    lim = int(r.integers(0, 50))
                    compare(gdk, ora, b, ob, P, OP, None, None, lim, tp1, tp2, unit, pre, sh)


def test_special_bounds(gdk, ora):
    """unbounded (type max) and current row (0) shortcuts, and the error
    paths: negative / nil limits, unsupported types, groups on non-bit."""
    r = np.random.default_rng(5)
    n = 500
    parts = np.zeros(n, np.int8)
    parts[[0, 100, 250]] = 1
    P, OP = both(gdk, ora, BIT, parts)
    vals = order_partitions([int(x) for x in r.integers(0, 20, n)], parts, INT, "asc")
    b, ob = both(gdk, ora, INT, vals)
    fv = order_partitions(list(np.round(r.normal(0, 3, n), 0).astype(np.float64)), parts, DBL, "asc")
    fb, ofb = both(gdk, ora, DBL, fv)
    cases = [
        (b, ob, INT, INT, 1, (1 << 31) - 1), (b, ob, INT, INT, 1, 0), (b, ob, INT, LNG, 1, (1 << 63) - 1),
        (b, ob, INT, BTE, 1, 127), (b, ob, INT, INT, 1, -3), (b, ob, INT, LNG, 1, -(1 << 63)),
        (b, ob, INT, HGE, 1, (1 << 127) - 1), (b, ob, INT, HGE, 1, 0), (b, ob, INT, HGE, 1, 7),
        (b, ob, INT, FLT, 1, 2.0), (b, ob, INT, FLT, 1, 0.0), (fb, ofb, DBL, DBL, 1, 0.0),
        (fb, ofb, DBL, DBL, 1, 1.79769313486231570815e+308), (fb, ofb, DBL, DBL, 1, 1.5),
        (fb, ofb, DBL, DBL, 1, float("nan")), (fb, ofb, DBL, LNG, 1, 3),
        (b, ob, INT, LNG, 0, (1 << 63) - 1), (b, ob, INT, LNG, 0, 0), (b, ob, INT, LNG, 0, -1),
        (b, ob, INT, LNG, 2, 1), (b, ob, INT, DBL, 0, 1.0),
    ]
    for bb, obb, tp1, tp2, unit, lim in cases:
        for pre in (True, False):
            compare(gdk, ora, bb, obb, P, OP, None, None, lim, tp1, tp2, unit, pre, 1)


def test_narrow_overflow(gdk, ora):
    """bte values spanning more than 127: the reference's SUB_WITH_CHECK in
    the value type overflows on the stopping pair, even with small limits;
    the lng fast path must raise it exactly where the walk would."""
    for seed in range(6):
        r = np.random.default_rng(seed)
        n = 2000
        v = np.sort(r.integers(-120, 120, n)).astype(np.int8)
        b, ob = both(gdk, ora, BTE, v)
        for lim in (3, 100, 126, 200):
            for tp2 in (SHT, LNG):
                for pre in (True, False):
                    compare(gdk, ora, b, ob, None, None, None, None, lim, BTE, tp2, 1, pre, 0)


def test_range_large_int(gdk, ora):
    """DECIMAL(7,2)-style int column with partitions, 1M rows: the widened
    fast path against the oracle."""
    r = np.random.default_rng(11)
    n = 1_000_000
    parts = np.zeros(n, np.int8)
    parts[::5000] = 1
    v = np.sort(r.integers(0, 10_000_000, n)).astype(np.int32)
    b, ob = both(gdk, ora, INT, v)
    P, OP = both(gdk, ora, BIT, parts)
    for pre in (True, False):
        compare(gdk, ora, b, ob, P, OP, None, None, 100, INT, INT, 1, pre, 0)
