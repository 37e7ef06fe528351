"""Shared test helpers: replay of the reference's MAL fixtures against any GDK
implementation (oracle or product) and seeded random inputs."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "maltest_fixtures.json")))


def replay_select(G, make_bat, TYPE_int, NIL):
    """Run the 192 algebra.select cases of select.maltest; returns mismatches."""
    from monetdb_amd import mal
    fx = FIX["select"]
    vals = [NIL if v is None else v for v in fx["values"]]
    srt = sorted(vals)
    bats = {"b": make_bat(TYPE_int, vals),
            "s": make_bat(TYPE_int, srt),
            "r": make_bat(TYPE_int, srt[::-1])}
    bad = []
    for c in fx["cases"]:
        X = bats[c["bat"]]
        x = mal.ALGselect2(G, X, None, c["low"], c["high"], c["li"], c["hi"], c["anti"], nil=NIL)
        z = np.asarray(G.BATproject(x, X).values())
        got = [None] * int((z == NIL).sum()) + sorted(int(v) for v in z if v != NIL)
        if got != c["expected"]:
            bad.append((c, got))
    return bad


def replay_project(G, make_bat, TYPE_int, NIL):
    """algebra.select + algebra.projection cases of tst033 / tst034 /
    orderidx02.maltest: the printed (head, value) or (head, oid, value) rows,
    row-sorted as the tests print them.  Returns mismatches."""
    from monetdb_amd import mal
    bad = []
    for fx in FIX["project"]:
        for c in fx["cases"]:
            b = make_bat(TYPE_int, [NIL if v is None else v for v in c["values"]])
            s = mal.ALGselect2(G, b, None, c["low"], c["high"], c["li"], c["hi"], c["anti"], nil=NIL)
            z = [int(v) for v in np.asarray(G.BATproject(s, b).values())]
            oids = [int(v) for v in np.asarray(s.values())]
            width = len(c["expected_rows"][0]) if c["expected_rows"] else 2
            rows = [[i, v] for i, v in enumerate(z)] if width == 2 else \
                [[i, o, v] for i, (o, v) in enumerate(zip(oids, z))]
            if sorted(rows) != c["expected_rows"]:
                bad.append((fx["source"], c, rows))
    return bad


def rng(seed):
    return np.random.default_rng(seed)


def with_nils(a, nil, frac, r):
    a = a.copy()
    if frac > 0:
        m = r.random(a.shape[0]) < frac
        a[m] = nil
    return a


def firstn_cases(plain_only=False):
    """algebra.firstn cases of pqueue*.maltest as (case, b values, s, g)."""
    for fx in FIX["firstn"]:
        for c in fx["cases"]:
            if plain_only and (c["gids"] or c["distinct"]):
                continue
            yield fx["source"], c


def replay_window_frames(sumf, countf, make_bat, TYPE_int, TYPE_bit, TYPE_lng):
    """Windowed SUM / COUNT cases of analytics03.test.  Rows are ordered by
    (partition, order) keys; p / o mark partition and peer-group starts;
    frame 3 = unbounded preceding .. current row's peers, 5 = partition.
    sumf(b, p, o, tp2, frame) / countf(b, p, o, ignore_nils, frame) return
    per-row values in sorted order.  Returns mismatches."""
    bad = []
    for c in FIX["window_frames"]["cases"]:
        aa, bb = np.array(c["aa"], np.int32), np.array(c["bb"], np.int32)
        cols = {"aa": aa, "bb": bb}
        keys = [cols[k] for k in (c["order"], c["part"]) if k is not None]
        perm = np.lexsort(keys) if keys else np.arange(len(aa))
        part = cols[c["part"]][perm] if c["part"] else np.zeros(len(aa), np.int32)
        order = cols[c["order"]][perm] if c["order"] else np.zeros(len(aa), np.int32)
        p = np.zeros(len(aa), np.int8)
        p[0] = 1
        p[1:] = part[1:] != part[:-1]
        o = p.copy()
        o[1:] |= order[1:] != order[:-1]
        frame = 5 if c["frame"] == "all" else 3
        B, P, O = make_bat(TYPE_int, aa[perm]), make_bat(TYPE_bit, p), make_bat(TYPE_bit, o)
        if c["agg"] == "sum":
            got = sumf(B, P, O, TYPE_lng, frame)
        else:
            got = countf(B, P, O, c["agg"] == "count", frame)
        got = np.asarray(got, np.int64)
        if c["output_order"] == "bb,aa":
            back = np.empty_like(got)
            back[perm] = got
            got = back[np.lexsort((aa, bb))]
        if [int(x) for x in got] != c["expected"]:
            bad.append((c, list(got)))
    return bad


def replay_window_avg(avgf, make_bat, TYPE_int, TYPE_flt, TYPE_bit):
    """Windowed AVG cases of analytics03.test (frame 3 = unbounded preceding
    .. current row's peers, 4 = current row's peers .. unbounded following).
    avgf(b, p, o, frame) returns per-row dbl averages in sorted order; the
    reference prints 3 decimals (or floor()).  Returns mismatches."""
    bad = []
    for c in FIX["window_avg"]["cases"]:
        aa, bb = np.array(c["aa"], np.int32), np.array(c["bb"], np.int32)
        cols = {"aa": aa, "bb": bb}
        keys = [cols[k] for k in (c["order"], c["part"]) if k is not None]
        perm = np.lexsort(keys) if keys else np.arange(len(aa))
        part = cols[c["part"]][perm] if c["part"] else np.zeros(len(aa), np.int32)
        order = cols[c["order"]][perm] if c["order"] else np.zeros(len(aa), np.int32)
        p = np.zeros(len(aa), np.int8)
        p[0] = 1
        p[1:] = part[1:] != part[:-1]
        o = p.copy()
        o[1:] |= order[1:] != order[:-1]
        frame = {"upto": 3, "from": 4, "all": 5}[c["frame"]]
        b = make_bat(TYPE_flt, aa[perm].astype(np.float32)) if c["agg"] == "avgf" else make_bat(TYPE_int, aa[perm])
        got = np.asarray(avgf(b, make_bat(TYPE_bit, p), make_bat(TYPE_bit, o), frame), np.float64)
        got = np.floor(got) if c["floor"] else np.round(got, 3)
        if list(got) != c["expected"]:
            bad.append((c, list(got)))
    return bad


# ---- window frame bounds fixtures (window_functions.test, analytics07.test) --
INT_MAX, LNG_MAX = (1 << 31) - 1, (1 << 63) - 1
TYPE_INT, TYPE_LNG, TYPE_BIT, TYPE_OID = 5, 10, 2, 6
TYPE_DATE, TYPE_DAYTIME, TYPE_TIMESTAMP = 12, 13, 14
MSEC = {"second": 1000, "minute": 60_000, "hour": 3_600_000, "day": 86_400_000}


def mkdate(y, m, d):
    """gdk_time.c:27 mkdate (packed (year + 4712) * 12 + month - 1, day)."""
    return (((y + 4712) * 12 + m - 1) << 5) | d


def mkdaytime(h, mi, s, us=0):
    return ((h * 60 + mi) * 60 + s) * 1_000_000 + us


def mktimestamp(d, t):
    return (d << 37) | t


def temporal_value(kind, text):
    """Packed GDK value of a date / timestamp / time literal."""
    if kind == "date":
        y, m, d = (int(x) for x in text.split("-"))
        return TYPE_DATE, mkdate(y, m, d)
    if kind == "time":
        h, mi, s = (int(x) for x in text.split(":"))
        return TYPE_DAYTIME, mkdaytime(h, mi, s)
    day, clock = text.split()
    y, m, d = (int(x) for x in day.split("-"))
    h, mi, s = (int(x) for x in clock.split(":"))
    return TYPE_TIMESTAMP, mktimestamp(mkdate(y, m, d), mkdaytime(h, mi, s))


def bound_args(unit, bnd, is_start, col_tp, scale=0):
    """GDKanalyticalwindowbounds arguments (preceding, second_half, tp2,
    limit) of one frame bound as the SQL layer builds them
    (rel_select.c:4605-4710 generate_window_bound / calculate_window_bound,
    sql_rank.c:124-130): ROWS / GROUPS limits are lng; RANGE limits have the
    ORDER BY column's type (numeric) or are month (int) / msec (lng)
    intervals (temporal); UNBOUNDED is the bound type's max, CURRENT ROW 0."""
    kind, amount, word = bnd
    code = {"PRECEDING": 0, "FOLLOWING": 1, "CURRENT": 4, "UNBOUNDED": 0}[kind]
    if kind == "UNBOUNDED" and not is_start:
        code = 1
    if not is_start:
        code = {0: 2, 1: 3, 4: 5}[code]
    preceding = code % 2 == 0
    second_half = 0 if (code < 2 or code == 4) else 1
    temporal = col_tp in (TYPE_DATE, TYPE_DAYTIME, TYPE_TIMESTAMP)
    if unit != 1 or temporal:
        tp2 = TYPE_LNG
        if kind == "UNBOUNDED":
            return preceding, second_half, tp2, LNG_MAX
        if kind == "CURRENT":
            return preceding, second_half, tp2, 0
        if word == "month":
            return preceding, second_half, TYPE_INT, int(amount)
        if word is not None:
            return preceding, second_half, tp2, int(amount) * MSEC[word]
        return preceding, second_half, tp2, int(float(amount))
    tp2 = col_tp
    if kind == "UNBOUNDED":
        return preceding, second_half, tp2, INT_MAX
    if kind == "CURRENT":
        return preceding, second_half, tp2, 0
    return preceding, second_half, tp2, int(round(float(amount) * 10 ** scale))


def employee_frames():
    """window_functions.test employee rows ordered by (dep_name, salary):
    (ids, salary, partition bits, peer bits, cases)."""
    fx = FIX["window_bounds_employee"]
    emp = sorted(fx["employee"], key=lambda r: (r[1], r[2]))
    ids = [r[0] for r in emp]
    sal = np.array([r[2] for r in emp], np.int32)
    dep = [r[1] for r in emp]
    p = np.array([1] + [int(dep[i] != dep[i - 1]) for i in range(1, len(dep))], np.int8)
    o = p.copy()
    o[1:] |= (sal[1:] != sal[:-1]).astype(np.int8)
    return ids, sal, p, o, fx["cases"]


def replay_employee(bounds, make_bat):
    """bounds(b, p, l=None, bound, tp1, tp2, unit, preceding, second_half) ->
    numpy oid array.  Returns mismatches of the frame sums."""
    ids, sal, p, o, cases = employee_frames()
    B, P, O = make_bat(TYPE_INT, sal), make_bat(TYPE_BIT, p), make_bat(TYPE_BIT, o)
    bad = []
    for c in cases:
        col = O if c["unit"] == 2 else B
        coltp = TYPE_BIT if c["unit"] == 2 else TYPE_INT
        res = []
        for bnd, st in ((c["start"], True), (c["end"], False)):
            pre, sh, tp2, lim = bound_args(c["unit"], bnd, st, TYPE_INT, scale=2)
            res.append(np.asarray(bounds(col, P, None, lim, coltp, tp2, c["unit"], pre, sh), np.int64))
        s, e = res
        sums = [int(sal[s[i]:e[i]].sum()) for i in range(len(sal))]
        if ids != c["ids"] or sums != c["expected"]:
            bad.append((c, sums))
    return bad


def interval_cases(errors=False):
    """analytics07.test cases: (case, column type, sorted packed values)."""
    fx = FIX["window_bounds_intervals"]
    for c in fx["errors" if errors else "cases"]:
        vals = [temporal_value(k, t) for k, t in fx["tables"][c["table"]]]
        tp = vals[0][0]
        v = sorted(x[1] for x in vals)
        if c["desc"]:
            v = v[::-1]
        yield c, tp, np.array(v, np.int32 if tp == TYPE_DATE else np.int64)


def replay_intervals(bounds, make_bat):
    """count(*) over the analytics07 frames = end - start."""
    bad = []
    for c, tp, v in interval_cases():
        B = make_bat(tp, v)
        res = []
        for bnd, st in ((c["start"], True), (c["end"], False)):
            pre, sh, tp2, lim = bound_args(1, bnd, st, tp)
            res.append(np.asarray(bounds(B, None, None, lim, tp, tp2, 1, pre, sh), np.int64))
        got = [int(x) for x in res[1] - res[0]]
        if got != c["expected"]:
            bad.append((c, got))
    return bad


# ---- BATjoin shapes covering every algorithm BATjoin chooses -------------------
# (gdk_join.c:4542-4618).  Each case: l / r values with their GDK type, head
# bases, optional candidate lists (sorted oid arrays or ("dense", seq, n)),
# the flags the caller knows (both implementations start from the same
# ones) and the algorithm the reference takes for it.

def join_cases():
    r = rng(4242)
    I32, I64, U64 = np.int32, np.int64, np.uint64
    NI = -(1 << 31)
    cs = []

    def add(name, tp, lv, rv, algo, lh=0, rh=0, sl=None, sr=None, nil_matches=False,
            lflags=None, rflags=None, lvoid=None, rvoid=None):
        cs.append(dict(name=name, tp=tp, lv=lv, rv=rv, algo=algo, lh=lh, rh=rh, sl=sl, sr=sr,
                       nil_matches=nil_matches, lflags=lflags or {}, rflags=rflags or {},
                       lvoid=lvoid, rvoid=rvoid))

    # selectjoin: a single left candidate, an all-equal left, the same on the right
    rv = r.integers(0, 50, 5000).astype(I32)
    add("single_l", "int", np.array([7], I32), rv, "selectjoin", rh=3)
    add("single_l_cand", "int", r.integers(0, 50, 300).astype(I32), rv, "selectjoin", lh=10,
        sl=np.array([25], U64))
    add("const_l", "int", np.full(40, 9, I32), rv, "selectjoin", lh=5)
    add("const_l_nil", "int", np.full(30, NI, I32), np.where(rv < 3, NI, rv).astype(I32), "selectjoin",
        nil_matches=True)
    add("const_l_nil_nomatch", "int", np.full(30, NI, I32), np.where(rv < 3, NI, rv).astype(I32),
        "selectjoin")
    add("single_r", "int", r.integers(0, 50, 5000).astype(I32), np.array([11], I32), "selectjoin_swapped")
    add("const_r", "lng", r.integers(0, 20, 3000).astype(I64), np.full(17, 4, I64), "selectjoin_swapped",
        lh=2, rh=9)
    # mergejoin_void: a dense right (or left) side
    lo = r.integers(0, 3000, 8000).astype(U64)
    lo[::97] = 1 << 63
    add("dense_r", "oid", lo, None, "mergejoin_void", rvoid=(1000, 1500), rh=40)
    add("dense_r_cand", "oid", lo, None, "mergejoin_void", rvoid=(1000, 1500), rh=40,
        sr=("dense", 100, 700), sl=np.sort(r.choice(8000, 3000, replace=False)).astype(U64))
    add("dense_l", "oid", None, r.integers(0, 900, 6000).astype(U64), "mergejoin_void_swapped",
        lvoid=(200, 500), lh=7)
    add("dense_both_sorted_l", "oid", np.sort(r.integers(0, 900, 6000)).astype(U64), None,
        "mergejoin_void", rvoid=(100, 300))
    # both sorted: full dense candidates (mergejoin_int / _lng) and general
    ls = np.sort(r.integers(0, 4000, 20000)).astype(I32)
    rs = np.sort(r.integers(0, 4000, 9000)).astype(I32)
    add("sorted_int", "int", ls, rs, "mergejoin_sorted", lh=3, rh=11)
    add("sorted_lng_nil", "lng", np.sort(np.where(r.random(5000) < .05, -(1 << 63),
                                                  r.integers(0, 900, 5000))).astype(I64),
        np.sort(np.where(r.random(3000) < .05, -(1 << 63), r.integers(0, 900, 3000))).astype(I64),
        "mergejoin_sorted", nil_matches=True)
    add("sorted_lng_nil_nomatch", "lng", np.sort(np.where(r.random(5000) < .05, -(1 << 63),
                                                          r.integers(0, 900, 5000))).astype(I64),
        np.sort(np.where(r.random(3000) < .05, -(1 << 63), r.integers(0, 900, 3000))).astype(I64),
        "mergejoin_sorted")
    add("sorted_key_dense", "int", np.arange(100, 2100, dtype=I32), np.arange(0, 5000, 2, dtype=I32),
        "mergejoin_sorted")
    add("sorted_consec", "int", np.arange(0, 3000, dtype=I32), np.arange(1000, 9000, dtype=I32),
        "mergejoin_sorted", lh=50, rh=60)
    add("sorted_cands", "int", ls, rs, "mergejoin_sorted",
        sl=np.sort(r.choice(20000, 12000, replace=False)).astype(U64) + 3,
        sr=np.sort(r.choice(9000, 6000, replace=False)).astype(U64) + 11, lh=3, rh=11)
    add("sorted_sht", "sht", np.sort(r.integers(-300, 300, 6000)).astype(np.int16),
        np.sort(r.integers(-300, 300, 2000)).astype(np.int16), "mergejoin_sorted")
    add("ldesc_rasc", "int", ls[::-1].copy(), rs, "mergejoin_sorted", lh=3, rh=11)
    add("lasc_rdesc", "int", ls, rs[::-1].copy(), "mergejoin_sorted")
    add("both_desc", "lng", ls[::-1].astype(I64), rs[::-1].astype(I64), "mergejoin_sorted")
    # one side sorted and binary search cheaper than a hash
    rkey = np.sort(r.choice(1 << 20, 100_000, replace=False)).astype(I32)
    add("small_l_sorted_r", "int", r.choice(rkey, 3000).astype(I32), rkey, "mergejoin", rh=5)
    add("small_l_sorted_r_dups", "int", np.concatenate([r.integers(0, 5000, 1500),
                                                        np.repeat(r.integers(0, 5000, 300), 3)]).astype(I32),
        np.sort(r.integers(0, 5000, 60_000)).astype(I32), "mergejoin")
    add("two_rows_desc", "int", np.array([30, 10, 99], I32), np.arange(40, dtype=I32), "mergejoin")
    add("three_rows_desc", "int", np.array([30, 10, 5, 99], I32), np.arange(40, dtype=I32), "mergejoin")
    add("runs_unsorted", "int", np.array([5, 5, 3, 3, 8, 1, 5], I32), np.sort(r.integers(0, 10, 200)).astype(I32),
        "mergejoin")
    add("small_r_sorted_l", "int", rkey, r.choice(rkey, 3000).astype(I32), "mergejoin_swapped", lh=8)
    # hash joins: swapped (small left) and plain, duplicate build keys, nils
    add("hash_swapped", "int", r.choice(1 << 20, 1000, replace=False).astype(I32),
        r.integers(0, 1 << 20, 100_000).astype(I32), "hashjoin_swapped")
    add("hash_swapped_tiny", "int", np.array([1, 2, 1], I32), np.array([1, 1, 3, 1], I32), "hashjoin_swapped")
    add("hash_plain", "int", r.integers(0, 30_000, 100_000).astype(I32),
        r.choice(30_000, 20_000, replace=False).astype(I32), "hashjoin", lh=4, rh=17)
    add("hash_dups", "lng", r.integers(0, 3000, 50_000).astype(I64), r.integers(0, 3000, 9000).astype(I64),
        "hashjoin")
    add("hash_nils", "int", np.where(r.random(60_000) < .02, NI, r.integers(0, 9000, 60_000)).astype(I32),
        np.where(r.random(12_000) < .02, NI, r.integers(0, 9000, 12_000)).astype(I32), "hashjoin",
        nil_matches=True)
    add("hash_cands", "int", r.integers(0, 30_000, 80_000).astype(I32),
        r.choice(60_000, 30_000, replace=False).astype(I32), "hashjoin",
        sl=np.sort(r.choice(80_000, 50_000, replace=False)).astype(U64),
        sr=("dense", 2000, 20_000))
    add("hash_key_flag", "int", r.integers(0, 30_000, 100_000).astype(I32),
        r.choice(30_000, 20_000, replace=False).astype(I32), "hashjoin",
        lflags=dict(key=False), rflags=dict(key=True))
    add("hash_bte", "bte", r.integers(-100, 100, 40_000).astype(np.int8),
        r.integers(-100, 100, 5_000).astype(np.int8), "hashjoin_swapped")
    return cs


def join_expected(c, lv, rv, lcand, rcand):
    """The pairs BATjoin returns for algorithm c["algo"], from the order rule
    of each algorithm (per driving candidate in order; matches ascending for
    select / merge joins, descending for hash joins; swapped variants drive
    from the right)."""
    algo = c["algo"]
    swapped = algo.endswith("swapped")
    nm = c["nil_matches"]
    dv, ov, dc, oc = (rv, lv, rcand, lcand) if swapped else (lv, rv, lcand, rcand)
    dh, oh = (c["rh"], c["lh"]) if swapped else (c["lh"], c["rh"])
    desc = algo.startswith("hashjoin")
    from collections import defaultdict
    pos = defaultdict(list)
    for o in oc:
        pos[ov[o - oh]].append(o)
    out = []
    for o in dc:
        v = dv[o - dh]
        if v is None and not nm:
            continue
        m = pos.get(v, [])
        for x in (m[::-1] if desc else m):
            out.append((x, o) if swapped else (o, x))
    return out


# ---- window functions of analytics00 / 01 / 02.test ---------------------------
# The SQL layer (sql/server/rel_select.c:4970-5130, sql_rank.c) sorts the rows
# by the partition and order columns (stable: peers keep insertion order;
# ascending puts NULL first, descending last), marks partition starts p and
# peer-group starts o, and calls the GDK window function: first / last /
# nth_value with the frame bounds of sql.window_bound (no ORDER BY: the whole
# partition; ORDER BY: unbounded preceding .. the current row's last peer),
# aggregates with frame type 5 / 3 (rel_select.c:5117) or, for ROWS frames,
# type 0 with computed bounds; lag / lead / ntile with p alone.
FLT_TYPES = {"flt": 8, "dbl": 9}
SQLW_TYPE = {"int": TYPE_INT, "lng": TYPE_LNG, "flt": 8, "dbl": 9}
NILV = {TYPE_INT: -(1 << 31), TYPE_LNG: -(1 << 63)}


def sqlwin_api_gdk(gdk):
    def bounds(col, p, lim, pre, tp1, tp2, unit, sh):
        return gdk.GDKanalyticalwindowbounds(col, p, lim, pre, tp1=tp1, tp2=tp2, unit=unit, second_half=sh)
    return dict(
        mk=lambda tp, v: gdk.BAT.from_numpy(tp, v),
        bounds=bounds,
        ntile=lambda b, p, n, k, tpe: gdk.GDKanalyticalntile(b, p, n=n, ntile=k, tpe=tpe),
        first_value=gdk.GDKanalyticalfirst, last_value=gdk.GDKanalyticallast,
        nth_value=lambda b, s, e, t, nth: gdk.GDKanalyticalnthvalue(b, s, e, t=t, nth=nth),
        lag=gdk.GDKanalyticallag, lead=gdk.GDKanalyticallead,
        min=gdk.GDKanalyticalmin, max=gdk.GDKanalyticalmax, sum=gdk.GDKanalyticalsum,
        count=gdk.GDKanalyticalcount, avg=gdk.GDKanalyticalavg, prod=gdk.GDKanalyticalprod,
        stat=gdk.GDKanalytical_stat, BUN_NONE=gdk.BUN_NONE)


def sqlwin_api_ora(ora):
    def bounds(col, p, lim, pre, tp1, tp2, unit, sh):
        return ora.windowbounds(col, p, None, lim, tp1, tp2, unit, pre, sh)
    return dict(
        mk=lambda tp, v: ora.Bat.from_array(tp, v),
        bounds=bounds,
        ntile=lambda b, p, n, k, tpe: ora.analyticalntile(b, p, n=n, ntile=k, tpe=tpe),
        first_value=ora.analyticalfirst, last_value=ora.analyticallast,
        nth_value=lambda b, s, e, t, nth: ora.analyticalnthvalue(b, s, e, t=t, nth=nth),
        lag=ora.analyticallag, lead=ora.analyticallead,
        min=ora.analyticalmin, max=ora.analyticalmax, sum=ora.analyticalsum,
        count=ora.analyticalcount, avg=ora.analyticalavg, prod=ora.analyticalprod,
        stat=ora.analyticalstat, BUN_NONE=ora.BUN_NONE)


def _sqlwin_perm(tb, spec):
    """stable (partition, order) sort of the table's rows"""
    cols = {c: [r[i] for r in tb["rows"]] for i, c in enumerate(tb["names"])}
    perm = list(range(len(tb["rows"])))

    def key(v):
        return (0,) if v is None else (1, v)
    if spec["order"]:
        perm.sort(key=lambda i: key(cols[spec["order"]][i]), reverse=spec["desc"])
    if spec["part"]:
        pdesc = spec["desc"] and spec["part"] == spec["order"]
        perm.sort(key=lambda i: key(cols[spec["part"]][i]), reverse=pdesc)
    return cols, perm


def _sqlwin_col(api, tp_name, vals):
    tp = SQLW_TYPE[tp_name]
    if tp_name in FLT_TYPES:
        a = np.array([np.nan if v is None else v for v in vals], np.float32 if tp_name == "flt" else np.float64)
    else:
        a = np.array([NILV[tp] if v is None else v for v in vals], np.int32 if tp == TYPE_INT else np.int64)
    return api["mk"](tp, a), tp


def _sqlwin_out(bat, tp):
    vals = np.asarray(bat.values())
    out = []
    for v in vals:
        if tp in (8, 9):
            out.append(None if np.isnan(v) else float(v))
        else:
            out.append(None if int(v) == NILV.get(tp, -(1 << 63)) else int(v))
    return out


SQL_STATS = {"stddev_samp": "stddev_samp", "stddev_pop": "stddev_pop", "var_samp": "variance_samp",
             "var_pop": "variance_pop", "covar_samp": "covariance_samp", "covar_pop": "covariance_pop",
             "corr": "correlation"}


def sqlwin_eval(api, tb, c):
    """the window query's result rows in evaluation (sorted) order; a query
    mixing OVER clauses (spec None): each item in its own order, the rows in
    table order"""
    spec = c["spec"]
    if spec is None:
        # the plan sorts the relation by the first OVER clause that orders
        # anything; a window without PARTITION / ORDER sees that order
        n = len(tb["rows"])
        first = next((it["spec"] for it in c["items"] if it["kind"] == "win" and
                      (it["spec"]["part"] or it["spec"]["order"])), None)
        base = _sqlwin_perm(tb, first)[1] if first else list(range(n))
        tbb = dict(tb, rows=[tb["rows"][i] for i in base])
        cols = []
        for it in c["items"]:
            if it["kind"] == "col":
                cols.append([r[tb["names"].index(it["col"])] for r in tb["rows"]])
                continue
            plain = not (it["spec"]["part"] or it["spec"]["order"])
            tbx, bx = (tbb, base) if plain else (tb, list(range(n)))
            vals = [r[0] for r in sqlwin_eval(api, tbx, dict(items=[it], spec=it["spec"]))]
            _, perm = _sqlwin_perm(tbx, it["spec"])
            back = [None] * n
            for k, i in enumerate(perm):
                back[bx[i]] = vals[k]
            cols.append(back)
        return [list(r) for r in zip(*cols)]
    cols, perm = _sqlwin_perm(tb, spec)
    n = len(perm)
    types = tb["cols"]
    sc = {k: [v[i] for i in perm] for k, v in cols.items()}
    P = O = None
    pb = np.zeros(n, np.int8)
    if spec["part"]:
        pv = sc[spec["part"]]
        pb[0] = 1
        pb[1:] = [pv[i] != pv[i - 1] for i in range(1, n)]
        P = api["mk"](TYPE_BIT, pb)
    if spec["order"]:
        ov = sc[spec["order"]]
        ob = pb.copy()
        ob[0] = 1
        ob[1:] |= np.array([ov[i] != ov[i - 1] for i in range(1, n)], np.int8)
        O = api["mk"](TYPE_BIT, ob)
    rowsc = api["mk"](TYPE_LNG, np.arange(n, dtype=np.int64))

    def rows_bound(bnd, is_start):
        pre, sh, tp2, lim = bound_args(0, list(bnd[:2]) + [None], is_start, TYPE_LNG)
        return api["bounds"](rowsc, P, lim, pre, TYPE_LNG, tp2, 0, sh)

    def frame_bounds():
        if spec["rows"]:
            return rows_bound(spec["rows"][0], True), rows_bound(spec["rows"][1], False)
        s = rows_bound(["UNBOUNDED", None], True)
        if not spec["order"]:
            return s, rows_bound(["UNBOUNDED", None], False)
        pre, sh, tp2, lim = bound_args(2, ["CURRENT", 0, None], False, TYPE_BIT)
        return s, api["bounds"](O, P, lim, pre, TYPE_BIT, tp2, 2, sh)

    out_cols = []
    for it in c["items"]:
        if it["kind"] == "col":
            out_cols.append(sc[it["col"]])
            continue
        f = it["func"]
        b = btp = None
        if it["val"] is not None:
            b, btp = _sqlwin_col(api, types[it["val"]], sc[it["val"]])
        if f == "ntile":
            any_b = api["mk"](TYPE_INT, np.zeros(n, np.int32))
            a = it["args"][0]
            if "col" in a:
                nb, ntp = _sqlwin_col(api, types[a["col"]], sc[a["col"]])
                r, rtp = api["ntile"](any_b, P, nb, None, ntp), ntp
            else:
                k = NILV[TYPE_INT] if a["lit"] is None else a["lit"]
                r, rtp = api["ntile"](any_b, P, None, k, TYPE_INT), TYPE_INT
        elif f in ("first_value", "last_value"):
            s, e = frame_bounds()
            r, rtp = api[f](b, s, e), btp
        elif f == "nth_value":
            s, e = frame_bounds()
            a = it["args"][0]
            if "col" in a:
                t, _ = _sqlwin_col(api, "lng", sc[a["col"]])
                r = api["nth_value"](b, s, e, t, None)
            else:
                r = api["nth_value"](b, s, e, None, NILV[TYPE_LNG] if a["lit"] is None else a["lit"])
            rtp = btp
        elif f in ("lag", "lead"):
            k, dflt, fn = 1, None, f
            if it["args"]:
                a = it["args"][0]
                if "col" in a:
                    raise NotImplementedError("offset from a column")
                k = a["lit"]
            if len(it["args"]) > 1:
                dflt = it["args"][1]["lit"]
                dflt = None if dflt is None else (float(dflt) if btp in (8, 9) else int(dflt))
            if k is None:
                k = api["BUN_NONE"]
            elif k < 0:
                k, fn = -k, ("lead" if f == "lag" else "lag")
            dv = (float("nan") if btp in (8, 9) else NILV[btp]) if dflt is None else dflt
            r, rtp = api[fn](b, P, k, dv), btp
        else:
            if spec["rows"]:
                s, e = frame_bounds()
                ft = 0
            else:
                s = e = None
                ft = 3 if spec["order"] else 5
            if f in ("min", "max"):
                r, rtp = api[f](b, P, O, s, e, ft), btp
            elif f == "sum":
                rtp = btp if btp in (8, 9) else TYPE_LNG
                r = api["sum"](b, P, O, s, e, rtp, ft)
            elif f in SQL_STATS:
                b2 = None
                if f in ("covar_samp", "covar_pop", "corr"):
                    if "col" not in it["args"][0]:
                        raise NotImplementedError("a literal second argument")
                    b2, _ = _sqlwin_col(api, types[it["args"][0]["col"]], sc[it["args"][0]["col"]])
                r, rtp = api["stat"](SQL_STATS[f], b, b2, P, O, s, e, ft), 9
            elif f == "prod":
                rtp = btp if btp in (8, 9) else TYPE_LNG
                r = api["prod"](b, P, O, s, e, rtp, ft)
            elif f == "count":
                if b is None:
                    b = api["mk"](TYPE_INT, np.zeros(n, np.int32))
                r, rtp = api["count"](b, P, O, s, e, it["val"] is not None, ft), TYPE_LNG
            else:
                r, rtp = api["avg"](b, P, O, s, e, ft), 9
        vals = _sqlwin_out(r, rtp)
        if it["wrap"] == "floor":
            vals = [None if v is None else float(np.floor(v)) for v in vals]
        out_cols.append(vals)
    return [list(r) for r in zip(*out_cols)]


def _sqlwin_fmt(row, types):
    return tuple("NULL" if v is None else ("%.3f" % v if t == "R" else str(int(v))) for v, t in zip(row, types))


def replay_window_sqltests(api):
    """Every kept window query of analytics00 / 01 / 02.test; returns
    (cases run, mismatches)."""
    bad, ran = [], 0
    for fx in FIX["window_sqltests"]:
        for c in fx["cases"]:
            tb = fx["tables"][c["table"]]
            try:
                got = sqlwin_eval(api, tb, c)
            except NotImplementedError:
                continue
            ran += 1
            g = [_sqlwin_fmt(r, c["types"]) for r in got]
            w = [_sqlwin_fmt(r, c["types"]) for r in c["expected"]]
            if c["sortmode"] == "rowsort" or c["spec"] is None:
                g, w = sorted(g), sorted(w)
            if g != w:
                bad.append((fx["source"], c["table"], c["items"], c["spec"], w, g))
    return ran, bad
