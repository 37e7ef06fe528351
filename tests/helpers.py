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
