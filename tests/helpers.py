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
