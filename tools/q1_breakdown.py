"""Per-operator device time of the op-at-a-time TPC-H Q1 plan (the GDK API
path an unmodified MAL plan takes) at SF100 on one MI355X, checked against
the fused pass.

    python tools/q1_breakdown.py [--sf 100] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from monetdb_amd import gdk  # noqa: E402

OPS = ("select", "project", "group", "calc", "groupsum", "groupcount", "groupavg3", "sort", "q1_opatatime")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    n = int(6_001_215 * a.sf)
    cols = gdk.tpch_lineitem(1, 0, n, 20_000)
    from oracle import pyoracle as ora  # the checker: only for the date constant
    dmax = ora.mkdate(1998, 9, 2)
    fused = gdk.q1_fused(cols, dmax)
    op = gdk.q1_fused(cols, dmax, fused=False)
    key = lambda r: (r["returnflag"], r["linestatus"])
    same = sorted(fused, key=key) == sorted(op, key=key)
    gdk.sync()
    gdk.prof_reset()
    gdk.prof_enable(True)
    t = time.perf_counter()
    for _ in range(a.reps):
        gdk.q1_fused(cols, dmax, fused=False)
    wall = (time.perf_counter() - t) / a.reps * 1e3
    gdk.prof_enable(False)
    out = {"rows": n, "wall_ms": round(wall, 3), "fused_equals_opatatime": same}
    for k in OPS:
        ms, cnt = gdk.prof_get(k)
        out[k] = {"ms": round(ms / a.reps, 3), "calls": cnt // a.reps}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
