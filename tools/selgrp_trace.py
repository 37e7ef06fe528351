"""Config-1 thetaselect (100M int32, 1 / 10 % hits) and BATgroup (100M int32,
1000 groups) in a loop, for a rocprofv3 kernel trace: the trace's kernel
start / end stamps show each kernel's time and the gaps between the kernels
of one call (launches, host round trips).  Prints the library's own
event-window times (kernel_ms) per call for comparison.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/selgrp_trace.py
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monetdb_amd import gdk  # noqa: E402


def main():
    gdk.init(0)
    n = 100_000_000
    r = np.random.default_rng(1)
    b = gdk.BAT.from_numpy(gdk.TYPE_int, r.integers(0, 1000, n, dtype=np.int32), sorted_=False, revsorted=False,
                           key=False, nonil=True)
    out = {}
    for thr, reps in ((10, 20), (100, 10), (500, 10)):
        gdk.BATthetaselect(b, None, thr, "<")
        gdk.prof_reset()
        gdk.prof_enable(True)
        t = time.perf_counter()
        for _ in range(reps):
            s = gdk.BATthetaselect(b, None, thr, "<")
            del s
        wall = (time.perf_counter() - t) / reps * 1e3
        ms, k = gdk.prof_get("select")
        gdk.prof_enable(False)
        out["select_lt%d" % thr] = {"wall_ms": round(wall, 4), "kernel_ms": round(ms / max(1, k), 4)}
    gdk.BATgroup(b)
    gdk.prof_reset()
    gdk.prof_enable(True)
    t = time.perf_counter()
    for _ in range(10):
        res = gdk.BATgroup(b)
        del res
    wall = (time.perf_counter() - t) / 10 * 1e3
    ms, k = gdk.prof_get("group")
    gdk.prof_enable(False)
    out["group_1000"] = {"wall_ms": round(wall, 4), "kernel_ms": round(ms / max(1, k), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
