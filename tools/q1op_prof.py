"""Q1 through the GDK operators (mgdk_q1_opatatime) on SF100 lineitem, for a
kernel trace: python tools/q1op_prof.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from monetdb_amd import gdk  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    gdk.init(0)
    n = 600_121_500
    cols = gdk.tpch_lineitem(20241024, 0, n, 20_000_000)
    dmax = (((1998 + 4712) * 12 + 9 - 1) << 5) | 2      # GDK date of 1998-09-02 (bench.py mkdate)
    gdk.q1_fused(cols, dmax, fused=False)
    gdk.sync()
    t = time.perf_counter()
    for _ in range(reps):
        gdk.q1_fused(cols, dmax, fused=False)
    gdk.sync()
    print("q1 op-at-a-time ms", (time.perf_counter() - t) / reps * 1e3)


if __name__ == "__main__":
    main()
