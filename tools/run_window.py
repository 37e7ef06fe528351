"""One RANGE window bound computation over BASELINE config 5 (1B rows) for
profiling runs: python tools/run_window.py [n] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monetdb_amd import gdk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
gdk.init(0)
v, p = gdk.gen_window_column(5, n, 100_000)
for _ in range(reps):
    r = gdk.GDKanalyticalwindowbounds(v, p, 100, True)
    del r
print("ok")
