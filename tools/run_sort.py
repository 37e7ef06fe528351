"""BATsort of 100M random int32 (with order and groups) for profiling runs:
python tools/run_sort.py [n] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monetdb_amd import gdk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
gdk.init(0)
vals = np.random.default_rng(9).integers(0, 1 << 30, n, dtype=np.int32)
b = gdk.BAT.from_numpy(gdk.TYPE_int, vals, sorted_=False, revsorted=False, key=False, nonil=True)
for _ in range(reps):
    gdk.OIDXdestroy(b)   # the previous sort's order index would answer
    r = gdk.BATsort(b)
    del r
gdk.sync()
print("ok")
