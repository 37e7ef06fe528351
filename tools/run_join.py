"""BATjoin config 3 (60M probe x 15M unique build, shuffled) for profiling
runs: python tools/run_join.py [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monetdb_amd import gdk  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
gdk.init(0)
r = np.random.default_rng(5)
ok = (np.arange(15_000_000, dtype=np.int64) // 8) * 32 + (np.arange(15_000_000) % 8) + 1
ok = ok.astype(np.int32)
lk = np.repeat(ok, 4)
r.shuffle(ok)
r.shuffle(lk)
L = gdk.BAT.from_numpy(gdk.TYPE_int, lk, sorted_=False, revsorted=False, key=False, nonil=True)
R = gdk.BAT.from_numpy(gdk.TYPE_int, ok, sorted_=False, revsorted=False, key=True, nonil=True)
for _ in range(reps):
    a, b = gdk.BATjoin(L, R)
    del a, b
gdk.sync()
print("ok")
