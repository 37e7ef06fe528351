"""Config-3 BATjoin (60M probe x 15M unique build, shuffled) wall time per
environment variant, one child process per variant (the knobs are read once
per process): python tools/join_variants.py 'MGDK_JOIN_CGT=0' 'MGDK_JOIN_CK=64' ..."""
import json
import os
import subprocess
import sys
import time

CHILD = r'''
import os, sys, time, json
import numpy as np
sys.path.insert(0, os.environ["REPO"])
from monetdb_amd import gdk
gdk.init(0)
r = np.random.default_rng(3)
n = 15_000_000
i = np.arange(n, dtype=np.int64)
ok = ((i // 8) * 32 + (i % 8) + 1).astype(np.int32)
r.shuffle(ok)
lk = np.repeat(ok, r.integers(1, 8, n)).astype(np.int32)
r.shuffle(lk)
L = gdk.BAT.from_numpy(gdk.TYPE_int, lk, sorted_=False, revsorted=False, key=False, nonil=True)
R = gdk.BAT.from_numpy(gdk.TYPE_int, ok, sorted_=False, revsorted=False, key=True, nonil=True)
ts = []
for k in range(7):
    gdk.sync()
    t0 = time.perf_counter()
    a, b = gdk.BATjoin(L, R)
    gdk.sync()
    ts.append(time.perf_counter() - t0)
    if k == 0:
        cnt = a.count()
        # spot check: keys equal at matched positions
        av, bv = a.to_numpy()[:100000], b.to_numpy()[:100000]
        assert np.array_equal(lk[av.astype(np.int64)], ok[bv.astype(np.int64)])
        assert np.all(np.diff(av.astype(np.int64)) > 0)
    del a, b
print(json.dumps({"ms": sorted(ts)[len(ts) // 2] * 1e3, "min_ms": min(ts) * 1e3, "pairs": cnt, "probe": int(lk.size)}))
'''


def main():
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for v in sys.argv[1:] or [""]:
        env = dict(os.environ, REPO=repo)
        for kv in v.split():
            k, _, x = kv.partition("=")
            env[k] = x
        t0 = time.time()
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        out = p.stdout.strip().splitlines()
        print(json.dumps({"variant": v, "rc": p.returncode, "res": out[-1] if out else p.stderr[-800:],
                          "s": round(time.time() - t0, 1)}), flush=True)
        if p.returncode != 0:
            sys.exit(p.returncode)


if __name__ == "__main__":
    main()
