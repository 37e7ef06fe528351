"""Hash-join device time over build-side sizes (config-3 key shapes: sparse
unique o_orderkey-like build keys, 1-7 probe rows per key, both shuffled).
Run once per path selection (MGDK_JOIN_GT=0/1) to find the crossover.

    python tools/join_sweep.py [--sizes 100000 ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from monetdb_amd import gdk  # noqa: E402
from opbench import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", nargs="*", type=int,
                    default=[70_000, 150_000, 300_000, 600_000, 1_500_000, 4_000_000, 15_000_000])
    ap.add_argument("--lng", action="store_true", help="8-byte keys (the open-addressing path)")
    a = ap.parse_args()
    dt, tp = (np.int64, gdk.TYPE_lng) if a.lng else (np.int32, gdk.TYPE_int)
    gdk.init(0)
    out = {}
    for nr in a.sizes:
        r = np.random.default_rng(3)
        i = np.arange(nr, dtype=np.int64)
        okeys = ((i // 8) * 32 + (i % 8) + 1).astype(dt)
        r.shuffle(okeys)
        lkeys = np.repeat(okeys, r.integers(1, 8, nr)).astype(dt)
        r.shuffle(lkeys)
        L = gdk.BAT.from_numpy(tp, lkeys, sorted_=False, revsorted=False, key=False, nonil=True)
        R = gdk.BAT.from_numpy(tp, okeys, sorted_=False, revsorted=False, key=True, nonil=True)
        _, wall, kms = timed(lambda: gdk.BATjoin(L, R), reps=5, kernels=("join",))
        out[nr] = {"probe_rows": int(lkeys.size), "wall_ms": round(wall, 4), "kernel_ms": round(kms, 4)}
        del L, R
        gdk.lib().mgdk_mem_release_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
