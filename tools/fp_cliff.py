"""Times the order-dependent float folds on one huge group / partition:
the bit-exact one-lane replay (fp_parallel_min = never) against the parallel
form (the default from 2^20 rows), with the oracle's sequential C loop on a
10M-row sample beside them.

    python tools/fp_cliff.py [rows]      -> one JSON object on stdout
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from monetdb_amd import gdk  # noqa: E402
from oracle import pyoracle as ora  # noqa: E402


def timed(fn, reps):
    fn()
    gdk.sync()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    gdk.sync()
    return out, (time.perf_counter() - t) / reps * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    par_only = len(sys.argv) > 2 and sys.argv[2] == "par"     # profiling runs: no replay, no oracle
    ns = min(n, 10_000_000)
    gdk.init(0)
    r = np.random.default_rng(5)
    x = r.standard_normal(n) * 100.0 + 50.0
    B = gdk.BAT.from_numpy(gdk.TYPE_dbl, x, sorted_=False, revsorted=False, key=False)
    OS = ora.Bat.from_array(ora.TYPE_dbl, x[:ns])
    g = gdk.BATconstant(gdk.TYPE_oid, 0, n)
    e = gdk.BAT.dense(0, 1)
    o = np.zeros(n, np.int8)
    o[::16] = 1                       # peer groups of 16 rows
    O = gdk.BAT.from_numpy(gdk.TYPE_bit, o)
    ops = {
        "stdev_population": (lambda: gdk.BATcalcvariance(B, False, stdev=True)[0],
                             lambda: ora.BATcalcstat("stdev", OS, None, False)[0]),
        "groupavg_one_group": (lambda: float(gdk.BATgroupavg(B, g, e, True)[0].to_numpy()[0]),
                               lambda: float(np.asarray(ora.BATgroupavg(
                                   OS, ora.Bat.from_array(ora.TYPE_oid, np.zeros(ns, np.uint64)),
                                   ora.Bat.dense(0, 1), True)[0].values())[0])),
        "running_sum_unpartitioned": (lambda: gdk.GDKanalyticalsum(B, None, O, None, None, gdk.TYPE_dbl, 3),
                                      lambda: ora.analyticalsum(OS, None, ora.Bat.from_array(ora.TYPE_bit, o[:ns]),
                                                                None, None, ora.TYPE_dbl, 3)),
    }
    res = {"rows": n, "oracle_sample_rows": ns}
    for name, (dev, orf) in ops.items():
        par, ms_par = timed(dev, 5)
        if par_only:
            res[name] = {"parallel_ms": round(ms_par, 3)}
            print(json.dumps({name: res[name]}), file=sys.stderr, flush=True)
            continue
        prev = gdk.set_fp_parallel_min(None)
        try:
            seq, ms_seq = timed(dev, 1)
        finally:
            gdk.set_fp_parallel_min(prev)
        t = time.perf_counter()
        orf()
        ms_ora = (time.perf_counter() - t) * 1e3 * n / ns
        d = {"replay_ms": round(ms_seq, 3), "parallel_ms": round(ms_par, 3),
             "oracle_ms_scaled": round(ms_ora, 1)}
        if isinstance(seq, float):
            d["replay"] = seq
            d["parallel"] = par
            d["diff_ulp"] = float(abs(seq - par) / np.spacing(abs(seq))) if seq == seq else None
        else:
            a, b = seq.to_numpy(), par.to_numpy()
            d["max_abs_diff"] = float(np.nanmax(np.abs(a - b)))
            d["max_abs_value"] = float(np.nanmax(np.abs(a)))
        res[name] = d
        print(json.dumps({name: d}), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
