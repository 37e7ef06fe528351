"""Per-operator measurements for the BASELINE.json configs on one MI355X.

Each entry reports the device kernel time (HIP events on the library stream,
summed over the op's kernels), the wall time of the GDK call, Grows/s and the
algorithmic GB/s of SURVEY.md §8(d).

    python tools/opbench.py [--quick]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from monetdb_amd import gdk  # noqa: E402

HBM_PEAK = 8000.0


def timed(fn, reps=5, kernels=()):
    fn()
    gdk.prof_reset()
    gdk.prof_enable(True)
    t = time.perf_counter()
    out = None
    for _ in range(reps):
        out = None          # release the previous result (its HBM returns to the cache)
        out = fn()
    wall = (time.perf_counter() - t) / reps * 1e3
    gdk.prof_enable(False)
    kms = 0.0
    for k in kernels:
        ms, n = gdk.prof_get(k)
        kms += ms / max(1, reps)
    gdk.prof_reset()
    return out, wall, kms


def entry(rows, nbytes, wall, kms, **kw):
    t = kms if kms > 0 else wall
    d = {"rows": rows, "wall_ms": round(wall, 3), "kernel_ms": round(kms, 3),
         "grows_per_s": round(rows / wall / 1e6, 2),
         "algorithmic_GB": round(nbytes / 1e9, 3),
         "hbm_gbs": round(nbytes / t / 1e6, 1), "roofline_frac": round(nbytes / t / 1e6 / HBM_PEAK, 4)}
    d.update(kw)
    return d


def config1_thetaselect(n=100_000_000):
    r = np.random.default_rng(1)
    vals = r.integers(0, 1000, n, dtype=np.int32)
    b = gdk.BAT.from_numpy(gdk.TYPE_int, vals, sorted_=False, revsorted=False, key=False, nonil=True)
    out = {}
    for thr, name in ((10, "1pct"), (100, "10pct"), (500, "50pct")):
        res, wall, kms = timed(lambda: gdk.BATthetaselect(b, None, thr, "<"), kernels=("select",))
        hits = res.count()
        out[name] = entry(n, n * 4 + hits * 8, wall, kms, hits=hits)
    return out


def config2_q6(sf=10):
    rows = int(round(sf * 6_001_215))
    cols = gdk.tpch_lineitem(7, 0, rows, int(sf * 200_000))
    mk = lambda y, m, d: (((y + 4712) * 12 + m - 1) << 5) | d
    args = (cols["shipdate"], cols["discount"], cols["quantity"], cols["extendedprice"],
            mk(1994, 1, 1), mk(1995, 1, 1), 5, 7, 2400)
    _, wall, kms = timed(lambda: gdk.q6_fused(*args), kernels=("q6_fused",))
    # the fused Q6 is a predicate cascade: it reads shipdate whole and only
    # the 128-B lines of the other columns that hold a qualifying row
    lines = gdk.q6_last_lines()
    fused = entry(rows, rows * 4 + lines * 128 if lines else rows * 28, wall, kms, bytes_full_read=rows * 28,
                  kernel="k_q6s" if lines else "k_q6c")
    _, wall2, kms2 = timed(lambda: gdk.q6_opatatime(*args), reps=3,
                           kernels=("select", "project", "calc", "sum"))
    op = entry(rows, rows * 28, wall2, kms2)
    return {"sf": sf, "fused": fused, "op_at_a_time": op}


def config3_hashjoin(sf=10):
    r = np.random.default_rng(3)
    n_orders = int(sf * 1_500_000)
    i = np.arange(n_orders, dtype=np.int64)
    okeys = ((i // 8) * 32 + (i % 8) + 1).astype(np.int32)   # first 8 of every 32 (TPC-H)
    r.shuffle(okeys)
    lines = r.integers(1, 8, n_orders)
    lkeys = np.repeat(okeys, lines).astype(np.int32)
    r.shuffle(lkeys)
    nl = lkeys.shape[0]
    L = gdk.BAT.from_numpy(gdk.TYPE_int, lkeys, sorted_=False, revsorted=False, key=False, nonil=True)
    R = gdk.BAT.from_numpy(gdk.TYPE_int, okeys, sorted_=False, revsorted=False, key=True, nonil=True)
    res, wall, kms = timed(lambda: gdk.BATjoin(L, R), reps=3, kernels=("join",))
    nout = res[0].count()
    return entry(nl, 4 * (nl + n_orders) + 16 * nout, wall, kms, probe_rows=nl, build_rows=n_orders,
                 matches=nout)


def config4_q1(sf=100):
    rows = int(round(sf * 6_001_215))
    cols = gdk.tpch_lineitem(7, 0, rows, int(sf * 200_000))
    dmax = (((1998 + 4712) * 12 + 9 - 1) << 5) | 2
    res, wall, kms = timed(lambda: gdk.q1_fused(cols, dmax), kernels=("q1_fused",))
    fused = entry(rows, rows * 38, wall, kms, groups=len(res))
    out = {"sf": sf, "fused": fused}
    if sf <= 10:
        _, wall2, kms2 = timed(lambda: gdk.q1_fused(cols, dmax, fused=False), reps=2,
                               kernels=("select", "project", "group", "calc", "groupsum",
                                        "groupcount"))
        out["op_at_a_time"] = entry(rows, rows * 38, wall2, kms2)
    return out


def config4_group_sums(sf=100):
    """the config-4 leg's local step: GROUP BY an l_orderkey-shaped key (4
    rows per key, ordered) with exact sums of l_quantity and
    l_extendedprice (mgdk_group_sums_ordered); bytes: 24 per row read, 56
    per group written"""
    rows = int(round(sf * 6_001_215))
    cols = gdk.tpch_lineitem(7, 0, rows, int(sf * 200_000))
    okey = gdk.BATconvert(gdk.BAT.dense(0, rows), None, gdk.TYPE_lng)
    okey = gdk.BATcalcdivmod("/", okey, None, gdk.TYPE_lng, c2=4, t2=gdk.TYPE_lng)
    okey.s.tsorted, okey.s.trevsorted, okey.s.tkey, okey.s.tnonil = 1, 0, 0, 1
    vals = [cols["quantity"], cols["extendedprice"]]
    res, wall, kms = timed(lambda: gdk.group_sums_ordered(okey, vals), reps=5, kernels=("group_sums_ordered",))
    ng = res[0].count()
    return entry(rows, rows * 24 + ng * 56, wall, kms, groups=ng)


def config5_window(n=1_000_000_000, plen=100_000, limit=100):
    v, p = gdk.gen_window_column(5, n, plen)
    res, wall, kms = timed(lambda: gdk.GDKanalyticalwindowbounds(v, p, limit, True), reps=3,
                           kernels=("windowbounds",))
    out = entry(n, 17 * n, wall, kms, partitions=n // plen, limit=limit)
    # the frame's SUM (RANGE BETWEEN limit PRECEDING AND limit FOLLOWING) over
    # the same column, hge result: s, e bounds in, 8 B value + 16 B sum per row
    e = gdk.GDKanalyticalwindowbounds(v, p, limit, False)
    _, wall2, kms2 = timed(lambda: gdk.GDKanalyticalsum(v, p, None, res, e, gdk.TYPE_hge, 1), reps=3,
                           kernels=("analyticalsum",))
    out["frame_sum_hge"] = entry(n, n * (8 + 8 + 8 + 16), wall2, kms2)
    return out


def other_ops(n=100_000_000):
    r = np.random.default_rng(9)
    out = {}
    vals = r.integers(0, 1 << 30, n, dtype=np.int32)
    b = gdk.BAT.from_numpy(gdk.TYPE_int, vals, sorted_=False, revsorted=False, key=False, nonil=True)
    def sort_step():
        # drop the order index the previous sort left (it would answer the next)
        gdk.OIDXdestroy(b)
        return gdk.BATsort(b)
    _, wall, kms = timed(sort_step, reps=3, kernels=("sort",))
    out["sort_int32"] = entry(n, n * (4 + 4 + 8), wall, kms)
    g = r.integers(0, 1000, n, dtype=np.int32)
    gb = gdk.BAT.from_numpy(gdk.TYPE_int, g, sorted_=False, revsorted=False, key=False, nonil=True)
    res, wall, kms = timed(lambda: gdk.BATgroup(gb), reps=3, kernels=("group",))
    out["group_int32_1000"] = entry(n, n * (4 + 8), wall, kms, groups=res[1].count())
    lo = np.sort(r.choice(n, n // 10, replace=False)).astype(np.uint64)
    lb = gdk.BAT.from_numpy(gdk.TYPE_oid, lo, sorted_=True, revsorted=False, key=True, nonil=True)
    _, wall, kms = timed(lambda: gdk.BATproject(lb, b), kernels=("project",))
    out["project_10pct_int32"] = entry(n // 10, (n // 10) * (8 + 4 + 4), wall, kms)
    return out


def run(quick=False, only=None):
    gdk.init(0)
    res = {}
    for name, fn in (("config1_thetaselect_100M_int32", config1_thetaselect),
                     ("config2_q6_sf10", config2_q6),
                     ("config3_hashjoin_sf10", config3_hashjoin),
                     ("config4_q1_sf100", config4_q1),
                     ("config4_group_sums_sf100", config4_group_sums),
                     ("config5_window_range_1B", (lambda: config5_window(200_000_000)) if quick
                      else config5_window),
                     ("other_ops", other_ops)):
        if only and not any(o in name for o in only):
            continue
        try:
            res[name] = fn()
        except Exception as e:  # noqa: BLE001
            res[name] = {"error": str(e)}
        gdk.lib().mgdk_mem_release_cache()
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", nargs="*", default=None)
    a = ap.parse_args()
    print(json.dumps(run(a.quick, a.only), indent=1))
