#!/usr/bin/env python3
"""Benchmark: TPC-H Q6 (and Q1) column pipelines on MI355X, Grows/s + HBM roofline.

One step = one pass of the fused Q6 pipeline over this GPU's lineitem shard
(SF100 = 600,121,500 rows per GPU, columns resident in HBM): select(shipdate)
-> select(discount) -> thetaselect(quantity) -> project -> price*discount (hge)
-> sum, plus the exact combine of the per-GPU revenues.  Shards are independent
row ranges (weak scaling); the only cross-GPU step is gathering the 16-byte
partial revenues.

    python bench.py [--gpus N --steps K --warmup W --sf 100]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.  The `roofline` object prices the dominant kernel
(k_q6s, the predicate cascade: shipdate read whole, discount / quantity /
extendedprice read only in the 128-B lines holding a row that passed the
earlier predicates -- the lines the op-at-a-time plan's candidate lists touch)
from HIP events on the library stream, its bytes counted by the kernel itself
(`bytes_per_launch`; `bytes_full_read` is the 28 B/row of a full scan);
`cpu_baseline` times the CPU
oracle (oracle/, a restatement of the reference GDK operators, op-at-a-time
with mitosis-style threading) on a bounded sample of the same workload.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SF1_ROWS = 6_001_215          # lineitem rows at SF1
Q6_BYTES_PER_ROW = 28         # shipdate 4 + discount 8 + quantity 8 + price 8
Q1_BYTES_PER_ROW = 38         # shipdate 4 + flag 1 + status 1 + 4 x lng 8
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E peak (MI355X_MICROARCH.md)


def mkdate(y, m, d):
    return (((y + 4712) * 12 + m - 1) << 5) | d


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--sf", type=float, default=100.0, help="scale factor per GPU")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--no-q1", action="store_true", help="skip the Q1 side measurement")
    p.add_argument("--cpu-sf", type=float, default=20.0, help="CPU baseline sample scale factor")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) or gloo (rehearsal)")
    p.add_argument("--no-dist-legs", action="store_true",
                   help="skip the config-4 (l_orderkey group, all_to_all) and config-5 (RANGE bounds) legs")
    p.add_argument("--window-rows", type=int, default=1_000_000_000,
                   help="config 5: rows of the window column over ALL ranks (strong scaling)")
    p.add_argument("--leg-steps", type=int, default=3)
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    dev = "cpu"
    if world > 1:
        import torch
        import torch.distributed as dist
        ndev = torch.cuda.device_count()
        local = local % max(1, ndev)      # rehearsal: several ranks on one GPU (gloo)
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dev = "cuda:%d" % local
        import datetime
        # a rank stuck in a collective (another rank failed) ends the job
        # instead of waiting for the default 10 minutes
        dist.init_process_group(args.dist_backend, timeout=datetime.timedelta(seconds=240))

    from monetdb_amd import gdk
    gdk.init(local)

    rows = int(round(args.sf * SF1_ROWS))
    sf_parts = max(1, int(args.sf * 200_000))
    row0 = rank * rows
    t0 = time.time()
    cols = gdk.tpch_lineitem(20241024, row0, rows, sf_parts)
    gen_s = time.time() - t0

    d0, d1 = mkdate(1994, 1, 1), mkdate(1995, 1, 1)
    qargs = (cols["shipdate"], cols["discount"], cols["quantity"], cols["extendedprice"],
             d0, d1, 5, 7, 2400)

    def barrier():
        gdk.sync()                       # the library's HIP stream
        if dist is not None:
            if dev != "cpu":
                import torch
                torch.cuda.synchronize()     # torch's stream (collectives)
            dist.barrier()

    from monetdb_amd import dist as D

    def combine(rev):
        # exact 128-bit sum of the per-GPU partial revenues (all_gather of 16 B)
        return D.combine_hge(rev, dist, dev)

    def step():
        return combine(gdk.q6_fused(*qargs))

    for _ in range(args.warmup):
        step()
    barrier()
    t = time.perf_counter()
    for _ in range(args.steps):
        revenue = step()
    barrier()
    elapsed = time.perf_counter() - t
    if dist is not None:
        import torch
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    # kernel time from HIP events around the fused Q6 (k_q6s) on the library stream
    gdk.prof_reset()
    gdk.prof_enable(True)
    nprof = max(5, min(args.steps, 20))
    for _ in range(nprof):
        gdk.q6_fused(*qargs)
    ms_total, launches = gdk.prof_get("q6_fused")
    gdk.prof_enable(False)
    kern_ms = ms_total / max(1, launches)
    # bytes the launch had to read: shipdate whole + the counted column lines
    # (the cascade), or all four columns (a full-read variant)
    lines = gdk.q6_last_lines()
    q6_kernel = "k_q6s" if lines else "k_q6c"
    q6_bytes = rows * 4 + lines * 128 if lines else rows * Q6_BYTES_PER_ROW

    extra = {}
    if not args.no_q1:
        # Q1 over the same shards: fused pass per GPU + exact merge of the
        # per-GPU group partials (first-occurrence order over all rows)
        dmax = mkdate(1998, 9, 2)
        gdk.q1_fused(cols, dmax)
        barrier()
        t = time.perf_counter()
        for _ in range(5):
            q1 = D.combine_q1(gdk.q1_fused(cols, dmax), dist, dev, rows_per_rank=rows, rank=rank)
        barrier()
        q1_s = time.perf_counter() - t
        if dist is not None:
            import torch
            e = torch.tensor([q1_s], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            q1_s = float(e.item())
        q1_ms = q1_s / 5 * 1e3
        gdk.prof_reset()
        gdk.prof_enable(True)
        for _ in range(3):
            gdk.q1_fused(cols, dmax)
        q1k, q1n = gdk.prof_get("q1_fused")
        gdk.prof_enable(False)
        extra["q1"] = {"ms_per_step": round(q1_ms, 3),
                       "grows_per_s": round(rows * world / q1_ms / 1e6, 2),
                       "kernel_ms": round(q1k / max(1, q1n), 3),
                       "hbm_gbs_per_gpu": round(rows * Q1_BYTES_PER_ROW / (q1k / max(1, q1n)) / 1e6, 1),
                       "roofline_frac": round(rows * Q1_BYTES_PER_ROW / (q1k / max(1, q1n)) / 1e6
                                              / HBM_PEAK_GBS, 4),
                       "kernel": "k_q1n", "traffic": pmc_traffic("k_q1n", rows),
                       "groups": len(q1),
                       "count_order": sum(r["count_order"] for r in q1)}
    if not args.no_q1 and rank == 0:
        # the same Q6 plan operator by operator through the GDK C ABI
        r_op = gdk.q6_opatatime(*qargs)
        t = time.perf_counter()
        for _ in range(3):
            r_op = gdk.q6_opatatime(*qargs)
        op_ms = (time.perf_counter() - t) / 3 * 1e3
        assert r_op == gdk.q6_fused(*qargs)
        extra["q6_op_at_a_time"] = {"ms_per_step": round(op_ms, 3),
                                    "grows_per_s": round(rows / op_ms / 1e6, 2)}
        # the Q1 MAL plan operator by operator (select, group/subgroup,
        # projections, calc to hge, grouped sums / avg3 / count)
        dmax = mkdate(1998, 9, 2)
        q1_op = gdk.q1_fused(cols, dmax, fused=False)
        t = time.perf_counter()
        for _ in range(3):
            q1_op = gdk.q1_fused(cols, dmax, fused=False)
        op1_ms = (time.perf_counter() - t) / 3 * 1e3
        key = lambda r: (r["returnflag"], r["linestatus"])
        assert sorted((key(r), r["sum_charge"]) for r in q1_op) == \
            sorted((key(r), r["sum_charge"]) for r in gdk.q1_fused(cols, dmax))
        extra["q1_op_at_a_time"] = {"ms_per_step": round(op1_ms, 3),
                                    "grows_per_s": round(rows / op1_ms / 1e6, 2)}

    if not args.no_dist_legs:
        # a leg that fails (the same way on every rank) is reported in the
        # line instead of losing the headline measurement
        try:
            extra["config4_orderkey_group"] = leg_orderkey_group(args, gdk, D, dist, dev, cols, rows, row0, world,
                                                                 barrier)
        except Exception as ex:  # noqa: BLE001
            extra["config4_orderkey_group"] = {"error": str(ex)[:300]}
        del cols, qargs
        gdk.lib().mgdk_mem_release_cache()
        try:
            extra["config5_window_bounds"] = leg_window(args, gdk, D, dist, dev, rank, world, barrier)
        except Exception as ex:  # noqa: BLE001
            extra["config5_window_bounds"] = {"error": str(ex)[:300]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args)
        extra["cpu_baselines"] = cpu_baselines_other(args)

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        total_rows = rows * world
        achieved = q6_bytes / (kern_ms * 1e-3) / 1e9
        line = {
            "metric": "Grows/sec + HBM GB/s vs peak, TPC-H SF100 Q1/Q6 columns at 1/2/4/8 GPUs",
            "value": round(total_rows / (ms * 1e-3) / 1e9, 3),
            "unit": "Grows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (TPC-H distributions, counter-based generator in HBM)",
            "config": {"workload": "TPC-H Q6 fused column pipeline (select/select/thetaselect/"
                                   "project/mul->hge/sum), lineitem SF%g per GPU" % args.sf,
                       "rows_per_gpu": rows, "sf_per_gpu": args.sf,
                       "parallelism": "row-range shards x%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic(q6_kernel, rows), "kernel": q6_kernel,
                         "kernel_ms": round(kern_ms, 4),
                         "bytes_per_launch": q6_bytes,
                         "bytes_full_read": rows * Q6_BYTES_PER_ROW},
            "cpu_baseline": cpu,
            "revenue": str(revenue),
            "gen_s": round(gen_s, 3),
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _max_over_ranks(dist, dev, vals):
    if dist is None:
        return vals
    import torch
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu().tolist()]


def leg_orderkey_group(args, gdk, D, dist, dev, cols, rows, row0, world, barrier):
    """Config 4 with its exchange: GROUP BY an l_orderkey-shaped key (4
    lines per order, orders clustered as lineitem is) with exact sums of
    l_quantity and l_extendedprice, over the same SF100-per-GPU shards:
    local BATgroup + BATgroupsum, the partial rows hash-partitioned by key
    and shuffled with ONE RCCL all_to_all per column, merged on the owner,
    numbered in global first-occurrence order (opt_mergetable.c:1496-1885
    mat_group / mat_group_aggr).  Weak scaling (rows per GPU fixed)."""
    okey = gdk.BATconvert(gdk.BAT.dense(row0, rows, hseqbase=row0), None, gdk.TYPE_lng)
    okey = gdk.BATcalcdivmod("/", okey, None, gdk.TYPE_lng, c2=4, t2=gdk.TYPE_lng)
    okey.s.hseqbase = row0
    okey.s.tsorted, okey.s.trevsorted, okey.s.tkey, okey.s.tnonil = 1, 0, 0, 1
    vals = [cols["quantity"], cols["extendedprice"]]
    be = D.GdkBackend(dev)
    out = D.dist_group_aggr(be, dist, okey, vals)           # warm-up
    ngroups_local = out["gid"].count()
    del out
    barrier()
    D.STATS["exchange_s"] = 0.0
    t = time.perf_counter()
    for _ in range(args.leg_steps):
        out = D.dist_group_aggr(be, dist, okey, vals)
        del out
    barrier()
    tot = (time.perf_counter() - t) / args.leg_steps
    exch = D.STATS["exchange_s"] / args.leg_steps
    tot, exch, comp = _max_over_ranks(dist, dev, [tot, exch, tot - exch])
    ng = _gather_sum(dist, dev, ngroups_local)
    return {"ms_per_step": round(tot * 1e3, 3), "grows_per_s": round(rows * world / tot / 1e9, 3),
            "unit": "Grows/s", "exchange_ms": round(exch * 1e3, 3), "local_ms": round(comp * 1e3, 3),
            "groups": ng, "rows_per_gpu": rows, "scaling": "weak",
            "workload": "GROUP BY l_orderkey (4 lines/order) SUM(l_quantity), SUM(l_extendedprice): "
                        "dist_group_aggr, one all_to_all per partial column"}


def _gather_sum(dist, dev, v):
    if dist is None:
        return int(v)
    import torch
    t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return int(t.item())


def leg_window(args, gdk, D, dist, dev, rank, world, barrier, limit=100, plen=100_000):
    """Config 5: GDKanalyticalwindowbounds (RANGE 100 PRECEDING) over ONE
    column of --window-rows rows (1B) range-partitioned over the ranks
    (strong scaling); shards start at partition boundaries, so the move of
    rows to the partition's owner is empty and every rank computes its
    bounds locally (dist_window_bounds)."""
    n = args.window_rows // world
    v, p = gdk.gen_window_column(5 + rank, n, plen)
    v.s.hseqbase = p.s.hseqbase = rank * n
    be = D.GdkBackend(dev)
    r = D.dist_window_bounds(be, dist, v, p, limit, True)
    del r
    barrier()
    gdk.prof_reset()
    gdk.prof_enable(True)
    t = time.perf_counter()
    for _ in range(args.leg_steps):
        r = D.dist_window_bounds(be, dist, v, p, limit, True)
        del r
    barrier()
    tot = (time.perf_counter() - t) / args.leg_steps
    kms, kn = gdk.prof_get("windowbounds")
    gdk.prof_enable(False)
    kern = kms / max(1, kn) * 1e-3
    tot, kern = _max_over_ranks(dist, dev, [tot, kern])
    total_rows = n * world
    return {"ms_per_step": round(tot * 1e3, 3), "grows_per_s": round(total_rows / tot / 1e9, 3),
            "unit": "Grows/s", "kernel_ms": round(kern * 1e3, 3), "rows_total": total_rows,
            "rows_per_gpu": n, "partitions": total_rows // plen, "limit": limit, "scaling": "strong",
            "roofline_frac_kernel": round(17 * n / kern / 1e9 / HBM_PEAK_GBS, 4) if kern > 0 else None}


def pmc_traffic(kernel, rows):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json, made by tools/pmc_summary.py from
    separate --pmc FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled for
    gfx950's half-counted wide streaming reads), scaled to this row count."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))[kernel]
        return int(round(d["hbm_bytes_per_row"] * rows))
    except Exception:  # noqa: BLE001
        return None


def cpu_baseline(args):
    """Oracle Q6 op-at-a-time on the host cores over a bounded sample."""
    try:
        from oracle import pyoracle as ora
        ora.lib()
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "Grows/s", "cores": 0, "kind": "port",
                "sample": "oracle unavailable: %s" % e}
    # every core this process may run on (the GPU box grants one GPU's
    # share of the host; OMP_NUM_THREADS states that share there)
    nproc = os.cpu_count() or 1
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = args.cpu_threads or (min(share, avail) if share > 0 else avail)
    n = int(round(args.cpu_sf * SF1_ROWS))
    cols = ora.tpch_lineitem(20241024, 0, n, max(1, int(args.cpu_sf * 200_000)))
    ora.q6(cols, threads)
    times = []
    for _ in range(5):
        t = time.perf_counter()
        ora.q6(cols, threads)
        times.append(time.perf_counter() - t)
    med = statistics.median(times)
    # the same sample on one core (the reference's MAL plan runs the GDK
    # operators of one query single-threaded unless mitosis splits it)
    t1 = []
    for _ in range(3):
        t = time.perf_counter()
        ora.q6(cols, 1)
        t1.append(time.perf_counter() - t)
    med1 = statistics.median(t1)
    return {"value": round(n / med / 1e9, 4), "unit": "Grows/s", "cores": threads, "kind": "port",
            "nproc": nproc, "affinity_cpus": avail, "omp_num_threads": share or None,
            "sample": "TPC-H Q6 op-at-a-time (oracle GDK restatement), %d rows (SF%g), "
                      "%d threads, median of 5" % (n, args.cpu_sf, threads),
            "ms": round(med * 1e3, 2),
            "single_thread": {"value": round(n / med1 / 1e9, 4), "unit": "Grows/s", "cores": 1,
                              "ms": round(med1 * 1e3, 2), "sample": "same rows, median of 3"}}


def _cpu_quota():
    """The cgroup CPU quota of this process (cgroup v2 cpu.max), in CPUs."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:  # noqa: BLE001
        return None


def cpu_baselines_other(args):
    """CPU comparators (the oracle's restatement of the reference operators)
    for configs 3, 4 and 5 on bounded samples of the same workloads."""
    try:
        import numpy as np
        from oracle import pyoracle as ora
        ora.lib()
    except Exception as e:  # noqa: BLE001
        return {"error": "oracle unavailable: %s" % e}
    out = {"cgroup_cpu_quota": _cpu_quota(), "nproc": os.cpu_count()}
    r = np.random.default_rng(3)
    # config 3: BATjoin (hash path) lineitem x orders at SF1, single thread
    # (the reference's hashjoin is one thread per call)
    no = 1_500_000
    i = np.arange(no, dtype=np.int64)
    ok = ((i // 8) * 32 + (i % 8) + 1).astype(np.int32)
    r.shuffle(ok)
    lk = np.repeat(ok, r.integers(1, 8, no)).astype(np.int32)
    r.shuffle(lk)
    L = ora.Bat.from_array(ora.TYPE_int, lk, nonil=True)
    R = ora.Bat.from_array(ora.TYPE_int, ok, nonil=True, key=True)
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        ora.BATjoin(L, R)
        ts.append(time.perf_counter() - t)
    med = statistics.median(ts)
    out["config3_hashjoin"] = {"value": round(len(lk) / med / 1e9, 5), "unit": "Grows/s", "cores": 1,
                               "kind": "port", "ms": round(med * 1e3, 1),
                               "sample": "SF1: %d probe x %d unique shuffled build rows, median of 3"
                                         % (len(lk), no)}
    # config 4: Q1 op-at-a-time over an SF2 sample on the box's CPU share
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    n4 = 2 * SF1_ROWS
    cols = ora.tpch_lineitem(20241024, 0, n4, 400_000)
    ora.q1(cols, share)
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        ora.q1(cols, share)
        ts.append(time.perf_counter() - t)
    med = statistics.median(ts)
    out["config4_q1"] = {"value": round(n4 / med / 1e9, 5), "unit": "Grows/s", "cores": share, "kind": "port",
                         "ms": round(med * 1e3, 1),
                         "sample": "TPC-H Q1 op-at-a-time (oracle), SF2 = %d rows, %d threads, median of 3"
                                   % (n4, share)}
    # config 5: RANGE 100 PRECEDING bounds (the reference's walk), 2M rows
    n5 = 2_000_000
    v = np.cumsum(r.integers(0, 5, n5)).astype(np.int64)
    pb = np.zeros(n5, np.int8)
    pb[::100_000] = 1
    V = ora.Bat.from_array(ora.TYPE_lng, v, nonil=True, sorted_=True)
    P = ora.Bat.from_array(ora.TYPE_bit, pb)
    t = time.perf_counter()
    ora.rangebounds(V, P, 100, True)
    med = time.perf_counter() - t
    out["config5_rangebounds"] = {"value": round(n5 / med / 1e9, 5), "unit": "Grows/s", "cores": 1,
                                  "kind": "port", "ms": round(med * 1e3, 1),
                                  "sample": "%d rows, 20 partitions, limit 100, one run" % n5}
    # the same on the box's CPU share: whole partitions per thread (the
    # bounds never cross a partition), the oracle's C walk releases the GIL
    try:
        from concurrent.futures import ThreadPoolExecutor
        nparts = 8 * share
        n5m = nparts * 100_000
        vm = np.cumsum(r.integers(0, 5, n5m)).astype(np.int64)
        chunks = []
        per = nparts // share
        for k in range(share):
            lo, hi = k * per * 100_000, (k + 1) * per * 100_000
            pk = np.zeros(hi - lo, np.int8)
            pk[::100_000] = 1
            chunks.append((ora.Bat.from_array(ora.TYPE_lng, vm[lo:hi], nonil=True, sorted_=True),
                           ora.Bat.from_array(ora.TYPE_bit, pk)))
        with ThreadPoolExecutor(max_workers=share) as ex:
            t = time.perf_counter()
            list(ex.map(lambda c: ora.rangebounds(c[0], c[1], 100, True), chunks))
            med = time.perf_counter() - t
        out["config5_rangebounds_mt"] = {"value": round(n5m / med / 1e9, 5), "unit": "Grows/s", "cores": share,
                                         "kind": "port", "ms": round(med * 1e3, 1),
                                         "sample": "%d rows, %d partitions over %d threads, limit 100, one run"
                                                   % (n5m, nparts, share)}
    except Exception as e:  # noqa: BLE001
        out["config5_rangebounds_mt"] = {"error": str(e)[:200]}
    return out


if __name__ == "__main__":
    main()
