#!/usr/bin/env python3
"""Benchmark: TPC-H Q6 (and Q1) column pipelines on MI355X, Grows/s + HBM roofline.

One step = one pass of the fused Q6 pipeline over this GPU's lineitem shard
(SF100 = 600,037,902 rows per GPU, columns resident in HBM): select(shipdate)
-> select(discount) -> thetaselect(quantity) -> project -> price*discount (hge)
-> sum, plus the exact combine of the per-GPU revenues.  Shards are independent
row ranges (weak scaling); the only cross-GPU step is gathering the 16-byte
partial revenues.

    python bench.py [--gpus N --steps K --warmup W --sf 100]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.  The `roofline` object prices the dominant kernel
(k_q6) from HIP events on the library stream; `cpu_baseline` times the CPU
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
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

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
        gdk.sync()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    def combine(rev):
        if dist is None:
            return rev
        import torch
        t = torch.tensor([rev & ((1 << 64) - 1), (rev >> 64) & ((1 << 64) - 1)],
                         dtype=torch.uint64).view(torch.int64).cuda()
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        tot = 0
        for o in out:
            w = o.cpu().view(torch.uint64).tolist()
            tot += gdk.hge_to_int(w)
        return tot

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
        e = torch.tensor([elapsed], dtype=torch.float64).cuda()
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    # kernel time from HIP events around k_q6 on the library stream
    gdk.prof_reset()
    gdk.prof_enable(True)
    nprof = max(5, min(args.steps, 20))
    for _ in range(nprof):
        gdk.q6_fused(*qargs)
    ms_total, launches = gdk.prof_get("q6_fused")
    gdk.prof_enable(False)
    kern_ms = ms_total / max(1, launches)

    extra = {}
    if not args.no_q1 and rank == 0:
        dmax = mkdate(1998, 9, 2)
        gdk.q1_fused(cols, dmax)
        gdk.prof_reset()
        gdk.prof_enable(True)
        t = time.perf_counter()
        for _ in range(5):
            q1 = gdk.q1_fused(cols, dmax)
        q1_ms = (time.perf_counter() - t) / 5 * 1e3
        q1k, q1n = gdk.prof_get("q1_fused")
        gdk.prof_enable(False)
        extra["q1"] = {"ms_per_step": round(q1_ms, 3), "grows_per_s": round(rows / q1_ms / 1e6, 2),
                       "kernel_ms": round(q1k / max(1, q1n), 3),
                       "hbm_gbs": round(rows * Q1_BYTES_PER_ROW / (q1k / max(1, q1n)) / 1e6, 1),
                       "groups": len(q1)}
        # the same Q6 plan operator by operator through the GDK C ABI
        r_op = gdk.q6_opatatime(*qargs)
        t = time.perf_counter()
        for _ in range(3):
            r_op = gdk.q6_opatatime(*qargs)
        op_ms = (time.perf_counter() - t) / 3 * 1e3
        assert r_op == gdk.q6_fused(*qargs)
        extra["q6_op_at_a_time"] = {"ms_per_step": round(op_ms, 3),
                                    "grows_per_s": round(rows / op_ms / 1e6, 2)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args)

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        total_rows = rows * world
        achieved = rows * Q6_BYTES_PER_ROW / (kern_ms * 1e-3) / 1e9
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
                         "traffic": None, "kernel": "k_q6", "kernel_ms": round(kern_ms, 4),
                         "bytes_per_launch": rows * Q6_BYTES_PER_ROW},
            "cpu_baseline": cpu,
            "revenue": str(revenue),
            "gen_s": round(gen_s, 3),
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(args):
    """Oracle Q6 op-at-a-time on the host cores over a bounded sample."""
    try:
        from oracle import pyoracle as ora
        ora.lib()
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "Grows/s", "cores": 0, "kind": "port",
                "sample": "oracle unavailable: %s" % e}
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    n = int(round(args.cpu_sf * SF1_ROWS))
    cols = ora.tpch_lineitem(20241024, 0, n, max(1, int(args.cpu_sf * 200_000)))
    ora.q6(cols, threads)
    times = []
    for _ in range(5):
        t = time.perf_counter()
        ora.q6(cols, threads)
        times.append(time.perf_counter() - t)
    med = statistics.median(times)
    return {"value": round(n / med / 1e9, 4), "unit": "Grows/s", "cores": threads, "kind": "port",
            "sample": "TPC-H Q6 op-at-a-time (oracle GDK restatement), %d rows (SF%g), "
                      "%d threads, median of 5" % (n, args.cpu_sf, threads),
            "ms": round(med * 1e3, 2)}


if __name__ == "__main__":
    main()
