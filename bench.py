#!/usr/bin/env python3
"""Benchmark: TPC-H Q6 (and Q1) column pipelines on MI355X, Grows/s + HBM roofline.

One step = one pass of the fused Q6 pipeline over this GPU's lineitem shard
(SF100 = 600,121,500 rows per GPU, columns resident in HBM): select(shipdate)
-> select(discount) -> thetaselect(quantity) -> project -> price*discount (hge)
-> sum, plus the exact combine of the per-GPU revenues.  Shards are independent
row ranges (weak scaling); the only cross-GPU step is gathering the 16-byte
partial revenues.

    python bench.py [--gpus N --steps K --warmup W --sf 100]

With --gpus N > 1 and no WORLD_SIZE in the environment, this process starts N
fresh rank processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
one GPU each) before it touches any GPU, waits for them and exits with the
first failing rank's status; launched by torch.distributed.run it is one rank.

Rank 0 prints one JSON line.  The `roofline` object prices the dominant kernel
(k_q6s, the predicate cascade: shipdate read whole, discount / quantity /
extendedprice read only in the 128-B lines holding a row that passed the
earlier predicates -- the lines the op-at-a-time plan's candidate lists touch)
from HIP events on the library stream, its bytes counted by the kernel itself
(`bytes_per_launch`; `bytes_full_read` is the 28 B/row of a full scan);
`cpu_baseline` times the CPU oracle (oracle/, a restatement of the reference
GDK operators, op-at-a-time with mitosis-style threading) on a bounded sample
of the same workload.  Besides the headline, the line carries one leg per
BASELINE config (config1 thetaselect, Q1 = config 4's aggregation, config3 hash
join, config4 high-cardinality group with its exchange, config5 RANGE bounds)
and a `parity` object: the full-size results checked against the oracle
outside the timed regions (Q6 / Q1 per shard, the SF10 join's pairs, sampled
whole partitions of the 1B-row window bounds, the thetaselect oid lists).  A
parity mismatch makes the process exit non-zero after the line is printed.
"""
import argparse
import hashlib
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SF1_ROWS = 6_001_215          # lineitem rows at SF1
Q6_BYTES_PER_ROW = 28         # shipdate 4 + discount 8 + quantity 8 + price 8
Q1_BYTES_PER_ROW = 38         # shipdate 4 + flag 1 + status 1 + 4 x lng 8
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E peak (MI355X_MICROARCH.md)
SEED = 20241024


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
    p.add_argument("--no-parity", action="store_true", help="skip the full-size oracle checks")
    p.add_argument("--cpu-sf", type=float, default=20.0, help="CPU baseline sample scale factor")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) or gloo (rehearsal)")
    p.add_argument("--no-dist-legs", action="store_true",
                   help="skip the config-4 (l_orderkey group, all_to_all) and config-5 (RANGE bounds) legs")
    p.add_argument("--no-op-legs", action="store_true",
                   help="skip the config-1 (thetaselect) and config-3 (hash join) legs")
    p.add_argument("--window-rows", type=int, default=1_000_000_000,
                   help="config 5: rows of the window column over ALL ranks (strong scaling)")
    p.add_argument("--join-sf", type=float, default=10.0, help="config 3: scale factor of the join")
    p.add_argument("--select-rows", type=int, default=100_000_000,
                   help="config 1: rows of the int32 column over ALL ranks (strong scaling)")
    p.add_argument("--leg-steps", type=int, default=3)
    p.add_argument("--dry-dist", action="store_true",
                   help="launch and check the ranks and the process group, then exit (no GPU work)")
    return p.parse_args()


# ---------------------------------------------------------------------------
# launching N ranks (the parent never touches a GPU)
# ---------------------------------------------------------------------------

def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """Start n rank processes of this script (fresh interpreters; this
    process has made no HIP call and makes none) and wait for them.  When a
    rank fails the others are stopped -- they would wait in a collective for
    the failed one -- and its exit status is returned."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            st = p.poll()
            if st is None:
                continue
            live.remove(p)
            if st != 0 and rc == 0:
                rc = st
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc if rc >= 0 else 128 - rc


def sum_ranks(dist, dev, rank):
    import torch
    t = torch.tensor([rank], dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    return int(t.item())


# ---------------------------------------------------------------------------
# one rank
# ---------------------------------------------------------------------------

class Ctx:
    """What every leg needs: the rank, the process group, barriers."""

    def __init__(self, args, gdk, D, dist, dev, rank, world):
        self.args, self.gdk, self.D, self.dist, self.dev = args, gdk, D, dist, dev
        self.rank, self.world = rank, world

    def barrier(self):
        self.gdk.sync()                       # the library's HIP stream
        if self.dist is not None:
            if self.dev != "cpu":
                import torch
                torch.cuda.synchronize()      # torch's stream (collectives)
            self.dist.barrier()

    def max_over_ranks(self, vals):
        if self.dist is None:
            return vals
        import torch
        t = torch.tensor(vals, dtype=torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return [float(x) for x in t.cpu().tolist()]

    def sum_over_ranks(self, v):
        if self.dist is None:
            return int(v)
        return sum(self.D._s64(x[0]) for x in self.D._gather_int64(self.dist, self.dev, [int(v)]))

    def all_ok(self, ok):
        """True on every rank iff ok on every rank."""
        return self.max_over_ranks([0.0 if ok else 1.0])[0] == 0.0

    def leg(self, name, fn, out):
        """Run one leg on every rank; a failure on any rank is reported by all
        of them together (no rank moves on to the next leg's collectives
        while another is still in this one)."""
        err = None
        try:
            res = fn()
        except Exception as ex:  # noqa: BLE001
            err = "%s: %s" % (type(ex).__name__, str(ex)[:300])
            res = None
        if not self.all_ok(err is None):
            res = {"error": err or "failed on another rank"}
        out[name] = res
        return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
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
    seen = dist.get_world_size() if dist is not None else 1
    if seen != args.gpus:
        raise SystemExit("bench: --gpus %d but the process group has %d ranks" % (args.gpus, seen))
    if args.dry_dist:
        ranks = sum_ranks(dist, dev, rank) if dist is not None else 0
        if rank == 0:
            print(json.dumps({"n_gpus": seen, "world_size_seen": seen, "rank_sum": ranks,
                              "dist_backend": args.dist_backend if dist is not None else None}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    from monetdb_amd import dist as D
    from monetdb_amd import gdk
    gdk.init(local)
    cx = Ctx(args, gdk, D, dist, dev, rank, world)

    rows = int(round(args.sf * SF1_ROWS))
    sf_parts = max(1, int(args.sf * 200_000))
    row0 = rank * rows
    t0 = time.time()
    cols = gdk.tpch_lineitem(SEED, row0, rows, sf_parts)
    gen_s = time.time() - t0

    d0, d1 = mkdate(1994, 1, 1), mkdate(1995, 1, 1)
    qargs = (cols["shipdate"], cols["discount"], cols["quantity"], cols["extendedprice"],
             d0, d1, 5, 7, 2400)

    def step():
        # exact 128-bit sum of the per-GPU partial revenues (all_gather of 16 B)
        return D.combine_hge(gdk.q6_fused(*qargs), dist, dev)

    for _ in range(args.warmup):
        step()
    cx.barrier()
    t = time.perf_counter()
    for _ in range(args.steps):
        revenue = step()
    cx.barrier()
    elapsed = cx.max_over_ranks([time.perf_counter() - t])[0]

    # kernel time from HIP events around the fused Q6 (k_q6s) on the library stream
    gdk.prof_reset()
    gdk.prof_enable(True)
    nprof = max(5, min(args.steps, 20))
    for _ in range(nprof):
        part = gdk.q6_fused(*qargs)
    ms_total, launches = gdk.prof_get("q6_fused")
    gdk.prof_enable(False)
    kern_ms = cx.max_over_ranks([ms_total / max(1, launches)])[0]
    # bytes the launch had to read: shipdate whole + the counted column lines
    # (the cascade), or all four columns (a full-read variant)
    lines = gdk.q6_last_lines()
    q6_kernel = "k_q6s" if lines else "k_q6c"
    q6_bytes = rows * 4 + lines * 128 if lines else rows * Q6_BYTES_PER_ROW

    extra = {}
    parity = {}
    if not args.no_parity:
        cx.leg("q6", lambda: parity_q6(cx, part, row0, rows, sf_parts), parity)

    if not args.no_q1:
        q1_rows = cx.leg("q1", lambda: leg_q1(cx, cols, rows), extra)
        if not args.no_parity:
            cx.leg("q1", lambda: parity_q1(cx, cols, row0, rows, sf_parts), parity)
        del q1_rows
    if not args.no_q1:
        tmp = {}
        cx.leg("op", lambda: op_at_a_time(cx, cols, qargs) if rank == 0 else {}, tmp)
        extra.update(tmp["op"] if "error" not in tmp["op"] else {"op_at_a_time": tmp["op"]})

    if not args.no_dist_legs:
        cx.leg("config4_orderkey_group", lambda: leg_orderkey_group(cx, cols, rows, row0), extra)
    del cols, qargs
    gdk.lib().mgdk_mem_release_cache()
    if not args.no_op_legs:
        cx.leg("config1_thetaselect", lambda: leg_thetaselect(cx, parity), extra)
        gdk.lib().mgdk_mem_release_cache()
        cx.leg("config3_hashjoin", lambda: leg_hashjoin(cx, parity), extra)
        gdk.lib().mgdk_mem_release_cache()
    if not args.no_dist_legs:
        cx.leg("config5_window_bounds", lambda: leg_window(cx, parity), extra)
        gdk.lib().mgdk_mem_release_cache()
    if not args.no_op_legs:
        cx.leg("ops_sort_group", lambda: leg_sort_group(cx, parity), extra)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args)
        extra["cpu_baselines"] = cpu_baselines_other(args)

    # a parity entry is True only when it held on every rank (a check that
    # raised is reported as its error and counts as a mismatch)
    perr = {k: v["error"] for k, v in parity.items() if isinstance(v, dict)}
    parity = {k: v is True for k, v in parity.items()}
    parity = {k: cx.all_ok(v) for k, v in sorted(parity.items())}
    if perr:
        parity["errors"] = perr
    ok = all(v is True for k, v in parity.items() if k != "errors") and not perr
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        total_rows = rows * world
        achieved = q6_bytes / (kern_ms * 1e-3) / 1e9
        traffic, traffic_note = pmc_traffic(q6_kernel, rows)
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
            "dist_backend": args.dist_backend if world > 1 else None,
            "world_size_seen": dist.get_world_size() if dist is not None else 1,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_note, "kernel": q6_kernel,
                         "kernel_ms": round(kern_ms, 4),
                         "bytes_per_launch": q6_bytes,
                         "bytes_full_read": rows * Q6_BYTES_PER_ROW},
            "cpu_baseline": cpu,
            "revenue": str(revenue),
            "gen_s": round(gen_s, 3),
            "parity": parity if not args.no_parity else None,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


# ---------------------------------------------------------------------------
# legs
# ---------------------------------------------------------------------------

def _cpu_share():
    """Threads this rank may use on the host: OMP_NUM_THREADS (the GPU box's
    share per GPU), else the affinity set, divided among the local ranks."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    if share <= 0:
        share = max(1, avail // int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    return max(1, min(share, avail))


def parity_q6(cx, part, row0, rows, sf_parts, chunk=25_000_000):
    """This rank's partial Q6 revenue at full size against the oracle's
    op-at-a-time Q6 over the same generated rows (chunked: the generator is
    counter based, the revenue a sum)."""
    from oracle import pyoracle as ora
    ora.lib()
    th = _cpu_share()
    want = 0
    for lo in range(0, rows, chunk):
        c = ora.tpch_lineitem(SEED, row0 + lo, min(chunk, rows - lo), sf_parts)
        want += ora.q6(c, th)
        del c
    return part == want


def leg_q1(cx, cols, rows):
    """Q1 over the same shards: fused pass per GPU + exact merge of the
    per-GPU group partials (first-occurrence order over all rows)."""
    gdk, D = cx.gdk, cx.D
    dmax = mkdate(1998, 9, 2)
    gdk.q1_fused(cols, dmax)
    cx.barrier()
    # one timed pass: the wall clock and the HIP events around the fused
    # kernel come from the same five iterations
    gdk.prof_reset()
    gdk.prof_enable(True)
    t = time.perf_counter()
    for _ in range(5):
        q1 = D.combine_q1(gdk.q1_fused(cols, dmax), cx.dist, cx.dev, rows_per_rank=rows, rank=cx.rank)
    cx.barrier()
    q1_ms = (time.perf_counter() - t) / 5 * 1e3
    q1k, q1n = gdk.prof_get("q1_fused")
    gdk.prof_enable(False)
    q1_ms, kms = cx.max_over_ranks([q1_ms, q1k / max(1, q1n)])
    traffic, note = pmc_traffic("k_q1n", rows)
    return {"ms_per_step": round(q1_ms, 3),
            "grows_per_s": round(rows * cx.world / q1_ms / 1e6, 2),
            "kernel_ms": round(kms, 3),
            "hbm_gbs_per_gpu": round(rows * Q1_BYTES_PER_ROW / kms / 1e6, 1),
            "roofline_frac": round(rows * Q1_BYTES_PER_ROW / kms / 1e6 / HBM_PEAK_GBS, 4),
            "kernel": "k_q1n", "traffic": traffic, "traffic_source": note,
            "groups": len(q1),
            "count_order": sum(r["count_order"] for r in q1)}


def parity_q1(cx, cols, row0, rows, sf_parts, chunk=25_000_000):
    """This rank's fused Q1 group rows (exact sums, counts) at full size
    against the oracle's op-at-a-time Q1 over the same rows, chunk partials
    added exactly."""
    from oracle import pyoracle as ora
    ora.lib()
    th = _cpu_share()
    keys = ("sum_qty", "sum_base_price", "sum_disc_price", "sum_charge", "count_order")
    want = {}
    for lo in range(0, rows, chunk):
        c = ora.tpch_lineitem(SEED, row0 + lo, min(chunk, rows - lo), sf_parts)
        for r in ora.q1(c, th):
            w = want.setdefault((r["returnflag"], r["linestatus"]), dict.fromkeys(keys, 0))
            for k in keys:
                w[k] += r[k]
        del c
    got = {(r["returnflag"], r["linestatus"]): {k: r[k] for k in keys}
           for r in cx.gdk.q1_fused(cols, mkdate(1998, 9, 2))}
    return got == want


def op_at_a_time(cx, cols, qargs):
    """The same Q6 / Q1 plans operator by operator through the GDK C ABI
    (rank 0), checked against the fused results."""
    gdk = cx.gdk
    out = {}
    r_op = gdk.q6_opatatime(*qargs)
    t = time.perf_counter()
    for _ in range(3):
        r_op = gdk.q6_opatatime(*qargs)
    op_ms = (time.perf_counter() - t) / 3 * 1e3
    assert r_op == gdk.q6_fused(*qargs)
    rows = qargs[0].count()
    out["q6_op_at_a_time"] = {"ms_per_step": round(op_ms, 3), "grows_per_s": round(rows / op_ms / 1e6, 2)}
    # the Q1 MAL plan operator by operator (select, group/subgroup,
    # projections, calc to hge, grouped sums / avg3 / count)
    dmax = mkdate(1998, 9, 2)
    q1_op = gdk.q1_fused(cols, dmax, fused=False)
    t = time.perf_counter()
    for _ in range(3):
        q1_op = gdk.q1_fused(cols, dmax, fused=False)
    op1_ms = (time.perf_counter() - t) / 3 * 1e3

    def key(r):
        return (r["returnflag"], r["linestatus"])
    assert sorted((key(r), r["sum_charge"]) for r in q1_op) == \
        sorted((key(r), r["sum_charge"]) for r in gdk.q1_fused(cols, dmax))
    out["q1_op_at_a_time"] = {"ms_per_step": round(op1_ms, 3), "grows_per_s": round(rows / op1_ms / 1e6, 2)}
    return out


def leg_orderkey_group(cx, cols, rows, row0):
    """Config 4 with its exchange: GROUP BY an l_orderkey-shaped key (4
    lines per order, orders clustered as lineitem is) with exact sums of
    l_quantity and l_extendedprice, over the same SF100-per-GPU shards:
    local BATgroup + BATgroupsum, the partial rows hash-partitioned by key
    and shuffled with ONE RCCL all_to_all per column, merged on the owner,
    numbered in global first-occurrence order (opt_mergetable.c:1496-1885
    mat_group / mat_group_aggr); with one GPU the plan is the local BATgroup +
    BATgroupsum alone.  Weak scaling (rows per GPU fixed)."""
    gdk, D = cx.gdk, cx.D
    okey = gdk.BATconvert(gdk.BAT.dense(row0, rows, hseqbase=row0), None, gdk.TYPE_lng)
    okey = gdk.BATcalcdivmod("/", okey, None, gdk.TYPE_lng, c2=4, t2=gdk.TYPE_lng)
    okey.s.hseqbase = row0
    okey.s.tsorted, okey.s.trevsorted, okey.s.tkey, okey.s.tnonil = 1, 0, 0, 1
    vals = [cols["quantity"], cols["extendedprice"]]
    be = D.GdkBackend(cx.dev)
    out = D.dist_group_aggr(be, cx.dist, okey, vals)           # warm-up
    ngroups_local = out["gid"].count()
    del out
    cx.barrier()
    D.STATS["exchange_s"] = 0.0
    t = time.perf_counter()
    for _ in range(cx.args.leg_steps):
        out = D.dist_group_aggr(be, cx.dist, okey, vals)
        del out
    cx.barrier()
    tot = (time.perf_counter() - t) / cx.args.leg_steps
    exch = D.STATS["exchange_s"] / cx.args.leg_steps
    tot, exch, comp = cx.max_over_ranks([tot, exch, tot - exch])
    ng = cx.sum_over_ranks(ngroups_local)
    # byte floor of the plan that runs (the fused ordered GROUP BY + sums,
    # mgdk_group_sums_ordered): key 8 B + two lng values read per row; per
    # group the extent 8 B, key 8 B, histogram 8 B and two hge sums 32 B
    # written (no group-id column is written or read back)
    floor = rows * (8 + 16) + ng // cx.world * (8 + 8 + 8 + 32)
    return {"ms_per_step": round(tot * 1e3, 3), "grows_per_s": round(rows * cx.world / tot / 1e9, 3),
            "unit": "Grows/s", "exchange_ms": round(exch * 1e3, 3), "local_ms": round(comp * 1e3, 3),
            "groups": ng, "rows_per_gpu": rows, "scaling": "weak",
            "byte_floor_per_gpu": floor, "floor_frac": round(floor / tot / 1e9 / HBM_PEAK_GBS, 4),
            "workload": "GROUP BY l_orderkey (4 lines/order) SUM(l_quantity), SUM(l_extendedprice): "
                        "dist_group_aggr (fused ordered group + sums per rank; ordered shards merge "
                        "their edge groups, else one all_to_all per partial column)"}


def _int32_column(n, seed):
    import numpy as np
    return np.random.default_rng(seed).integers(0, 1000, n, dtype=np.int32)


def leg_thetaselect(cx, parity):
    """Config 1: BATthetaselect(b, NULL, v, "<") on ONE 100M-row int32 BAT
    (uniform [0, 1000), no nils, unsorted) range-partitioned over the ranks
    (strong scaling; select needs no exchange: each rank's oids are global
    because its shard's hseqbase is its first row), at 1 / 10 / 50 % hits.
    The device time is the HIP events around the entry point on the library
    stream; bytes = 4 B per row read + 8 B per hit written.
    Every result is compared with the oracle's BATthetaselect."""
    import numpy as np
    gdk = cx.gdk
    N = cx.args.select_rows
    per = (N + cx.world - 1) // cx.world
    lo, hi = min(N, cx.rank * per), min(N, (cx.rank + 1) * per)
    a = _int32_column(N, 7)[lo:hi]
    b = gdk.BAT.from_numpy(gdk.TYPE_int, a, hseqbase=lo, sorted_=False, revsorted=False, key=False,
                           nonil=True)
    res = {"rows_total": N, "rows_per_gpu": hi - lo, "scaling": "strong", "unit": "Grows/s", "hits": {}}
    ok = True
    ora = None
    if not cx.args.no_parity:
        from oracle import pyoracle as ora
        ora.lib()
        ob = ora.Bat.from_array(ora.TYPE_int, a, hseqbase=lo, nonil=True)
    for v, pct in ((10, 1), (100, 10), (500, 50)):
        s = gdk.BATthetaselect(b, None, v, "<")
        cx.barrier()
        gdk.prof_reset()
        gdk.prof_enable(True)
        t = time.perf_counter()
        for _ in range(cx.args.leg_steps * 3):
            s = gdk.BATthetaselect(b, None, v, "<")
        cx.barrier()
        wall = (time.perf_counter() - t) / (cx.args.leg_steps * 3)
        kms, kn = gdk.prof_get("select")
        gdk.prof_enable(False)
        k = kms / max(1, kn) * 1e-3
        nh = s.count()
        wall, k = cx.max_over_ranks([wall, k])
        hits = cx.sum_over_ranks(nh)
        byts = 4 * (hi - lo) + 8 * nh
        res["hits"]["%d%%" % pct] = {
            "hits": hits, "ms_per_step": round(wall * 1e3, 4), "kernel_ms": round(k * 1e3, 4),
            "grows_per_s": round(N / wall / 1e9, 2),
            "roofline_frac": round(byts / k / 1e9 / HBM_PEAK_GBS, 4) if k > 0 else None}
        if ora is not None:
            want = ora.BATthetaselect(ob, None, v, "<").values()
            ok &= bool(np.array_equal(s.to_numpy(), want.astype(np.uint64)))
        del s
    if ora is not None:
        parity["thetaselect"] = ok
    return res


def _join_inputs(sf, seed=3):
    """Config 3's sides: o_orderkey = 15M (SF10) unique sparse keys (the
    first 8 of every 32, as the TPC-H spec lays them out) shuffled;
    l_orderkey = 1-7 lines per order, shuffled (so BATjoin takes the hash
    path, gdk_join.c:4568)."""
    import numpy as np
    r = np.random.default_rng(seed)
    no = int(round(sf * 1_500_000))
    i = np.arange(no, dtype=np.int64)
    ok = ((i // 8) * 32 + (i % 8) + 1).astype(np.int32)
    r.shuffle(ok)
    lk = np.repeat(ok, r.integers(1, 8, no)).astype(np.int32)
    r.shuffle(lk)
    return lk, ok


def _pair_hash(r1, r2, first):
    """Order-sensitive 64-bit checksum of (position, r1, r2) triples, the
    position counted from `first` (a rank's offset in the global result)."""
    import numpy as np
    with np.errstate(over="ignore"):
        pos = np.arange(first, first + r1.size, dtype=np.uint64)
        x = r1.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        x ^= r2.astype(np.uint64) + pos * np.uint64(0xC2B2AE3D27D4EB4F)
        x ^= x >> np.uint64(29)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(32)
        return int(x.sum(dtype=np.uint64))


def leg_hashjoin(cx, parity):
    """Config 3: BATjoin(l_orderkey, o_orderkey) at SF10 -- 60M probe rows
    against 15M unique build rows, both shuffled int32, resident in HBM.
    One GPU: the entry point itself, timed by HIP events on the library
    stream (`kernel_ms`: the algorithm choice, partitioning, probe and the
    result in the reference's order); N GPUs: dist_join over row-range shards
    of both sides (strong scaling).  Algorithmic bytes: 4 B
    per input row + 2 x 8 B per result pair.  Parity: the pairs against the
    oracle's BATjoin on the same sides (exactly at N = 1, through an
    order-sensitive checksum of the concatenated global result at N > 1)."""
    import numpy as np
    gdk, D = cx.gdk, cx.D
    lk, ok = _join_inputs(cx.args.join_sf)
    nl, nr = lk.size, ok.size
    perl, perr = (nl + cx.world - 1) // cx.world, (nr + cx.world - 1) // cx.world
    l0, l1 = min(nl, cx.rank * perl), min(nl, (cx.rank + 1) * perl)
    r0, r1_ = min(nr, cx.rank * perr), min(nr, (cx.rank + 1) * perr)
    L = gdk.BAT.from_numpy(gdk.TYPE_int, lk[l0:l1], hseqbase=l0, sorted_=False, revsorted=False,
                           key=False, nonil=True)
    R = gdk.BAT.from_numpy(gdk.TYPE_int, ok[r0:r1_], hseqbase=r0, sorted_=False, revsorted=False,
                           key=True, nonil=True)
    be = D.GdkBackend(cx.dev)

    def run():
        if cx.world == 1:
            a, b = gdk.BATjoin(L, R)
            return a, b
        a, b, _ = D.dist_join(be, cx.dist, L, R, perl, perr)
        return a, b

    a, b = run()
    del a, b
    cx.barrier()
    gdk.prof_reset()
    gdk.prof_enable(True)
    steps = cx.args.leg_steps * 2
    t = time.perf_counter()
    for _ in range(steps):
        a, b = run()
        del a, b
    cx.barrier()
    wall = (time.perf_counter() - t) / steps
    kms, kn = gdk.prof_get("join")
    gdk.prof_enable(False)
    k = kms / max(1, kn) * 1e-3 if cx.world == 1 else 0.0
    wall, k = cx.max_over_ranks([wall, k])
    alg = 4 * (nl + nr) + 16 * nl
    t_alg = k if cx.world == 1 else wall
    res = {"rows_probe": int(nl), "rows_build": int(nr), "ms_per_step": round(wall * 1e3, 4),
           "kernel_ms": round(k * 1e3, 4) if cx.world == 1 else None,
           "grows_per_s": round(nl / wall / 1e9, 3), "unit": "Grows/s", "scaling": "strong",
           "algorithmic_bytes": alg,
           "roofline_frac": round(alg / t_alg / 1e9 / HBM_PEAK_GBS, 4),
           "path": "BATjoin" if cx.world == 1 else "dist_join"}
    if not cx.args.no_parity:
        a, b = run()
        ga, gb = a.to_numpy(), b.to_numpy()
        del a, b
        npairs = ga.size
        counts = [cx.D._s64(x[0]) for x in cx.D._gather_int64(cx.dist, cx.dev, [npairs])] \
            if cx.dist is not None else [npairs]
        first = sum(counts[:cx.rank])
        h = cx.sum_over_ranks(cx.D._s64(_pair_hash(ga, gb, first))) & ((1 << 64) - 1)
        ok_ = True
        if cx.rank == 0:
            from oracle import pyoracle as ora
            ora.lib()
            OL = ora.Bat.from_array(ora.TYPE_int, lk, nonil=True)
            OR = ora.Bat.from_array(ora.TYPE_int, ok, nonil=True, key=True)
            w1, w2 = ora.BATjoin(OL, OR)
            wa, wb = w1.values(), w2.values()
            if cx.world == 1:
                ok_ = bool(np.array_equal(ga, wa.astype(np.uint64)) and np.array_equal(gb, wb.astype(np.uint64)))
            else:
                ok_ = wa.size == sum(counts) and h == _pair_hash(wa, wb, 0)
            res["pairs"] = int(wa.size)
        parity["join"] = ok_
    return res


def leg_sort_group(cx, parity, n=100_000_000, ngroups=1000):
    """The two §8 rows BASELINE lists no config for, on every GPU (each rank
    its own column; times are the max over ranks):
    BATsort of a 100M-row int32 column (uniform over the whole int range,
    unsorted) with its order and group-id outputs (gdk_batop.c:2342, the
    stable LSD radix sort GDKrsort, gdk_rsort.c:21), and BATgroup of a
    100M-row int32 column with 1000 distinct values (gdk_group.c:1359:
    group ids, extents, histogram).  `kernel_ms`: HIP events around the
    entry point on the library stream.  Algorithmic bytes:
    sort 4 B key in + 4 B value + 8 B order + 8 B group id out = 24 B/row;
    group 4 B key in + 8 B group id out = 12 B/row.  Parity: sorted values,
    order and groups against numpy's stable argsort (GDKrsort is stable; the
    suite pins the device sort to the oracle's BATsort); group ids, extents
    and histogram against the oracle's BATgroup on the same column."""
    import numpy as np
    gdk = cx.gdk
    r = np.random.default_rng(11)
    res = {}
    a = r.integers(-(2**31) + 1, 2**31 - 1, n, dtype=np.int64).astype(np.int32)
    b = gdk.BAT.from_numpy(gdk.TYPE_int, a, sorted_=False, revsorted=False, key=False, nonil=True)
    # a sort that returns the order leaves it with b as b's order index (as
    # the reference's BATsort does, gdk_batop.c:2717-2765) and the next sort
    # of b would answer from it (:2510-2568): each step drops it first
    out = gdk.BATsort(b)
    del out
    gdk.OIDXdestroy(b)
    cx.barrier()
    gdk.prof_reset()
    gdk.prof_enable(True)
    steps = cx.args.leg_steps * 2
    t = time.perf_counter()
    for _ in range(steps):
        out = gdk.BATsort(b)
        del out
        gdk.OIDXdestroy(b)
    cx.barrier()
    wall = (time.perf_counter() - t) / steps
    kms, kn = gdk.prof_get("sort")
    gdk.prof_enable(False)
    wall, k = cx.max_over_ranks([wall, kms / max(1, kn)])
    res["sort"] = {"rows": n, "dtype": "int32", "outputs": "sorted + order + groups",
                   "ms_per_step": round(wall * 1e3, 4), "kernel_ms": round(k, 4),
                   "grows_per_s": round(n / wall / 1e9, 3), "bytes_per_row": 24,
                   "roofline_frac": round(24 * n / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if k > 0 else None}
    ora = None
    if not cx.args.no_parity:
        from oracle import pyoracle as ora
        ora.lib()
        sv, so, sg = gdk.BATsort(b)
        # the stable sort (GDKrsort) is pinned against the oracle's BATsort by
        # the test suite; at 100M rows its model here is numpy's stable radix
        # argsort (the same permutation: stable, no nils), group ids = runs of
        # equal sorted values
        wo = np.argsort(a, kind="stable")
        wv = a[wo]
        wg = np.concatenate(([0], np.cumsum(wv[1:] != wv[:-1]))).astype(np.uint64) if n else wv
        parity["sort"] = bool(np.array_equal(sv.to_numpy(), wv) and
                              np.array_equal(so.to_numpy().astype(np.uint64), wo.astype(np.uint64)) and
                              np.array_equal(sg.to_numpy().astype(np.uint64), wg))
        del sv, so, sg, wv, wo, wg
    del b, a
    gdk.lib().mgdk_mem_release_cache()
    a = r.integers(0, ngroups, n, dtype=np.int32)
    b = gdk.BAT.from_numpy(gdk.TYPE_int, a, sorted_=False, revsorted=False, key=False, nonil=True)
    out = gdk.BATgroup(b)
    del out
    cx.barrier()
    gdk.prof_reset()
    gdk.prof_enable(True)
    t = time.perf_counter()
    for _ in range(steps):
        out = gdk.BATgroup(b)
        del out
    cx.barrier()
    wall = (time.perf_counter() - t) / steps
    kms, kn = gdk.prof_get("group")
    gdk.prof_enable(False)
    wall, k = cx.max_over_ranks([wall, kms / max(1, kn)])
    res["group"] = {"rows": n, "groups": ngroups, "dtype": "int32", "outputs": "groups + extents + histo",
                    "ms_per_step": round(wall * 1e3, 4), "kernel_ms": round(k, 4),
                    "grows_per_s": round(n / wall / 1e9, 3), "bytes_per_row": 12,
                    "roofline_frac": round(12 * n / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if k > 0 else None}
    if ora is not None:
        g, e, h = gdk.BATgroup(b)
        wg, we, wh = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, a, nonil=True))
        parity["group"] = bool(np.array_equal(g.to_numpy().astype(np.uint64), wg.values().astype(np.uint64)) and
                               np.array_equal(e.to_numpy().astype(np.uint64), we.values().astype(np.uint64)) and
                               np.array_equal(h.to_numpy().astype(np.int64), wh.values().astype(np.int64)))
    return res


def leg_window(cx, parity, limit=100, plen=100_000, sample_parts=10):
    """Config 5: GDKanalyticalwindowbounds (RANGE 100 PRECEDING) over ONE
    column of --window-rows rows (1B) range-partitioned over the ranks
    (strong scaling); shards start at partition boundaries, so the move of
    rows to the partition's owner is empty and every rank computes its
    bounds locally (dist_window_bounds).  Parity: `sample_parts` whole
    partitions spread over each rank's rows (1M rows, up to the column's
    end, i.e. byte offsets past 2^32) recomputed by the oracle's walk."""
    import numpy as np
    gdk, D = cx.gdk, cx.D
    n = cx.args.window_rows // cx.world
    v, p = gdk.gen_window_column(5 + cx.rank, n, plen)
    v.s.hseqbase = p.s.hseqbase = cx.rank * n
    be = D.GdkBackend(cx.dev)
    r = D.dist_window_bounds(be, cx.dist, v, p, limit, True)
    del r
    cx.barrier()
    gdk.prof_reset()
    gdk.prof_enable(True)
    t = time.perf_counter()
    for _ in range(cx.args.leg_steps):
        r = D.dist_window_bounds(be, cx.dist, v, p, limit, True)
        del r
    cx.barrier()
    tot = (time.perf_counter() - t) / cx.args.leg_steps
    kms, kn = gdk.prof_get("windowbounds")
    gdk.prof_enable(False)
    kern = kms / max(1, kn) * 1e-3
    tot, kern = cx.max_over_ranks([tot, kern])
    total_rows = n * cx.world
    res = {"ms_per_step": round(tot * 1e3, 3), "grows_per_s": round(total_rows / tot / 1e9, 3),
           "unit": "Grows/s", "kernel_ms": round(kern * 1e3, 3), "rows_total": total_rows,
           "rows_per_gpu": n, "partitions": total_rows // plen, "limit": limit, "scaling": "strong",
           "roofline_frac_kernel": round(17 * n / kern / 1e9 / HBM_PEAK_GBS, 4) if kern > 0 else None}
    if not cx.args.no_parity:
        from oracle import pyoracle as ora
        ora.lib()
        first, bnd = D.dist_window_bounds(be, cx.dist, v, p, limit, True)
        held = bnd.count()
        ok = True
        nparts = held // plen
        picks = sorted({(k * (nparts - 1)) // max(1, sample_parts - 1) for k in range(sample_parts)}) \
            if nparts else []
        checked = 0
        for k in picks:
            s = k * plen + (first - cx.rank * n)       # first held row is a partition start
            e = min(s + plen, n)
            if s < 0 or e <= s:
                continue
            vv = gdk.BATslice(v, s, e).to_numpy()
            pp = gdk.BATslice(p, s, e).to_numpy()
            got = gdk.BATslice(bnd, k * plen, k * plen + (e - s)).to_numpy()
            want = ora.rangebounds(ora.Bat.from_array(ora.TYPE_lng, vv, nonil=bool((vv != -(1 << 63)).all())),
                                   ora.Bat.from_array(ora.TYPE_bit, pp.view(np.int8)), limit, True).values()
            ok &= bool(np.array_equal(got.astype(np.int64), want.astype(np.int64) + first + k * plen))
            checked += e - s
        del bnd
        parity["window_sample"] = ok and checked > 0
        res["parity_rows_checked_per_gpu"] = checked
    return res


def pmc_traffic(kernel, rows):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json, made by tools/pmc_summary.py from
    separate --pmc FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled for
    gfx950's half-counted wide streaming reads), scaled to this row count --
    only while the kernel's source file is the one that was measured (its
    recorded sha256); otherwise None, with the reason."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))[kernel]
    except Exception:  # noqa: BLE001
        return None, "no PMC summary for %s" % kernel
    src = d.get("kernel_source")
    if not src:
        return None, "PMC summary of %s predates source tracking: stale" % kernel
    try:
        sha = hashlib.sha256(open(os.path.join(ROOT, src), "rb").read()).hexdigest()[:16]
    except OSError:
        return None, "kernel source %s missing" % src
    if sha != d.get("kernel_source_sha16"):
        return None, "%s changed since its PMC pass (%s): stale" % (src, d.get("source"))
    return int(round(d["hbm_bytes_per_row"] * rows)), "PMC %s, %s sha %s" % (
        ", ".join(d.get("source", [])), src, sha)


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
    cols = ora.tpch_lineitem(SEED, 0, n, max(1, int(args.cpu_sf * 200_000)))
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
    for configs 1, 3, 4 and 5 on bounded samples of the same workloads."""
    try:
        import numpy as np
        from oracle import pyoracle as ora
        ora.lib()
    except Exception as e:  # noqa: BLE001
        return {"error": "oracle unavailable: %s" % e}
    out = {"cgroup_cpu_quota": _cpu_quota(), "nproc": os.cpu_count()}
    r = np.random.default_rng(3)
    # config 1: BATthetaselect on the 100M int32 column, 10 % hits, one
    # thread (a MAL call of algebra.thetaselect is one thread)
    a = _int32_column(args.select_rows, 7)
    B = ora.Bat.from_array(ora.TYPE_int, a, nonil=True)
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        ora.BATthetaselect(B, None, 100, "<")
        ts.append(time.perf_counter() - t)
    med = statistics.median(ts)
    out["config1_thetaselect"] = {"value": round(a.size / med / 1e9, 4), "unit": "Grows/s", "cores": 1,
                                  "kind": "port", "ms": round(med * 1e3, 1),
                                  "sample": "%d int32 rows, < 100 (10 %% hits), median of 3" % a.size}
    del B, a
    # config 3: BATjoin (hash path) lineitem x orders at SF1, single thread
    # (the reference's hashjoin is one thread per call)
    lk, ok = _join_inputs(1.0)
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
                                         % (len(lk), len(ok))}
    # config 4: Q1 op-at-a-time over an SF2 sample on the box's CPU share
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    n4 = 2 * SF1_ROWS
    cols = ora.tpch_lineitem(SEED, 0, n4, 400_000)
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
