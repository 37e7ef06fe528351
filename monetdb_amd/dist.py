"""Multi-GPU plumbing for the row-range sharded pipelines.

One process per GPU (torchrun); rank r owns lineitem rows [r*N, (r+1)*N) in
its own HBM -- the mitosis partitioning of opt_mitosis.c:150-230 -- and the
per-rank partial aggregates are combined the way mergetable re-aggregates
packed partials (opt_mergetable.c:1496-1670): exact 128-bit sums, counts, and
group keys renumbered by global first occurrence.  The only collectives are
all_gathers of a few dozen bytes (RCCL over xGMI with backend "nccl", or gloo
on the CPU in tests).
"""

MASK64 = (1 << 64) - 1


def _words(v):
    v &= (1 << 128) - 1
    return [v & MASK64, v >> 64]


def _from_words(lo, hi):
    v = ((hi & MASK64) << 64) | (lo & MASK64)
    return v - (1 << 128) if v >= (1 << 127) else v


def shard(rows_per_rank, rank):
    """Row range [row0, row0 + n) of `rank` under weak scaling."""
    return rank * rows_per_rank, rows_per_rank


def _gather_int64(dist, device, vals):
    import torch
    t = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in vals], dtype=torch.int64,
                     device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[int(x) & MASK64 for x in o.cpu().tolist()] for o in out]


def combine_hge(value, dist=None, device="cpu"):
    """Exact sum of one 128-bit integer per rank."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    parts = _gather_int64(dist, device, _words(value))
    return sum(_from_words(lo, hi) for lo, hi in parts)


Q1_SUMS = ("sum_qty", "sum_base_price", "sum_disc_price", "sum_charge", "sum_disc")
Q1_MAXG = 16


def combine_q1(rows, dist=None, device="cpu", rows_per_rank=0, rank=0):
    """Merge per-rank Q1 group rows: key (returnflag, linestatus), exact sums
    and counts added, first_row = global minimum (first-occurrence order)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return sorted(rows, key=lambda r: r["first_row"])
    flat = [len(rows)]
    for i in range(Q1_MAXG):
        if i < len(rows):
            r = rows[i]
            flat += [r["returnflag"], r["linestatus"], r["first_row"], r["count_order"]]
            for k in Q1_SUMS:
                flat += _words(r[k])
        else:
            flat += [0] * (4 + 2 * len(Q1_SUMS))
    merged = {}
    for part in _gather_int64(dist, device, flat):
        n = part[0]
        for i in range(n):
            base = 1 + i * (4 + 2 * len(Q1_SUMS))
            key = (part[base], part[base + 1])
            first = part[base + 2]
            m = merged.setdefault(key, {"returnflag": key[0], "linestatus": key[1],
                                        "first_row": first, "count_order": 0,
                                        **{k: 0 for k in Q1_SUMS}})
            m["first_row"] = min(m["first_row"], first)
            m["count_order"] += part[base + 3]
            for j, k in enumerate(Q1_SUMS):
                m[k] += _from_words(part[base + 4 + 2 * j], part[base + 5 + 2 * j])
    return sorted(merged.values(), key=lambda r: r["first_row"])


def avg3(total, count):
    """BATgroupavg3 rounding of an exact sum (gdk/gdk_aggr.c:2070-2095):
    floor average, then half away from zero; returns (avg, remainder)."""
    q, r = divmod(total, count)
    if r > 0:
        if q < 0:
            if 2 * r > count:
                q, r = q + 1, r - count
        elif 2 * r >= count:
            q, r = q + 1, r - count
    return q, r
