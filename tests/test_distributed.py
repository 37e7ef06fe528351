"""World-size-2 gloo tests (CPU) of the multi-GPU sharding and combine logic that
bench.py runs over RCCL: every rank owns a row range of lineitem, computes its
partial Q6 / Q1 aggregates, and the exact combine must equal the single-node
answer over all rows."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _first_rows(cols, row0, dmax):
    m = cols["shipdate"] <= dmax
    idx = np.flatnonzero(m)
    code = cols["returnflag"][idx].astype(np.int64) * 256 + cols["linestatus"][idx]
    u, first = np.unique(code, return_index=True)
    return {(int(c >> 8), int(c & 255)): int(idx[f]) + row0 for c, f in zip(u, first)}


def _worker(rank, world, port, n, out_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    from monetdb_amd import dist as D
    from oracle import pyoracle as ora

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    row0, cnt = D.shard(n, rank)
    cols = ora.tpch_lineitem(11, row0, cnt, 20_000)
    q6 = D.combine_hge(ora.q6(cols, 1), dist, "cpu")
    dmax = ora.mkdate(1998, 9, 2)
    firsts = _first_rows(cols, row0, dmax)
    rows = []
    for r in ora.q1(cols, 1):
        r = dict(r)
        r["first_row"] = firsts[(r["returnflag"], r["linestatus"])]
        r["sum_disc"] = 0
        rows.append(r)
    q1 = D.combine_q1(rows, dist, "cpu")
    if rank == 0:
        full = ora.tpch_lineitem(11, 0, n * world, 20_000)
        want6 = ora.q6(full, 2)
        want1 = ora.q1(full, 2)
        wf = _first_rows(full, 0, dmax)
        ok6 = q6 == want6
        got1 = {(r["returnflag"], r["linestatus"]): r for r in q1}
        ok1 = len(got1) == len(want1) and all(
            got1[(w["returnflag"], w["linestatus"])][k] == w[k]
            for w in want1 for k in ("sum_qty", "sum_base_price", "sum_disc_price", "sum_charge",
                                     "count_order"))
        order_ok = [(r["returnflag"], r["linestatus"]) for r in q1] == \
            [k for k, _ in sorted(wf.items(), key=lambda kv: kv[1])]
        avg_ok = all(D.avg3(got1[(w["returnflag"], w["linestatus"])]["sum_qty"],
                            w["count_order"]) == (w["avg_qty"], w["rem_qty"]) for w in want1)
        with open(out_path, "w") as f:
            f.write("%d %d %d %d" % (ok6, ok1, order_ok, avg_ok))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_q6_q1(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.txt")
    mp.spawn(_worker, args=(2, _free_port(), 150_001, out), nprocs=2, join=True)
    assert open(out).read().split() == ["1", "1", "1", "1"]


def test_combine_single_process_is_identity():
    from monetdb_amd import dist as D
    assert D.combine_hge(-(1 << 100)) == -(1 << 100)
    rows = [{"first_row": 5, "x": 1}, {"first_row": 2, "x": 2}]
    assert [r["first_row"] for r in D.combine_q1(rows)] == [2, 5]
    assert D.avg3(3, 2) == (2, -1) and D.avg3(-3, 2) == (-2, 1) and D.avg3(23, 3) == (8, -1)


# ---- exchange steps (dist_group_aggr / dist_join / dist_sort / dist_window_bounds)

def _exchange_worker(rank, world, port, out_dir, backend="oracle"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch
    import torch.distributed as dist

    from dist_backends import OracleBackend
    from monetdb_amd import dist as D
    from oracle import pyoracle as ora

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    if backend == "gdk":
        # the product operators on the GPU; shuffles staged through the host (gloo)
        from monetdb_amd import gdk
        gdk.init(0)
        be = D.GdkBackend("cpu")
    else:
        be = OracleBackend()

    def Col(tp, arr, hseq):     # noqa: N802 -- a column of the active backend
        return be.column(tp, arr, hseq)
    errs = []
    r = np.random.default_rng(7)
    per = 6_000
    N = per * world
    keys = r.integers(0, 700, N).astype(np.int32)
    keys[r.random(N) < 0.02] = np.iinfo(np.int32).min           # nils group together
    v1 = r.integers(-10**12, 10**12, N).astype(np.int64)
    v2 = r.integers(0, 100, N).astype(np.int64)
    lo, hi = rank * per, (rank + 1) * per

    # group + sums
    got = D.dist_group_aggr(be, dist, Col(ora.TYPE_int, keys[lo:hi], lo),
                            [Col(ora.TYPE_lng, v1[lo:hi], lo), Col(ora.TYPE_lng, v2[lo:hi], lo)])
    g, e, h = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, keys))
    ev, hv = e.values().astype(np.int64), h.values()
    s1 = ora.BATgroupsum(ora.Bat.from_array(ora.TYPE_lng, v1), g, e, ora.TYPE_hge).values()
    s2 = ora.BATgroupsum(ora.Bat.from_array(ora.TYPE_lng, v2), g, e, ora.TYPE_hge).values()
    V = lambda c: np.asarray([int(x) for x in be.values(c)], dtype=object)   # noqa: E731
    gid = V(got["gid"]).astype(np.int64)
    if len(gid) and not (np.diff(gid) > 0).all():
        errs.append("gids not ascending")
    if len(gid):
        ev_ = ev[gid]
        kw = keys[ev_].astype(np.int64)
        kw[keys[ev_] == np.iinfo(np.int32).min] = np.iinfo(np.int64).min
        for name, have, want in (("key", V(got["key"]), kw), ("first", V(got["first_row"]), ev_),
                                 ("count", V(got["count"]), hv[gid]),
                                 ("sum1", V(got["sums"][0]), np.asarray(s1, dtype=object)[gid]),
                                 ("sum2", V(got["sums"][1]), np.asarray(s2, dtype=object)[gid])):
            if [int(x) for x in have] != [int(x) for x in want]:
                errs.append("group column %s mismatch" % name)
    tot = torch.tensor([len(gid)])
    dist.all_reduce(tot)
    if int(tot) != len(ev):
        errs.append("groups %d != %d" % (int(tot), len(ev)))

    # group + sums over ORDERED shards whose key ranges meet at the shard
    # edges (l_orderkey-like): the ordered merge, no hash shuffle.  Rank 1
    # (of 3) holds one key only, shared with both neighbours (a chain).
    ok_ = np.sort(r.integers(0, 40, N)).astype(np.int64)
    if world == 3:
        ok_[per - 200:2 * per + 300] = ok_[per - 200]
    ok_[:3] = np.iinfo(np.int64).min                                   # nils first
    before = D.STATS.get("ordered_merge", 0)
    got = D.dist_group_aggr(be, dist, Col(ora.TYPE_lng, ok_[lo:hi], lo),
                            [Col(ora.TYPE_lng, v1[lo:hi], lo), Col(ora.TYPE_lng, v2[lo:hi], lo)])
    if D.STATS.get("ordered_merge", 0) != before + 1:
        errs.append("ordered shards did not take the ordered merge")
    g, e, h = ora.BATgroup(ora.Bat.from_array(ora.TYPE_lng, ok_))
    ev, hv = e.values().astype(np.int64), h.values()
    s1 = ora.BATgroupsum(ora.Bat.from_array(ora.TYPE_lng, v1), g, e, ora.TYPE_hge).values()
    s2 = ora.BATgroupsum(ora.Bat.from_array(ora.TYPE_lng, v2), g, e, ora.TYPE_hge).values()
    gid = V(got["gid"]).astype(np.int64)
    if len(gid) and not (np.diff(gid) > 0).all():
        errs.append("ordered: gids not ascending")
    if len(gid):
        for name, have, want in (("key", V(got["key"]), ok_[ev[gid]]), ("first", V(got["first_row"]), ev[gid]),
                                 ("count", V(got["count"]), hv[gid]),
                                 ("sum1", V(got["sums"][0]), np.asarray(s1, dtype=object)[gid]),
                                 ("sum2", V(got["sums"][1]), np.asarray(s2, dtype=object)[gid])):
            if [int(x) for x in have] != [int(x) for x in want]:
                errs.append("ordered: group column %s mismatch" % name)
    tot = torch.tensor([len(gid)])
    dist.all_reduce(tot)
    if int(tot) != len(ev):
        errs.append("ordered: groups %d != %d" % (int(tot), len(ev)))
    g, e, h = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, keys))
    ev, hv = e.values().astype(np.int64), h.values()

    # group + AVG: per-shard BATgroupavg3 partials, one shuffle, BATgroupavg3combine
    v3 = v1.copy()
    v3[r.random(N) < 0.03] = np.iinfo(np.int64).min
    gota = D.dist_group_avg(be, dist, Col(ora.TYPE_int, keys[lo:hi], lo), Col(ora.TYPE_lng, v3[lo:hi], lo))
    av, _, _ = ora.BATgroupavg3(ora.Bat.from_array(ora.TYPE_lng, v3), g, e, True)
    av = av.values()
    gida = V(gota["gid"]).astype(np.int64)
    if len(gida) and ([int(x) for x in V(gota["first_row"])] != [int(x) for x in ev[gida]] or
                      [int(x) for x in V(gota["avg"])] != [int(x) for x in np.asarray(av, dtype=object)[gida]]):
        errs.append("avg groups mismatch")
    tot = torch.tensor([len(gida)])
    dist.all_reduce(tot)
    if int(tot) != len(ev):
        errs.append("avg groups %d != %d" % (int(tot), len(ev)))

    # hash join, duplicates on both sides
    lk = r.integers(0, 3000, N).astype(np.int32)
    rk = r.integers(0, 3000, N).astype(np.int32)
    # three shapes: plain hash join, swapped (small left), both sorted
    for name, lkk, rkk in (("hash", lk, rk),
                           ("swap", r.choice(1 << 20, world * 300, replace=False).astype(np.int32),
                            r.integers(0, 1 << 20, N).astype(np.int32)),
                           ("merge", np.sort(lk), np.sort(rk))):
        lper, rper = len(lkk) // world, len(rkk) // world
        a, b, drv = D.dist_join(be, dist, Col(ora.TYPE_int, lkk[rank * lper:(rank + 1) * lper], rank * lper),
                                Col(ora.TYPE_int, rkk[rank * rper:(rank + 1) * rper], rank * rper), lper, rper)
        wa, wb = ora.BATjoin(ora.Bat.from_array(ora.TYPE_int, lkk), ora.Bat.from_array(ora.TYPE_int, rkk))
        wa, wb = wa.values(), wb.values()
        dv, per_ = (wa, lper) if drv == "l" else (wb, rper)
        sel = (dv >= rank * per_) & (dv < (rank + 1) * per_)
        if not (np.array_equal(be.values(a), wa[sel]) and np.array_equal(be.values(b), wb[sel])):
            errs.append("join mismatch " + name)

    # stable sort
    sk = r.integers(-50, 50, N).astype(np.int64)
    s, o = D.dist_sort(be, dist, Col(ora.TYPE_lng, sk[lo:hi], lo), sample=16)
    ws, wo = ora.BATsort(ora.Bat.from_array(ora.TYPE_lng, sk))
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([be.n(s)]))
    off = sum(int(x) for x in sizes[:rank])
    if not (np.array_equal(be.values(s), ws.values()[off:off + be.n(s)]) and
            np.array_equal(be.values(o), wo.values()[off:off + be.n(s)])):
        errs.append("sort mismatch")

    # RANGE window bounds; partitions straddle shard edges, one shard has none
    plen = [2500, 9000, 700, 4000, 1800]
    bits = np.zeros(N, np.int8)
    p, k = 0, 0
    while p < N:
        bits[p] = 1
        p += plen[k % len(plen)]
        k += 1
    vals = np.concatenate([np.cumsum(r.integers(0, 5, 100)) for _ in range(N // 100)]).astype(np.int64)
    order_ = np.zeros(N, np.int64)
    starts = np.flatnonzero(bits)
    for a0, a1 in zip(starts, list(starts[1:]) + [N]):
        order_[a0:a1] = np.sort(vals[a0:a1])
    for preceding in (True, False):
        first, bnd = D.dist_window_bounds(be, dist, Col(ora.TYPE_lng, order_[lo:hi], lo),
                                          Col(ora.TYPE_bit, bits[lo:hi], lo), 7, preceding)
        want = ora.rangebounds(ora.Bat.from_array(ora.TYPE_lng, order_),
                               ora.Bat.from_array(ora.TYPE_bit, bits), 7, preceding).values()
        bnd = np.asarray(be.values(bnd), dtype=np.int64)
        if not np.array_equal(bnd, want[first:first + len(bnd)].astype(np.int64)):
            errs.append("window mismatch preceding=%s" % preceding)
        cnt = torch.tensor([len(bnd)])
        dist.all_reduce(cnt)
        if int(cnt) != N:
            errs.append("window rows %d != %d" % (int(cnt), N))
    with open(os.path.join(out_dir, "rank%d.txt" % rank), "w") as f:
        f.write("\n".join(errs) if errs else "ok")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange_steps(tmp_path, world):
    import torch.multiprocessing as mp
    mp.spawn(_exchange_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for rk in range(world):
        assert open(tmp_path / ("rank%d.txt" % rk)).read() == "ok", rk
