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
