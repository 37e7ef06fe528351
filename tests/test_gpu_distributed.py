"""The exchange steps of monetdb_amd/dist.py with the PRODUCT backend: every
local operator runs through libmgdk on the GPU (two ranks sharing the box's
one GPU), shuffles over gloo staged through the host; results checked
against the single-node oracle (tests/test_distributed.py's worker)."""
import pytest

from test_distributed import _exchange_worker, _free_port

pytestmark = pytest.mark.gpu


def test_gpu_exchange_steps_world2(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_exchange_worker, args=(2, _free_port(), str(tmp_path), "gdk"), nprocs=2, join=True)
    for rk in range(2):
        assert open(tmp_path / ("rank%d.txt" % rk)).read() == "ok", rk


def test_gdk_backend_device_pack_unpack_roundtrip():
    """GdkBackend(device="cuda:0").pack / unpack -- the branch RCCL runs on:
    lng, oid and hge columns into one (rows, k) int64 device tensor and back
    into device BATs, bit-exact (no host staging)."""
    import numpy as np
    import torch

    from monetdb_amd import dist as D
    from monetdb_amd import gdk
    gdk.init(0)
    be = D.GdkBackend("cuda:0")
    r = np.random.default_rng(3)
    n = 100_003
    lv = r.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    ov = r.integers(0, 2**40, n).astype(np.uint64)
    hv = [int(x) * (1 << 64) + int(y) for x, y in zip(r.integers(-2**62, 2**62, n), r.integers(0, 2**63, n))]
    hv[5] = -(1 << 127)          # nil
    hw = np.array([[x & (2**64 - 1), (x >> 64) & (2**64 - 1)] for x in hv], dtype=np.uint64)
    cols = [gdk.BAT.from_numpy(gdk.TYPE_lng, lv), gdk.BAT.from_numpy(gdk.TYPE_hge, hw),
            gdk.BAT.from_numpy(gdk.TYPE_oid, ov)]
    t = be.pack(cols)
    assert t.is_cuda and t.shape == (n, 4) and t.dtype == torch.int64
    assert np.array_equal(t[:, 0].cpu().numpy(), lv)
    back = be.unpack(t, [gdk.TYPE_lng, gdk.TYPE_hge, gdk.TYPE_oid], hseq=7)
    assert np.array_equal(back[0].to_numpy(), lv)
    assert [int(x) for x in back[1].values()] == hv
    assert np.array_equal(back[2].to_numpy(), ov)
    assert all(b.hseqbase == 7 and b.count() == n for b in back)
    # empty
    e = be.unpack(be.pack([gdk.BAT.from_numpy(gdk.TYPE_lng, lv[:0])]), [gdk.TYPE_lng])
    assert e[0].count() == 0


def _hicard(rank, world, per):
    """l_orderkey-shaped keys (sorted, 1-7 rows per order) and small values"""
    import numpy as np
    r = np.random.default_rng(11)
    reps = r.integers(1, 8, per * world // 2)
    keys = np.repeat(np.arange(len(reps), dtype=np.int64) * 4 + 1, reps)[:per * world]
    vals = r.integers(0, 1_000_000, per * world).astype(np.int64)
    return keys, vals


def _hicard_expect(keys, vals):
    import numpy as np
    u, first, inv, cnt = np.unique(keys, return_index=True, return_inverse=True, return_counts=True)
    order = np.argsort(first, kind="stable")
    gid_of = np.empty(len(u), np.int64)
    gid_of[order] = np.arange(len(u))
    sums = np.bincount(inv, weights=vals.astype(np.float64), minlength=len(u)).astype(np.int64)
    key_g = np.empty(len(u), np.int64)
    first_g = np.empty(len(u), np.int64)
    cnt_g = np.empty(len(u), np.int64)
    sum_g = np.empty(len(u), np.int64)
    key_g[gid_of], first_g[gid_of], cnt_g[gid_of], sum_g[gid_of] = u, first, cnt, sums
    return key_g, first_g, cnt_g, sum_g


def _check_groups(got, want, errs):
    import numpy as np
    from monetdb_amd import gdk
    gid = got["gid"].to_numpy().astype(np.int64)
    key_g, first_g, cnt_g, sum_g = want
    if len(gid) and not (np.diff(gid) > 0).all():
        errs.append("gids not ascending")
    chk = (("key", got["key"].to_numpy(), key_g), ("first", got["first_row"].to_numpy(), first_g),
           ("count", got["count"].to_numpy(), cnt_g))
    for name, have, w in chk:
        if not np.array_equal(have.astype(np.int64), w[gid]):
            errs.append("column %s mismatch" % name)
    s = got["sums"][0]
    assert s.ttype == gdk.TYPE_hge
    words = s.to_numpy().view(np.int64).reshape(-1, 2)
    if not (np.array_equal(words[:, 0], sum_g[gid]) and (words[:, 1] == 0).all()):
        errs.append("sum mismatch")
    return len(gid)


def _hicard_worker(rank, world, port, per, out_dir):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import numpy as np
    import torch
    import torch.distributed as dist

    from monetdb_amd import dist as D
    from monetdb_amd import gdk
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    gdk.init(0)
    be = D.GdkBackend("cpu")      # product operators on the GPU, shuffles staged through the host
    keys, vals = _hicard(rank, world, per)
    lo, hi = rank * per, (rank + 1) * per
    got = D.dist_group_aggr(be, dist, gdk.BAT.from_numpy(gdk.TYPE_lng, keys[lo:hi], hseqbase=lo),
                            [gdk.BAT.from_numpy(gdk.TYPE_lng, vals[lo:hi], hseqbase=lo)])
    errs = []
    assert all(isinstance(got[k], gdk.BAT) for k in ("gid", "key", "first_row", "count"))
    n = _check_groups(got, _hicard_expect(keys, vals), errs)
    tot = torch.tensor([n])
    dist.all_reduce(tot)
    if int(tot) != len(np.unique(keys)):
        errs.append("groups %d" % int(tot))
    with open(os.path.join(out_dir, "rank%d.txt" % rank), "w") as f:
        f.write("\n".join(errs) if errs else "ok")
    dist.barrier()
    dist.destroy_process_group()


def test_gpu_group_aggr_high_cardinality_world2(tmp_path):
    """l_orderkey-keyed GROUP BY + SUM over 2 x 5M rows (~2.5M groups) in the
    world-2 rehearsal: results stay device BATs, no per-group host objects."""
    import torch.multiprocessing as mp
    mp.spawn(_hicard_worker, args=(2, _free_port(), 5_000_000, str(tmp_path)), nprocs=2, join=True)
    for rk in range(2):
        assert open(tmp_path / ("rank%d.txt" % rk)).read() == "ok", rk


def test_gpu_group_aggr_high_cardinality_device_backend():
    """The same on one rank with the device backend (cuda:0): numbering and
    ordering as device operators."""
    from monetdb_amd import dist as D
    from monetdb_amd import gdk
    gdk.init(0)
    keys, vals = _hicard(0, 1, 10_000_000)
    be = D.GdkBackend("cuda:0")
    got = D.dist_group_aggr(be, None, gdk.BAT.from_numpy(gdk.TYPE_lng, keys),
                            [gdk.BAT.from_numpy(gdk.TYPE_lng, vals)])
    errs = []
    _check_groups(got, _hicard_expect(keys, vals), errs)
    assert not errs, errs


def test_gdk_backend_rccl_exchange_cols_world1():
    """GdkBackend.exchange_cols -- the RCCL path of every dist_* shuffle: one
    all_to_all per column straight from the BAT heaps (CUDA array interface
    views, no packing) into new BATs.  World 1 over RCCL on the box's GPU:
    the collective runs for real; the received columns equal the sent ones
    (lng, oid, hge, a dense column, an empty exchange)."""
    import os

    import numpy as np
    import torch
    import torch.distributed as dist

    from monetdb_amd import dist as D
    from monetdb_amd import gdk
    from test_distributed import _free_port
    gdk.init(0)
    torch.cuda.set_device(0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        be = D.GdkBackend("cuda:0")
        r = np.random.default_rng(4)
        n = 200_003
        lv = r.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
        ov = r.integers(0, 2**40, n).astype(np.uint64)
        hw = r.integers(0, 2**63, (n, 2)).astype(np.uint64)
        cols = [gdk.BAT.from_numpy(gdk.TYPE_lng, lv), gdk.BAT.from_numpy(gdk.TYPE_oid, ov),
                gdk.BAT.from_numpy(gdk.TYPE_hge, hw), gdk.BAT.dense(1000, n)]
        types = [gdk.TYPE_lng, gdk.TYPE_oid, gdk.TYPE_hge, gdk.TYPE_oid]
        out, recv = be.exchange_cols(dist, cols, types, [n])
        assert recv == [n]
        assert np.array_equal(out[0].to_numpy(), lv)
        assert np.array_equal(out[1].to_numpy(), ov)
        assert np.array_equal(out[2].to_numpy(), hw)
        assert np.array_equal(out[3].to_numpy(), np.arange(1000, 1000 + n, dtype=np.uint64))
        # a slice (view) as the source, and nothing to send
        s = gdk.BATslice(cols[0], 10, 110)
        out, _ = be.exchange_cols(dist, [s], [gdk.TYPE_lng], [100])
        assert np.array_equal(out[0].to_numpy(), lv[10:110])
        out, _ = be.exchange_cols(dist, [gdk.BATslice(cols[0], 0, 0)], [gdk.TYPE_lng], [0])
        assert out[0].count() == 0
        # the whole high-cardinality group + sum through the RCCL path
        keys, vals = _hicard(0, 1, 50_000)
        got = D.dist_group_aggr(be, dist, gdk.BAT.from_numpy(gdk.TYPE_lng, keys),
                                [gdk.BAT.from_numpy(gdk.TYPE_lng, vals)])
        errs = []
        _check_groups(got, _hicard_expect(keys, vals), errs)
        assert not errs, errs
    finally:
        dist.destroy_process_group()


def test_gdk_backend_exchange_sources_outlive_collectives():
    """exchange_cols releases nothing the collectives may still read: the
    caller drops its source BATs right after the call while another thread
    (its own library stream, the same caching allocator) allocates and fills
    BATs of the same size; every received column must still equal what was
    sent (dist.py: the sources are held until an event recorded after the
    collectives completes)."""
    import os
    import threading

    import numpy as np
    import torch
    import torch.distributed as dist

    from monetdb_amd import dist as D
    from monetdb_amd import gdk
    from test_distributed import _free_port
    gdk.init(0)
    torch.cuda.set_device(0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1)
    stop = threading.Event()
    errs = []

    def churn():
        try:
            k = 0
            while not stop.is_set():
                b = gdk.BATconstant(gdk.TYPE_lng, -7 - k, n)
                assert b.count() == n
                del b
                k += 1
        except Exception as e:      # surfaced below
            errs.append(e)

    try:
        be = D.GdkBackend("cuda:0")
        r = np.random.default_rng(5)
        n = 4_000_000
        th = threading.Thread(target=churn)
        th.start()
        try:
            for it in range(6):
                vals = [r.integers(-2**62, 2**62, n, dtype=np.int64) for _ in range(3)]
                cols = [gdk.BAT.from_numpy(gdk.TYPE_lng, v) for v in vals]
                out, recv = be.exchange_cols(dist, cols, [gdk.TYPE_lng] * 3, [n])
                del cols                     # the caller lets go at once
                assert recv == [n]
                for o, v in zip(out, vals):
                    assert np.array_equal(o.to_numpy(), v), it
        finally:
            stop.set()
            th.join()
        assert not errs, errs
        be.drain(wait=True)
        assert be._pending == []
    finally:
        dist.destroy_process_group()
