"""bench.py's multi-GPU launch on the CPU: `--gpus N` starts N rank processes
itself (no torchrun), the ranks form a process group of N and rank 0 reports
the world size the group saw; a launcher whose world disagrees with --gpus is
refused.  `--dry-dist` stops before any GPU work, so gloo runs it here."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(cmd, env=None, timeout=180):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd="/tmp")


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_n_ranks(n):
    p = _run([sys.executable, BENCH, "--gpus", str(n), "--dist-backend", "gloo", "--dry-dist"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout                 # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["world_size_seen"] == n
    assert d["rank_sum"] == n * (n - 1) // 2          # every rank joined the group
    assert d["dist_backend"] == "gloo"


def test_bench_single_rank_default():
    p = _run([sys.executable, BENCH, "--dry-dist"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_bench_world_mismatch_refused():
    """torchrun with 2 ranks but --gpus 3: every rank exits non-zero."""
    p = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", "29533", BENCH, "--gpus", "3",
              "--dist-backend", "gloo", "--dry-dist"])
    assert p.returncode != 0
    assert "process group has 2 ranks" in p.stderr


def test_pair_hash_order_sensitive():
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    a = np.arange(10, dtype=np.uint64)
    b = a[::-1].copy()
    h = bench._pair_hash(a, b, 0)
    # split into two ranks' slices: the sum of the parts is the whole
    assert (bench._pair_hash(a[:4], b[:4], 0) + bench._pair_hash(a[4:], b[4:], 4)) % (1 << 64) == h
    # swapping two pairs changes it
    a2, b2 = a.copy(), b.copy()
    a2[[2, 3]] = a2[[3, 2]]
    b2[[2, 3]] = b2[[3, 2]]
    assert bench._pair_hash(a2, b2, 0) != h
