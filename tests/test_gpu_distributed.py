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
