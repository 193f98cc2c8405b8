"""Row-sharded GPU paths with 2 ranks sharing cuda:0 (gloo carries the collectives; RCCL needs one
GPU per rank, which the 8-GPU driver run exercises). The sharded HIP tree engine / GLM Gram /
KMeans must reproduce the single-process GPU model."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _worker(rank, world, port, algo, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from test_distributed import _data, _info, _train
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X, y = _data()
        N = X.shape[1]
        sl = slice(rank * N // world, (rank + 1) * N // world)
        out = _train(algo, X[:, sl].contiguous().cuda(), y[sl].contiguous().cuda(), _info(X.shape[0]))
        if rank == 0:
            q.put(out.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("algo", ["gbm", "glm", "kmeans"])
def test_gpu_sharded_equals_single(algo):
    import socket
    from test_distributed import _data, _info, _train
    X, y = _data()
    single = _train(algo, X.cuda(), y.cuda(), _info(X.shape[0])).cpu().numpy()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, algo, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert np.allclose(single, res, atol=1e-3, rtol=1e-3), (single[:5], res[:5])
