"""DeepLearning data parallelism with H2O's model-averaging semantics (gloo, world 2 and 4).

Reference semantics: ``DeepLearningTask.java:169-224`` (each node trains its local model on its own rows for one
iteration, the reduce adds the models and ``postGlobal`` divides by the node count) and
``DeepLearningModelInfo.java:485-536`` (``add``/``div`` cover weights, biases, momenta and the ADADELTA state),
``timeAverage`` (elastic averaging, equation 6 of arXiv:1412.6651).

The reference computation: every rank also trains with ``H2O_DL_DP=local`` (the same local steps, no averaging);
the all-gathered local models, averaged here, must equal the model-averaging run."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data(N=2400, F=6, seed=3):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(F, N, generator=g)
    y = X[0] - 0.5 * X[1] * X[2] + 0.1 * torch.randn(N, generator=g)
    return X, y


def _fit(X, y, **kw):
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    F = X.shape[0]
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", None)
    prm = dict(hidden=[8, 8], seed=5, mini_batch_size=40, standardize=False, overwrite_with_best_model=False,
               stopping_rounds=0, score_interval=1e9, score_training_samples=0, activation="Tanh")
    prm.update(kw)
    m = DeepLearningTrainer(prm).fit(X, y, None, None, info)
    return m, torch.cat([q.detach().reshape(-1) for q in m.net.parameters()]).double()


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      H2O_AMD_DEVICE="cpu", OMP_NUM_THREADS="1")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X, y = _data()
        N = X.shape[1]
        sl = slice(rank * N // world, (rank + 1) * N // world)
        Xs, ys = X[:, sl].contiguous(), y[sl].contiguous()
        kw = dict(case)
        iters = kw.pop("iters")
        # train_samples_per_iteration = one epoch; `iters` epochs = `iters` averaging rounds
        kw.update(epochs=float(iters), train_samples_per_iteration=N)
        os.environ["H2O_DL_DP"] = "local"
        locs = []
        for it in range(1, iters + 1):       # the local trajectory after 1 .. iters iterations
            _, pl = _fit(Xs, ys, **dict(kw, epochs=float(it)))
            parts = [torch.zeros_like(pl) for _ in range(world)]
            dist.all_gather(parts, pl)
            locs.append(torch.stack(parts))
        os.environ["H2O_DL_DP"] = "average"
        m, pa = _fit(Xs, ys, **kw)
        assert m.output["data_parallel"].startswith("model_averaging")
        assert m.output["averaging_rounds"] == iters
        others = [torch.zeros_like(pa) for _ in range(world)]
        dist.all_gather(others, pa)
        if rank == 0:
            q.put((np.stack([t.numpy() for t in locs]), pa.numpy(), np.stack([o.numpy() for o in others])))
    finally:
        dist.destroy_process_group()


def _run(world, case):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=400)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,case", [
    (2, dict(iters=1, adaptive_rate=True)),
    (4, dict(iters=1, adaptive_rate=False, rate=0.01, momentum_start=0.5, momentum_stable=0.5)),
    (2, dict(iters=2, adaptive_rate=True, elastic_averaging=True, elastic_averaging_regularization=0.0,
             elastic_averaging_moving_rate=0.7)),
])
def test_model_averaging_equals_average_of_local_models(world, case):
    locs, pa, others = _run(world, case)
    # every rank ends with the same (averaged / consensus) model
    for o in others:
        np.testing.assert_allclose(o, pa, rtol=0, atol=0)
    if not case.get("elastic_averaging"):
        # one iteration: the average of the local models after that iteration
        np.testing.assert_allclose(pa, locs[-1].mean(0), rtol=1e-5, atol=1e-6)
    else:
        # elastic, no pull (regularization 0): the local models never see the consensus, and the consensus is
        # pa * mean(locals at iteration 2) + (1 - pa) * mean(locals at iteration 1)
        r = case["elastic_averaging_moving_rate"]
        ref = r * locs[1].mean(0) + (1 - r) * locs[0].mean(0)
        np.testing.assert_allclose(pa, ref, rtol=1e-5, atol=1e-6)
    # the local models really differ (each rank trained on its own rows)
    assert np.abs(locs[-1][0] - locs[-1][1]).max() > 1e-3
