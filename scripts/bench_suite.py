#!/usr/bin/env python
"""Secondary benchmarks for the other BASELINE.json configs (one JSON line each, rank 0).

  --which xgb   : XGBoost hist, 500 trees (default --trees), depth 6, on a 100M x 50 synthetic matrix
  --which dl    : DeepLearning MLP [200,200] on 10M x 784 synthetic, bf16 compute, 1 epoch
  --which glm   : GLM binomial on 10k x 20 synthetic CSV through h2o.init()/import_file (plumbing)
  --which kmeans: KMeans k=10 Lloyd iterations on 10M x 20
Rows/features can be reduced with --rows/--cols for quick runs (reported in the config).
Multi-GPU: launch with torchrun; rows are sharded, statistics all-reduced over RCCL.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _sync():
    from llama_github_io_amd.parallel import collectives as coll
    coll.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _emit(d):
    from llama_github_io_amd.parallel import collectives as coll
    if coll.rank() == 0:
        print(json.dumps(d), flush=True)


def bench_xgb(a, dev, world, rank):
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.xgboost import XGBoostTrainer
    N = a.rows or 100_000_000
    F = a.cols or 50
    n = N // world
    g = torch.Generator(device=dev).manual_seed(7 + rank)
    X = torch.randn(F, n, device=dev, generator=g)
    logit = X[0] - 0.5 * X[1] + 0.25 * X[2] * X[3] + 0.3 * torch.sin(X[4])
    y = (torch.rand(n, device=dev, generator=g) < torch.sigmoid(logit)).float()
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    T = a.trees or 500
    _sync()
    t0 = time.perf_counter()
    m = XGBoostTrainer(dict(ntrees=T, max_depth=6, learn_rate=0.3, seed=1, max_bins=256)).fit(X, y, None, None, info)
    _sync()
    dt = time.perf_counter() - t0
    _emit(dict(metric="XGBoost hist train rows/sec (500 trees, depth 6, 100M x 50)", value=N * T / dt / T, unit="rows/s",
               n_gpus=world, seconds=dt, ms_per_tree=dt * 1000 / T, trees=T, rows=N, cols=F,
               train_auc=m.output["training_metrics"]["AUC"], dtype="fp32", data="synthetic"))


def bench_dl(a, dev, world, rank):
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    N = a.rows or 10_000_000
    F = a.cols or 784
    n = N // world
    g = torch.Generator(device=dev).manual_seed(11 + rank)
    X = torch.rand(F, n, device=dev, generator=g)
    y = (X[:20].sum(0) > 10).float()
    info = DataInfo([f"p{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    # untimed warmup fit on a slice: library init / kernel autotuning / graph capture code paths
    DeepLearningTrainer(dict(hidden=[200, 200], epochs=1, compute_dtype="bf16", mini_batch_size=a.batch, seed=1,
                             stopping_rounds=0, score_interval=1e9, standardize=False)).fit(
        X[:, :8 * a.batch].contiguous(), y[:8 * a.batch].contiguous(), None, None, info)
    _sync()
    t0 = time.perf_counter()
    m = DeepLearningTrainer(dict(hidden=[200, 200], epochs=a.epochs, compute_dtype="bf16", mini_batch_size=a.batch,
                                 seed=1, stopping_rounds=0, score_interval=1e9, standardize=False)).fit(X, y, None, None, info)
    _sync()
    dt = time.perf_counter() - t0
    _emit(dict(metric="DeepLearning MLP [200,200] train samples/sec (10M x 784, bf16, data-parallel)",
               value=N * a.epochs / dt, unit="samples/s", n_gpus=world, seconds=dt, rows=N, cols=F, batch=a.batch,
               train_auc=m.output["training_metrics"]["AUC"], dtype="bf16", data="synthetic"))


def bench_glm(a, dev, world, rank):
    import tempfile
    import h2o
    from h2o.estimators import H2OGeneralizedLinearEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(0)
    n, F = a.rows or 10_000, a.cols or 20
    Xn = rng.normal(size=(n, F))
    yb = (rng.random(n) < 1 / (1 + np.exp(-(Xn[:, 0] - Xn[:, 1])))).astype(int)
    path = os.path.join(tempfile.mkdtemp(), "glm.csv")
    np.savetxt(path, np.column_stack([Xn, yb]), delimiter=",", header=",".join([f"x{i}" for i in range(F)] + ["y"]),
               comments="", fmt="%.6f")
    t0 = time.perf_counter()
    fr = h2o.import_file(path)
    fr["y"] = fr["y"].asfactor()
    m = H2OGeneralizedLinearEstimator(family="binomial")
    m.train(y="y", training_frame=fr)
    dt = time.perf_counter() - t0
    _emit(dict(metric="GLM binomial 10k x 20 via h2o.init/import_file/train (seconds)", value=dt, unit="s",
               higher_is_better=False, auc=m.auc(), n_gpus=world))


def bench_kmeans(a, dev, world, rank):
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.kmeans import KMeansTrainer
    N = a.rows or 10_000_000
    F = a.cols or 20
    n = N // world
    g = torch.Generator(device=dev).manual_seed(3 + rank)
    X = torch.randn(F, n, device=dev, generator=g)
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, None, None)
    _sync()
    t0 = time.perf_counter()
    KMeansTrainer(dict(k=10, max_iterations=10, init="Random", seed=1, standardize=False)).fit(X, None, None, None, info)
    _sync()
    dt = time.perf_counter() - t0
    _emit(dict(metric="KMeans k=10, 10 Lloyd iterations, rows/sec", value=N * 10 / dt, unit="rows/s", n_gpus=world,
               seconds=dt, rows=N, cols=F))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="xgb", choices=["xgb", "dl", "glm", "kmeans"])
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--cols", type=int, default=0)
    ap.add_argument("--trees", type=int, default=0)
    ap.add_argument("--epochs", type=float, default=1.0)
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    dict(xgb=bench_xgb, dl=bench_dl, glm=bench_glm, kmeans=bench_kmeans)[a.which](a, dev, world, rank)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
