#!/usr/bin/env python
"""Secondary benchmarks for the other BASELINE.json configs (one JSON line each, rank 0).

  --which xgb   : XGBoost hist, 500 trees (default --trees), depth 6, on a 100M x 50 synthetic matrix
  --which dl    : DeepLearning MLP [200,200] on 10M x 784 synthetic, bf16 compute, 1 epoch
  --which glm   : GLM binomial on 10k x 20 synthetic CSV through h2o.init()/import_file (plumbing)
  --which kmeans: KMeans k=10 Lloyd iterations on 10M x 20
  --which automl: AutoML (GBM/DRF/GLM/DL/XGBoost + StackedEnsembles) on 1M x 100 within --budget seconds,
                  then the leader's MOJO export -> import_mojo -> prediction parity
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


def _emit(d, iterations=None):
    """One JSON line (rank 0) with the collective counters of the timed fit (calls / bytes through the process
    group's backend: RCCL under torchrun or H2O_FORCE_SHARDED=1) and, given iterations, calls per iteration."""
    from llama_github_io_amd.parallel import collectives as coll
    st = coll.stats()
    d = dict(d, collectives=dict(calls=st["calls"], bytes=st["bytes"], backend=_backend()))
    if iterations:
        d["collectives_per_iteration"] = round(st["calls"] / float(iterations), 2)
    if coll.rank() == 0:
        print(json.dumps(d), flush=True)


def _backend():
    import torch.distributed as dist
    return dist.get_backend() if dist.is_available() and dist.is_initialized() else None


def _reset_stats():
    from llama_github_io_amd.parallel import collectives as coll
    coll.stats(reset=True)


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
    # untimed warmup fit on a slice: library / kernel code objects page in on a fresh box (a cold first fit
    # measured 230 ms/tree instead of ~22)
    XGBoostTrainer(dict(ntrees=2, max_depth=6, learn_rate=0.3, seed=1, max_bins=256)).fit(
        X[:, :1_000_000].contiguous(), y[:1_000_000].contiguous(), None, None, info)
    _sync()
    _reset_stats()
    t0 = time.perf_counter()
    m = XGBoostTrainer(dict(ntrees=T, max_depth=6, learn_rate=0.3, seed=1, max_bins=256)).fit(X, y, None, None, info)
    _sync()
    dt = time.perf_counter() - t0
    _emit(dict(metric="XGBoost hist train rows/sec (500 trees, depth 6, 100M x 50)", value=N * T / dt / T, unit="rows/s",
               n_gpus=world, seconds=dt, ms_per_tree=dt * 1000 / T, trees=T, rows=N, cols=F,
               train_auc=m.output["training_metrics"]["AUC"], dtype="fp32", data="synthetic"), iterations=T)


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
    cd = a.dtype
    DeepLearningTrainer(dict(hidden=[200, 200], epochs=1, compute_dtype=cd, mini_batch_size=a.batch, seed=1,
                             stopping_rounds=0, score_interval=1e9, standardize=a.standardize)).fit(
        X[:, :8 * a.batch].contiguous(), y[:8 * a.batch].contiguous(), None, None, info)
    _sync()
    _reset_stats()
    t0 = time.perf_counter()
    m = DeepLearningTrainer(dict(hidden=[200, 200], epochs=a.epochs, compute_dtype=cd, mini_batch_size=a.batch,
                                 seed=1, stopping_rounds=0, score_interval=1e9, standardize=a.standardize)).fit(X, y, None, None, info)
    _sync()
    dt = time.perf_counter() - t0
    _emit(dict(metric=f"DeepLearning MLP [200,200] train samples/sec (10M x 784, {cd}, data-parallel)",
               value=N * a.epochs / dt, unit="samples/s", n_gpus=world, seconds=dt, rows=N, cols=F, batch=a.batch,
               train_auc=m.output["training_metrics"]["AUC"], train_logloss=m.output["training_metrics"].get("logloss"),
               standardize=a.standardize, dtype=cd, data="synthetic",
               step_mode=m.output.get("training_step_mode"), explicit=m.output.get("training_step_explicit"),
               fused_mfma=m.output.get("training_step_fused_mfma"),
               phases=m.output.get("phase_seconds")), iterations=m.output.get("averaging_rounds") or len(m.output.get("scoring_history") or []) or None)


def bench_automl(a, dev, world, rank):
    import tempfile
    import h2o
    import pandas as pd
    from h2o.automl import H2OAutoML
    h2o.init(verbose=False)
    n, F = a.rows or 1_000_000, a.cols or 100
    g = torch.Generator(device=dev).manual_seed(21)
    X = torch.randn(n, F, device=dev, generator=g)
    logit = X[:, 0] - 0.8 * X[:, 1] + 0.5 * X[:, 2] * X[:, 3] + 0.4 * torch.sin(3 * X[:, 4]) - 0.3 * (X[:, 5] > 1).float()
    y = (torch.rand(n, device=dev, generator=g) < torch.sigmoid(logit)).long()
    df = pd.DataFrame(X.cpu().numpy(), columns=[f"c{i}" for i in range(F)])
    df["y"] = y.cpu().numpy().astype(str)
    fr = h2o.H2OFrame(df, column_types={"y": "enum"})
    _sync()
    t0 = time.perf_counter()
    aml = H2OAutoML(max_runtime_secs=a.budget, max_models=a.trees or None, seed=1, nfolds=3)
    import threading
    stop = threading.Event()

    def beat():   # progress line every 30 s (long AutoML runs must not look silent)
        while not stop.wait(30):
            print(f"[automl] {time.perf_counter() - t0:.0f}s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    try:
        aml.train(y="y", training_frame=fr)
    finally:
        stop.set()
    _sync()
    dt = time.perf_counter() - t0
    lb = aml.leaderboard.as_data_frame()
    leader = aml.leader
    path = leader.download_mojo(tempfile.mkdtemp())
    gm = h2o.import_mojo(path)
    sub = fr[:100000, :]
    pa = leader.predict(sub).as_data_frame().iloc[:, -1].values
    pb = gm.predict(sub).as_data_frame().iloc[:, -1].values
    _emit(dict(metric="AutoML on 1M x 100: models trained within budget + leader MOJO round trip",
               value=len(lb), unit="models", n_gpus=world, seconds=dt, budget_secs=a.budget, rows=n, cols=F,
               leader=str(lb.iloc[0, 0]), leader_auc=float(lb.iloc[0, 1]),
               mojo_max_abs_diff=float(np.max(np.abs(pa - pb))), algos=sorted({str(m).split("_")[0] for m in lb.iloc[:, 0]}),
               leaderboard=[{k: (float(v) if isinstance(v, (int, float, np.floating)) else str(v)) for k, v in r.items()}
                            for r in lb.head(30).to_dict(orient="records")],
               data="synthetic"))


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


def bench_glm_big(a, dev, world, rank):
    """GLM binomial IRLSM on a 10M x 50 device matrix (the MFMA Gram / X'v / Z.beta kernels at scale)."""
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.glm import GLMTrainer
    N = a.rows or 10_000_000
    F = a.cols or 50
    n = N // world
    g = torch.Generator(device=dev).manual_seed(5 + rank)
    X = torch.randn(F, n, device=dev, generator=g)
    beta = torch.linspace(-1, 1, F, device=dev)
    y = (torch.rand(n, device=dev, generator=g) < torch.sigmoid((beta[:, None] * X).sum(0) * 0.3)).float()
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    prm = dict(family="binomial", solver="IRLSM", lambda_=0.0, standardize=True)
    GLMTrainer(dict(prm, max_iterations=1)).fit(X[:, :100000].contiguous(), y[:100000].contiguous(), None, None, info)
    _sync()
    _reset_stats()
    t0 = time.perf_counter()
    m = GLMTrainer(prm).fit(X, y, None, None, info)
    _sync()
    dt = time.perf_counter() - t0
    _emit(dict(metric="GLM binomial IRLSM 10M x 50 (seconds)", value=dt, unit="s", higher_is_better=False,
               iterations=m.output.get("iterations"), auc=m.output["training_metrics"].get("AUC"), rows=N, cols=F,
               n_gpus=world), iterations=m.output.get("iterations"))


def bench_kmeans(a, dev, world, rank):
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.kmeans import KMeansTrainer
    N = a.rows or 10_000_000
    F = a.cols or 20
    n = N // world
    g = torch.Generator(device=dev).manual_seed(3 + rank)
    X = torch.randn(F, n, device=dev, generator=g)
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, None, None)
    KMeansTrainer(dict(k=10, max_iterations=2, init="Random", seed=1, standardize=False)).fit(X, None, None, None, info)
    times, iters = {}, {}
    calls = {}
    for it in (10, 30):
        _sync()
        _reset_stats()
        t0 = time.perf_counter()
        m = KMeansTrainer(dict(k=10, max_iterations=it, init="Random", seed=1, standardize=False)).fit(X, None, None, None, info)
        _sync()
        times[it] = time.perf_counter() - t0
        iters[it] = m.output["iterations"]
        from llama_github_io_amd.parallel import collectives as coll
        calls[it] = coll.stats()["calls"]
    dt = times[10]
    per_iter = (times[30] - times[10]) / max(iters[30] - iters[10], 1)
    _emit(dict(metric="KMeans k=10, 10 Lloyd iterations, rows/sec", value=N * 10 / dt, unit="rows/s", n_gpus=world,
               seconds=dt, rows=N, cols=F, lloyd_ms_per_iteration_end_to_end=round(per_iter * 1e3, 3),
               iterations=iters, fixed_seconds=round(dt - iters[10] * per_iter, 4),
               collectives_per_lloyd_iteration=round((calls[30] - calls[10]) / max(iters[30] - iters[10], 1), 2)),
          iterations=iters[30])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="xgb", choices=["xgb", "dl", "glm", "glm_big", "kmeans", "automl"])
    ap.add_argument("--budget", type=float, default=240.0, help="AutoML max_runtime_secs")
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--cols", type=int, default=0)
    ap.add_argument("--trees", type=int, default=0)
    ap.add_argument("--epochs", type=float, default=1.0)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dtype", default="bf16", help="DeepLearning compute_dtype (bf16 | float32)")
    ap.add_argument("--no-standardize", dest="standardize", action="store_false",
                    help="DeepLearning: skip input standardization (H2O's default standardize=True; unstandardized "
                    "[0, 1] inputs leave the 1-epoch ADADELTA model miscalibrated, profiles/r5_dl_calibration.md)")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    forced = os.environ.get("H2O_FORCE_SHARDED") == "1"
    if world > 1 or forced:
        # H2O_FORCE_SHARDED=1 on one GPU: a 1-rank RCCL group; every trainer takes its sharded path and its
        # collectives run through ProcessGroupNCCL
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    dict(xgb=bench_xgb, dl=bench_dl, glm=bench_glm, glm_big=bench_glm_big, kmeans=bench_kmeans, automl=bench_automl)[a.which](a, dev, world, rank)
    if world > 1 or forced:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
