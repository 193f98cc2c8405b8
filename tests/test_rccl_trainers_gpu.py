"""Every trainer's collectives through RCCL on the 1-GPU box: a 1-rank ``nccl`` process group with
``H2O_FORCE_SHARDED=1`` makes ``collectives.is_dist()`` true, so GLM (Gram / IRLS all-reduces), KMeans (centroid
sums), DeepLearning (per-step gradient sync AND H2O model averaging), metrics (score-lattice merges), quantiles /
GBM order-statistic leaves (distributed order statistics), isotonic / CoxPH (``exchange_rows`` all-to-all), the
custom-metric reduce, the tree exchange (native RCCL transport) and the frame-level reductions of the parse all run
ProcessGroupNCCL collectives on device tensors. Each case must reproduce the single-process GPU model (reference:
``water/MRTask.java`` — the cluster size never changes the answer), and the sharded run must issue collectives."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = ["glm_default_lambda", "glm_lambda_search", "glm_gaussian_pvalues", "glm_multinomial", "kmeans", "pca",
         "naivebayes", "deeplearning", "deeplearning_avg", "quantile", "quantile_weighted_low", "isotonic",
         "isotonic_weighted", "coxph", "gbm_custom_metric", "gbm_bernoulli", "gbm_quantile", "drf", "xgboost",
         "targetencoder", "svd_gram", "gam_cr", "isolationforest", "upliftdrf", "dt"]


def _worker(mode, port, csv, out_path):
    sys.path.insert(0, HERE)
    os.environ.update(H2O_AMD_DEVICE="cuda", OMP_NUM_THREADS="4", H2O_AGG_CHUNK="250")
    if mode == "rccl":
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                          H2O_FORCE_SHARDED="1")
    import test_distributed_api as T
    T.CASES["deeplearning_avg"] = ("deeplearning", dict(hidden=[8, 8], epochs=2, seed=1, mini_batch_size=64,
                                                        score_interval=1e9), "yb")
    import llama_github_io_amd.parallel.collectives as coll
    orig = T._run_cases

    def run(csv_, names, out):
        os.environ["H2O_DL_DP"] = "sync"
        res = {}
        for n in names:                       # deeplearning_avg: the default model-averaging data parallelism
            os.environ["H2O_DL_DP"] = "average" if n == "deeplearning_avg" else "sync"
            orig(csv_, [n], out)
            with open(out) as f:
                r = json.load(f)
            for k, v in r.items():
                if isinstance(v, dict) and k in res and isinstance(res[k], dict):
                    res[k].update(v)
                else:
                    res[k] = v
        res["backend"] = (__import__("torch.distributed", fromlist=["x"]).get_backend()
                          if coll.world_active() else None)
        with open(out, "w") as f:
            json.dump(res, f)

    run(csv, CASES, out_path)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def _launch(mode, csv, out_path):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = mp.get_context("spawn").Process(target=_worker, args=(mode, port, csv, out_path))
    p.start()
    p.join(900)
    assert p.exitcode == 0, f"{mode} run exited with {p.exitcode}"
    with open(out_path) as f:
        return json.load(f)


def test_all_trainers_through_rccl_match_single(tmp_path):
    sys.path.insert(0, HERE)
    import test_distributed_api as T
    csv = str(tmp_path / "data.csv")
    T._write_csv(csv)
    single = _launch("single", csv, str(tmp_path / "single.json"))
    rccl = _launch("rccl", csv, str(tmp_path / "rccl.json"))
    assert rccl["backend"] == "nccl" and single["backend"] is None
    assert rccl["nrows"] == single["nrows"] and rccl["cat_levels"] == single["cat_levels"]
    assert np.allclose(rccl["mean_x0"], single["mean_x0"], rtol=1e-12)
    bad = []
    for name in CASES:
        a, b = np.asarray(single[name]["pred"]), np.asarray(rccl[name]["pred"])
        tol = 1e-4 if name.startswith(("glm_multinomial", "glm_lambda", "glm_default", "deeplearning")) else 2e-5
        if a.shape != b.shape or not np.allclose(a, b, atol=tol, rtol=tol, equal_nan=True):
            bad.append((name, "pred", float(np.nanmax(np.abs(a - b))) if a.shape == b.shape else "shape"))
        for k, v in single[name]["metrics"].items():
            if abs(v - rccl[name]["metrics"][k]) > tol * max(1.0, abs(v)):
                bad.append((name, k, v, rccl[name]["metrics"][k]))
        # the sharded run goes through the process group; the single process issues none
        if rccl["calls"][name] <= 0:
            bad.append((name, "no collectives"))
        assert single["calls"][name] == 0, name
    assert not bad, bad
