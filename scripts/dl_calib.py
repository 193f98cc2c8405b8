"""DeepLearning calibration on the bench target (10M x 784 uniform inputs, y = sum of the first 20 > 10, MLP [200, 200]
Rectifier, ADADELTA, 1 epoch): final training logloss / AUC and the scoring history for fp32 vs bf16 compute, with and
without input standardization (H2O's default is standardize=True; the throughput bench runs standardize=False), at
4096-row and 256-row steps. GPU box: python scripts/dl_calib.py [--rows 10000000]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--batches", default="4096")
    a = ap.parse_args()
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    dev = torch.device("cuda", 0)
    N, F = a.rows, 784
    g = torch.Generator(device=dev).manual_seed(11)
    X = torch.rand(F, N, device=dev, generator=g)
    y = (X[:20].sum(0) > 10).float()
    info = DataInfo([f"p{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    for bs in [int(b) for b in a.batches.split(",")]:
        for std in (False, True):
            for cd in ("float32", "bf16"):
                m = DeepLearningTrainer(dict(hidden=[200, 200], epochs=1, compute_dtype=cd, mini_batch_size=bs, seed=1,
                                             stopping_rounds=0, score_interval=0.02, standardize=std,
                                             overwrite_with_best_model=False)).fit(X, y, None, None, info)
                tm = m.output["training_metrics"]
                hist = [(round(e.get("epochs", 0), 3), round(e.get("training_logloss", float("nan")), 4),
                         round(e.get("training_auc", float("nan")), 4)) for e in m.output.get("scoring_history", [])]
                print(json.dumps(dict(batch=bs, standardize=std, dtype=cd, logloss=tm.get("logloss"), auc=tm.get("AUC"),
                                      history=hist[:3] + hist[-3:])), flush=True)


if __name__ == "__main__":
    main()
