"""Host-side profile (cProfile) of the GLM 10M x 50 binomial fit of bench_suite --which glm_big: where the fit's
idle GPU gaps come from. usage: python scripts/glm_hostprof.py [--rows N]"""
import argparse
import cProfile
import io
import pstats
import time

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--top", type=int, default=35)
    a = ap.parse_args()
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.glm import GLMTrainer
    dev = torch.device("cuda", 0)
    F, n = 50, a.rows
    g = torch.Generator(device=dev).manual_seed(5)
    X = torch.randn(F, n, device=dev, generator=g)
    beta = torch.linspace(-1, 1, F, device=dev)
    y = (torch.rand(n, device=dev, generator=g) < torch.sigmoid((beta[:, None] * X).sum(0) * 0.3)).float()
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    prm = dict(family="binomial", solver="IRLSM", lambda_=0.0, standardize=True)
    GLMTrainer(dict(prm)).fit(X, y, None, None, info)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    GLMTrainer(dict(prm)).fit(X, y, None, None, info)
    torch.cuda.synchronize()
    pr.disable()
    print(f"fit {1e3 * (time.perf_counter() - t0):.2f} ms (under cProfile)")
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(s.getvalue())


if __name__ == "__main__":
    main()
