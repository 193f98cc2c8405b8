#!/usr/bin/env python
"""Phase clocks of k_dl_rows (diagnostic build: scripts/build_alt.sh dlt -DDL_TIMING, run with
H2O_HIP_LIB=llama_github_io_amd/lib_alt/dlt.so): trains the DL bench shape, then prints per-phase durations of
the last fused step's workgroups (wall clock, 100 MHz)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    N, F, B = 262144, 784, 4096
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(11)
    X = torch.rand(F, N, device=dev, generator=g)
    y = (X[:20].sum(0) > 10).float()
    info = DataInfo([f"p{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    DeepLearningTrainer(dict(hidden=[200, 200], epochs=1, compute_dtype=dt, mini_batch_size=B, seed=1,
                             stopping_rounds=0, score_interval=1e9, standardize=False)).fit(X, y, None, None, info)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.environ["H2O_HIP_LIB"])
    nb = B // 16
    buf = (ctypes.c_ulonglong * (4096 * 16))()
    assert lib.h2o_dl_timing(buf, 4096 * 16) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 16)[:nb].astype(np.int64)
    marks = [0, 1, 2, 3, 4, 8, 10, 9, 15]
    names = ["zero+meta", "gather x", "fwd l1 (+hT0)", "fwd l2", "output", "bwd l2", "bwd l1", "tail"]
    t0 = t[:, 0].min()
    print(f"{dt}: {nb} workgroups; start spread {(t[:, 0].max() - t0) / 100:.2f} us, "
          f"kernel span {(t[:, 15].max() - t0) / 100:.2f} us, mean WG life {(t[:, 15] - t[:, 0]).mean() / 100:.2f} us")
    for i in range(len(marks) - 1):
        d = (t[:, marks[i + 1]] - t[:, marks[i]]) / 100.0
        print(f"  {names[i]:14s} mean {d.mean():7.2f} us  p10 {np.percentile(d, 10):7.2f}  p90 {np.percentile(d, 90):7.2f}")


if __name__ == "__main__":
    main()
