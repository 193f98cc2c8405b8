"""Per-tree device time across a 100-tree GBM job on the bench data (CUDA events around every
boosting iteration), to see how the cost of early trees (the bench's timed window) compares with
the job average. Run on the GPU box."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from llama_github_io_amd.models.base import DataInfo  # noqa: E402
from llama_github_io_amd.models.gbm import GBMTrainer  # noqa: E402

ev = []


class T(GBMTrainer):
    def _prepare(self, t, k):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append(e)
        return super()._prepare(t, k)


def main():
    n = int(os.environ.get("ROWS", 11_000_000))
    dev = torch.device("cuda", 0)
    X, y = bench.make_higgs_like(n, 1234, dev)
    F = X.shape[0]
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    p = dict(ntrees=100, max_depth=6, min_rows=10, learn_rate=0.1, seed=42, distribution="bernoulli",
             histogram_type="QuantilesGlobal")
    GBMTrainer(dict(p, ntrees=3)).fit(X, y, None, None, info)
    m = T(p).fit(X, y, None, None, info)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in zip(ev[:-1], ev[1:])]
    leaves = [t.n_leaves() for t in m.forest.trees]
    print(json.dumps({"ms_trees_0_4": ms[:5], "mean_5_24": float(np.mean(ms[5:25])), "mean_25_98": float(np.mean(ms[25:])),
                      "leaves_5_24": float(np.mean(leaves[5:25])), "leaves_25_99": float(np.mean(leaves[25:]))}), flush=True)


if __name__ == "__main__":
    main()
