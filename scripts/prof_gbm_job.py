"""Phase breakdown of the whole 100-tree GBM job on the bench data (binning, bin assignment, builder
setup, tree loop, drain, training metrics, ...): every phase is bracketed by torch.cuda.synchronize so
the host clock measures device time too. Run on the GPU box: python scripts/prof_gbm_job.py."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from llama_github_io_amd.models import shared_tree as st  # noqa: E402
from llama_github_io_amd.models.base import DataInfo  # noqa: E402
from llama_github_io_amd.models.gbm import GBMTrainer  # noqa: E402
from llama_github_io_amd.ops import tree as T  # noqa: E402

PH = {}


def timed(name, fn):
    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        PH[name] = PH.get(name, 0.0) + (time.perf_counter() - t0) * 1e3
        return r
    return w


def main():
    n = int(os.environ.get("ROWS", 11_000_000))
    dev = torch.device("cuda", 0)
    X, y = bench.make_higgs_like(n, 1234, dev)
    F = X.shape[0]
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    params = dict(ntrees=100, max_depth=6, min_rows=10, learn_rate=0.1, seed=42, distribution="bernoulli",
                  histogram_type="QuantilesGlobal")
    GBMTrainer(dict(params, ntrees=3)).fit(X, y, None, None, info)      # module loads / allocations
    st.fit_binning = timed("fit_binning", st.fit_binning)
    st.apply_binning = timed("apply_binning", st.apply_binning)
    T.make_builder = timed("make_builder", T.make_builder)
    for nm in ("_init_model", "_finish", "_training_metrics", "_summary"):
        setattr(GBMTrainer, nm, timed(nm, getattr(GBMTrainer, nm)))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = GBMTrainer(params).fit(X, y, None, None, info)
    torch.cuda.synchronize()
    total = (time.perf_counter() - t0) * 1e3
    PH["total"] = total
    PH["other(tree loop etc)"] = total - sum(v for k, v in PH.items() if k != "total")
    print(json.dumps({k: round(v, 2) for k, v in PH.items()}), flush=True)
    print("AUC", m.output["training_metrics"].get("AUC"), flush=True)


if __name__ == "__main__":
    main()
