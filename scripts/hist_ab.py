"""A/B of the ROOT histogram pass of the headline tree (11M HIGGS shape) in isolation: the real k_hist_build (via
h2o_tree_root = amax + qscale + root histogram + reduce) timed with CUDA events, under switches and data variants.
Run on the GPU box: python scripts/hist_ab.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from llama_github_io_amd.models.base import DataInfo  # noqa: E402
from llama_github_io_amd.models.gbm import GBMTrainer  # noqa: E402
from llama_github_io_amd.ops import tree as T  # noqa: E402
from llama_github_io_amd.ops import _native as nat  # noqa: E402

builders = []
_init = T.GpuTreeBuilder.__init__


def _rec(self, *a, **k):
    _init(self, *a, **k)
    builders.append(self)


T.GpuTreeBuilder.__init__ = _rec


def time_root(b, reps=20):
    P = b._plan
    s = nat.stream_ptr(b.dev)
    ref = ctypes.byref(P)
    for _ in range(3):
        nat.check(b.lib.h2o_tree_root(ref, s), "root")
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        nat.check(b.lib.h2o_tree_root(ref, s), "root")
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
    return float(np.median(ms)) * 1000.0


def main():
    n = int(os.environ.get("ROWS", 11_000_000))
    dev = torch.device("cuda", 0)
    X, y = bench.make_higgs_like(n, 1234, dev)
    F = X.shape[0]
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    p = dict(ntrees=3, max_depth=6, min_rows=10, learn_rate=0.1, seed=42, distribution="bernoulli",
             histogram_type="QuantilesGlobal")
    GBMTrainer(p).fit(X, y, None, None, info)
    b = builders[-1]
    out = {"rows": n, "stride": b.stride, "planar": b.planar}
    out["root_us_default"] = time_root(b)
    os.environ["H2O_HIST_REPL"] = "0"
    out["root_us_no_replicas"] = time_root(b)
    del os.environ["H2O_HIST_REPL"]
    os.environ["H2O_HIST_BUF"] = "0"
    out["root_us_no_buf"] = time_root(b)
    del os.environ["H2O_HIST_BUF"]
    for dbg, tag in (("1", "no_flush"), ("2", "no_atomics"), ("3", "loads_only")):
        os.environ["H2O_HIST_DBG"] = dbg
        out["root_us_" + tag] = time_root(b)
    del os.environ["H2O_HIST_DBG"]
    # data variants: uniform random bins in the real buffer (28 features, zero padding bytes)
    m = b.master
    keep = m.clone()
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    r = torch.randint(0, 255, m.shape, generator=g, device=dev, dtype=torch.int32).to(torch.uint8)
    if not b.planar:
        r[:, F:] = 0
    m.copy_(r)
    out["root_us_uniform_bins"] = time_root(b)
    m.copy_(keep)
    # per-feature distinct bins of the real data (first 1M rows)
    mm = keep[:1_000_000].cpu().numpy() if not b.planar else None
    if mm is not None:
        out["distinct_bins_per_feature"] = [int(len(np.unique(mm[:, f]))) for f in range(F)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
