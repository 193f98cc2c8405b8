"""fit_binning's batched edge extraction (two gathers + one nonzero, one host copy each) gives exactly the edges of
the per-feature algorithm (GlobalQuantilesCalc: all distinct values when <= max_bins, else quantile cut points)."""
import numpy as np
import torch

from llama_github_io_amd.ops.binning import fit_binning


def _ref_edges(x, max_bins):
    x = torch.where(torch.isnan(x), torch.full_like(x, float("inf")), x)
    row_all, _ = torch.sort(x)
    n = int(torch.isfinite(row_all).sum())
    if n == 0:
        return np.zeros(0, np.float32)
    row = row_all[:n]
    nd = int(((row_all[1:] != row_all[:-1]) & torch.isfinite(row_all[1:])).sum() + torch.isfinite(row_all[:1]).sum())
    if nd <= max_bins:
        e = torch.unique_consecutive(row)[1:]
    else:
        q = (torch.arange(1, max_bins, dtype=torch.int64) * n) // max_bins
        e = torch.unique_consecutive(row[q])
        e = e[e > row[0]]
    return e.float().numpy()


def test_batched_edges_match_per_feature_algorithm():
    g = torch.Generator().manual_seed(0)
    N = 50_000
    cols = [torch.randn(N, generator=g),
            torch.randint(0, 3, (N,), generator=g).float(),            # 3 distinct values
            torch.randint(0, 300, (N,), generator=g).float(),          # 300 distinct (> 255): quantiles with ties
            torch.full((N,), 7.0),                                      # constant
            torch.randn(N, generator=g).exp() ** 3]                     # heavy tail
    nanc = torch.randn(N, generator=g)
    nanc[::7] = float("nan")
    cols.append(nanc)
    ninf = torch.randn(N, generator=g)
    ninf[:5] = float("-inf")                                           # -inf: the per-feature fallback
    cols.append(ninf)
    X = torch.stack(cols)
    F = X.shape[0]
    for mb in (255, 64):
        b = fit_binning(X, np.zeros(F, np.int32), max_bins=mb, sample=1 << 20)
        for f in range(F):
            np.testing.assert_array_equal(b.edges[f], _ref_edges(X[f], mb), err_msg=f"feature {f} max_bins {mb}")
