"""Regression: the binomial threshold table indexes ``uniq`` on a float64 lattice.

A float32 ``linspace(0, n - 1)`` rounds ``n - 1`` up past 2^24 distinct scores; the last index then
pointed one element past the end (on the GPU an out-of-bounds gather: the HSA 0x1016 memory fault of
the 100M x 50 XGBoost run)."""
import torch

from llama_github_io_amd import metrics


def test_threshold_table_index_in_bounds_past_2_pow_24():
    n = (1 << 25) + 4          # n - 1 = 2^25 + 3 is not a float32 value (rounds up to 2^25 + 4 = n)
    assert int(torch.linspace(0, n - 1, steps=400)[-1].round()) > n - 1   # the old lattice overflowed
    uniq = torch.arange(n, dtype=torch.float32).flip(0) / n
    tp = torch.arange(1, n + 1, dtype=torch.float32)
    fp = torch.zeros(n, dtype=torch.float32)
    rows = metrics._threshold_table(uniq, tp, fp, 400)
    assert len(rows) == 400
    assert rows[-1]["threshold"] == float(uniq[-1])


def test_lattice_path_masks_excluded_rows(monkeypatch):
    """Lattice-path binomial metrics keep NaN-response / zero-weight rows in place with weight 0 (no compaction):
    every metric equals the one computed on the compacted rows."""
    import torch
    from llama_github_io_amd import metrics as M
    monkeypatch.setattr(M, "LATTICE_AUC_ROWS", 1000)
    g = torch.Generator().manual_seed(11)
    n = 20_000
    p = torch.rand(n, generator=g, dtype=torch.float64)
    y = (torch.rand(n, generator=g, dtype=torch.float64) < p).double()
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.1
    y[::7] = float("nan")
    w[::11] = 0.0
    p[::7] = float("nan")          # excluded rows may carry any score
    ok = ~torch.isnan(y) & (w > 0)
    a = M.binomial_metrics(y, p, w)
    b = M.binomial_metrics(y[ok], p[ok], w[ok])
    assert a["nobs"] == b["nobs"] == int(ok.sum())
    for k in ("MSE", "logloss", "AUC", "pr_auc", "r2", "max_f1_threshold"):
        assert abs(a[k] - b[k]) <= 1e-12 * max(1.0, abs(b[k])), k
    assert a["thresholds_and_metric_scores"] == b["thresholds_and_metric_scores"]
    assert a["gains_lift_table"] == b["gains_lift_table"]
