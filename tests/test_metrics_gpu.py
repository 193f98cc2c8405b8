"""The binomial metrics' HIP score lattice (csrc/metrics_kernels.hip) against the torch reductions it replaces."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_score_hist_matches_torch(monkeypatch):
    from llama_github_io_amd import metrics as M
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    n = 1_000_003
    p = torch.rand(n, device=dev, generator=g, dtype=torch.float64)
    p[:5] = torch.tensor([0.0, 1.0, 0.5, 1e-9, 1 - 1e-12], dtype=torch.float64)
    y = (torch.rand(n, device=dev, generator=g) < p).double()
    w = torch.rand(n, device=dev, generator=g, dtype=torch.float64) + 0.1
    a = M._score_hist(p, None, None, y=y, w=w)
    monkeypatch.setenv("H2O_METRICS_HIP", "0")
    b = M._score_hist(p, None, None, y=y, w=w)
    torch.testing.assert_close(a[:2], b[:2], rtol=1e-12, atol=1e-9)
    assert torch.equal(a[2], b[2])


def test_binomial_metrics_hip_equals_torch(monkeypatch):
    from llama_github_io_amd import metrics as M
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    n = 300_000
    p = torch.rand(n, device=dev, generator=g)
    y = (torch.rand(n, device=dev, generator=g) < p).float()
    m1 = M.binomial_metrics(y, p)
    monkeypatch.setenv("H2O_METRICS_HIP", "0")
    m0 = M.binomial_metrics(y, p)
    for k in ("AUC", "pr_auc", "logloss", "MSE", "max_f1_threshold"):
        assert abs(m1[k] - m0[k]) < 1e-12, k
