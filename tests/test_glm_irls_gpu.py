"""The fused IRLS pass (k_zbeta's IrlsOut epilogue, ops/gram.irls_wz) against the fp64 torch chain of glm.Family
(linkinv / dlink / variance) it replaces, for every covered family / link pair."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [("gaussian", "identity"), ("binomial", "logit"), ("quasibinomial", "logit"), ("poisson", "log"),
         ("gamma", "inverse"), ("gamma", "log"), ("gaussian", "log"), ("poisson", "identity")]


@pytest.mark.parametrize("fam,link", CASES)
def test_irls_wz_matches_torch_chain(fam, link):
    from llama_github_io_amd.models.glm import Family
    from llama_github_io_amd.ops import gram as G
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    N, P = 100_003, 37
    Z = torch.randn(N, P, device=dev, generator=g)
    beta = 0.05 * torch.randn(P, device=dev, generator=g, dtype=torch.float64)
    if link == "inverse":
        beta[-1] = 2.0
        Z[:, -1] = 1.0
    off = 0.1 * torch.randn(N, device=dev, generator=g, dtype=torch.float64)
    w = torch.rand(N, device=dev, generator=g, dtype=torch.float64) + 0.5
    if fam in ("binomial", "quasibinomial"):
        y = (torch.rand(N, device=dev, generator=g) < 0.4).double()
    elif fam in ("poisson",):
        y = torch.poisson(torch.full((N,), 3.0, device=dev), generator=g).double()
    else:
        y = torch.rand(N, device=dev, generator=g, dtype=torch.float64) * 3 + 0.2
    out = G.irls_wz(Z, beta, off, y, w, fam, link)
    assert out is not None
    f = Family(fam, link)
    eta = G.zbeta(Z, beta, off)
    mu = f.linkinv(eta)
    gp = f.dlink(mu)
    var = f.variance(mu)
    wi = (w / (var * gp * gp).clamp(min=1e-30)).float()
    zi = (eta - off + (y - mu) * gp).float()
    torch.testing.assert_close(out[0], wi, rtol=2e-6, atol=1e-6)
    torch.testing.assert_close(out[1], zi, rtol=2e-6, atol=1e-5)


def test_glm_fit_fused_equals_torch_chain(monkeypatch):
    """A whole binomial IRLSM fit: the fused pass and the torch chain give the same coefficients."""
    import numpy as np
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.glm import GLMTrainer
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    F, N = 12, 200_000
    X = torch.randn(F, N, device=dev, generator=g)
    y = (torch.rand(N, device=dev, generator=g) < torch.sigmoid(X[0] - 0.5 * X[1] + 0.2)).float()
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    prm = dict(family="binomial", lambda_=0.0, standardize=True)
    mf = GLMTrainer(dict(prm)).fit(X, y, None, None, info)
    monkeypatch.setenv("H2O_GLM_FUSED_IRLS", "0")
    mt = GLMTrainer(dict(prm)).fit(X, y, None, None, info)
    assert np.allclose(mf.beta.cpu().numpy(), mt.beta.cpu().numpy(), atol=1e-6)
