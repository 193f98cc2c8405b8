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


@pytest.mark.parametrize("fam,link", CASES)
@pytest.mark.parametrize("P", [13, 37, 63])
def test_gram_irls_matches_two_pass(fam, link, P, monkeypatch):
    """k_gram_irls (eta / wi / zi inside the augmented Gram pass) against irls_wz + gram and the fp64 chain."""
    monkeypatch.setenv("H2O_GLM_GRAM_IRLS", "1")
    from llama_github_io_amd.models.glm import Family
    from llama_github_io_amd.ops import gram as G
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(P)
    N = 200_017
    Z = torch.randn(N, P, device=dev, generator=g)
    beta = 0.05 * torch.randn(P, device=dev, generator=g, dtype=torch.float64)
    if link == "inverse":
        beta[-1] = 2.0
        Z[:, -1] = 1.0
    off = 0.1 * torch.randn(N, device=dev, generator=g, dtype=torch.float64)
    w = torch.rand(N, device=dev, generator=g, dtype=torch.float64) + 0.5
    if fam in ("binomial", "quasibinomial"):
        y = (torch.rand(N, device=dev, generator=g) < 0.4).double()
    elif fam == "poisson":
        y = torch.poisson(torch.full((N,), 3.0, device=dev), generator=g).double()
    else:
        y = torch.rand(N, device=dev, generator=g, dtype=torch.float64) * 3 + 0.2
    out = G.gram_irls(Z, beta, off, y, w, fam, link)
    assert out is not None
    wi, zi = G.irls_wz(Z, beta, off, y, w, fam, link)
    Gt, rt = G.gram(Z, wi, zi)
    scale = float(Gt.abs().max())
    torch.testing.assert_close(out[0], Gt, rtol=1e-5, atol=1e-6 * scale)
    torch.testing.assert_close(out[1], rt, rtol=1e-5, atol=1e-6 * max(scale, float(rt.abs().max())))
    # fp64 oracle of the whole iteration
    f = Family(fam, link)
    eta = Z.double() @ beta + off
    mu = f.linkinv(eta)
    gp = f.dlink(mu)
    wd = w / (f.variance(mu) * gp * gp).clamp(min=1e-30)
    zd = eta - off + (y - mu) * gp
    Zd = Z.double()
    torch.testing.assert_close(out[0], (Zd * wd[:, None]).T @ Zd, rtol=1e-4, atol=1e-4 * scale)
    torch.testing.assert_close(out[1], Zd.T @ (wd * zd), rtol=1e-4, atol=1e-4 * scale)


def test_gram_irls_tiny_and_refusals(monkeypatch):
    """N smaller than one 16-row batch, no offset; P + 1 > 64 and CPU fall back (None)."""
    monkeypatch.setenv("H2O_GLM_GRAM_IRLS", "1")
    from llama_github_io_amd.ops import gram as G
    dev = torch.device("cuda", 0)
    Z = torch.randn(5, 7, device=dev)
    beta = torch.randn(7, device=dev, dtype=torch.float64) * 0.1
    y = torch.rand(5, device=dev, dtype=torch.float64)
    w = torch.ones(5, device=dev, dtype=torch.float64)
    Gm, r = G.gram_irls(Z, beta, None, y, w, "gaussian", "identity")
    Zd = Z.double()
    torch.testing.assert_close(Gm, Zd.T @ Zd, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(r, Zd.T @ y, rtol=1e-5, atol=1e-5)
    assert G.gram_irls(torch.randn(10, 64, device=dev), torch.zeros(64, device=dev, dtype=torch.float64), None,
                       y.new_zeros(10), y.new_ones(10), "gaussian", "identity") is None
    assert G.gram_irls(Z.cpu(), beta.cpu(), None, y.cpu(), w.cpu(), "gaussian", "identity") is None


def test_glm_fit_takes_fused_gram_irls_path(monkeypatch):
    """A GPU IRLSM fit with P + 1 <= 64 runs k_gram_irls: the two-pass kernels are never called, and the fit equals
    the two-pass one (H2O_GLM_GRAM_IRLS=0)."""
    import numpy as np
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.glm import GLMTrainer
    from llama_github_io_amd.ops import gram as G
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(9)
    F, N = 20, 300_000
    X = torch.randn(F, N, device=dev, generator=g)
    y = torch.poisson(torch.exp(0.2 * X[0] - 0.1 * X[1] + 0.5), generator=g)
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", None)
    prm = dict(family="poisson", lambda_=0.0, standardize=True)
    calls = {"fused": 0}
    real = G.gram_irls

    def spy(*a, **k):
        out = real(*a, **k)
        calls["fused"] += out is not None
        return out

    def boom(*a, **k):
        raise AssertionError("two-pass IRLS kernel called on the fused path")

    monkeypatch.setattr(G, "gram_irls", spy)
    monkeypatch.setattr(G, "irls_wz", boom)
    mf = GLMTrainer(dict(prm)).fit(X, y, None, None, info)
    assert calls["fused"] >= 2
    monkeypatch.undo()
    monkeypatch.setenv("H2O_GLM_GRAM_IRLS", "0")
    mt = GLMTrainer(dict(prm)).fit(X, y, None, None, info)
    assert np.allclose(mf.beta.cpu().numpy(), mt.beta.cpu().numpy(), atol=1e-6)
    assert abs(mf.output["residual_deviance"] - mt.output["residual_deviance"]) <= 1e-6 * mt.output["residual_deviance"]
