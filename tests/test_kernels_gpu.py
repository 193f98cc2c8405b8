"""HIP kernels vs fp32/fp64 PyTorch references of the same op (run on an MI355X)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def test_native_library_loads():
    from llama_github_io_amd.ops import _native
    lib = _native.hip()
    assert lib is not None and hasattr(lib, "h2o_gram") and hasattr(lib, "h2o_kmeans_assign")


@pytest.mark.parametrize("N,P", [(1000, 7), (70001, 64), (5000, 130), (33, 200)])
def test_gram_matches_fp64(N, P):
    from llama_github_io_amd.ops.gram import gram, xtv
    g = torch.Generator(device=dev).manual_seed(N + P)
    Z = torch.randn(N, P, device=dev, generator=g)
    w = torch.rand(N, device=dev, generator=g)
    G = gram(Z, w)
    ref = (Z.double() * w.double()[:, None]).T @ Z.double()
    scale = (Z.double().abs() * w.double()[:, None]).T @ Z.double().abs()
    assert torch.all((G - ref).abs() <= 1e-5 * scale + 1e-6)
    v = torch.randn(N, 3, device=dev, generator=g)
    assert torch.allclose(xtv(Z, v), Z.double().T @ v.double(), rtol=1e-4, atol=1e-3)
    assert torch.allclose(gram(Z), Z.double().T @ Z.double(), rtol=1e-4, atol=1e-2)
    # augmented pass (GLM IRLS): Zᵀ W Z and Zᵀ W u from one read of Z
    u = torch.randn(N, device=dev, generator=g)
    G2, r = gram(Z, w, u)
    assert torch.all((G2 - ref).abs() <= 1e-5 * scale + 1e-6)
    rref = (Z.double() * w.double()[:, None]).T @ u.double()
    rsc = (Z.double().abs() * w.double()[:, None]).T @ u.double().abs()
    assert torch.all((r - rref).abs() <= 1e-5 * rsc + 1e-6)


def test_kmeans_assign_matches_reference():
    from llama_github_io_amd.ops.dense import kmeans_assign
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(10007, 13, device=dev, generator=g)
    C = torch.randn(9, 13, device=dev, generator=g)
    a, d = kmeans_assign(X, C)
    D = ((X[:, None, :].double() - C[None].double()) ** 2).sum(-1)
    dref, aref = D.min(1)
    assert (a == aref).float().mean() > 0.999
    assert torch.allclose(d.double(), dref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("act", ["rectifier", "tanh", "exprectifier", "linear"])
@pytest.mark.parametrize("drop", [0.0, 0.3])
def test_bias_act_fwd_bwd(act, drop):
    from llama_github_io_amd.ops.dense import bias_act
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn(517, 70, device=dev, generator=g)
    b = torch.randn(70, device=dev, generator=g)
    gy = torch.randn(517, 70, device=dev, generator=g)
    xg = x.clone().requires_grad_(True)
    bg = b.clone().requires_grad_(True)
    y = bias_act(xg, bg, act, drop, 1234)
    y.backward(gy)
    xc = x.cpu().requires_grad_(True)
    bc = b.cpu().requires_grad_(True)
    yc = bias_act(xc, bc, act, drop, 1234)
    yc.backward(gy.cpu())
    assert torch.allclose(y.cpu(), yc, atol=1e-5, rtol=1e-5)
    assert torch.allclose(xg.grad.cpu(), xc.grad, atol=1e-5, rtol=1e-5)
    assert torch.allclose(bg.grad.cpu(), bc.grad, atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("act", ["rectifier", "tanh"])
@pytest.mark.parametrize("drop", [0.0, 0.3])
def test_bias_act_bf16_matches_fp32_reference(act, drop):
    # bf16 activations in/out (fp32 bias + math): equal to the fp32 PyTorch reference up to bf16 rounding
    from llama_github_io_amd.ops.dense import bias_act
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(4096, 200, device=dev, generator=g)
    b = torch.randn(200, device=dev, generator=g)
    gy = torch.randn(4096, 200, device=dev, generator=g)
    xb = x.bfloat16().requires_grad_(True)
    bg = b.clone().requires_grad_(True)
    y = bias_act(xb, bg, act, drop, 77)
    assert y.dtype == torch.bfloat16
    y.backward(gy.bfloat16())
    xc = xb.detach().float().cpu().requires_grad_(True)
    bc = b.cpu().requires_grad_(True)
    yc = bias_act(xc, bc, act, drop, 77)
    yc.backward(gy.bfloat16().float().cpu())
    assert torch.allclose(y.float().cpu(), yc, atol=2e-2, rtol=1e-2)
    assert torch.allclose(xb.grad.float().cpu(), xc.grad, atol=3e-2, rtol=2e-2)
    assert torch.allclose(bg.grad.cpu(), bc.grad, atol=0.5, rtol=1e-2)


def _info(F, dom=("0", "1")):
    from llama_github_io_amd.models.base import DataInfo
    return DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", list(dom) if dom else None)


def test_glm_gpu_matches_cpu():
    from llama_github_io_amd.models.glm import GLMTrainer
    g = torch.Generator().manual_seed(0)
    X = torch.randn(6, 20000, generator=g)
    y = (torch.rand(20000, generator=g) < torch.sigmoid(X[0] - 2 * X[1] + 0.3)).float()
    mc = GLMTrainer(dict(family="binomial", lambda_=0.0)).fit(X, y, None, None, _info(6))
    mg = GLMTrainer(dict(family="binomial", lambda_=0.0)).fit(X.to(dev), y.to(dev), None, None, _info(6))
    assert np.allclose(mc.beta.cpu().numpy(), mg.beta.cpu().numpy(), atol=1e-4)


def test_tree_family_trains_on_gpu():
    from llama_github_io_amd.models.drf import DRFTrainer
    from llama_github_io_amd.models.isoforest import IsolationForestTrainer
    from llama_github_io_amd.models.xgboost import XGBoostTrainer
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(8, 50000, device=dev, generator=g)
    y = (torch.rand(50000, device=dev, generator=g) < torch.sigmoid(2 * X[0] - X[1] * X[2])).float()
    m = DRFTrainer(dict(ntrees=10, max_depth=8, seed=1)).fit(X, y, None, None, _info(8))
    assert m.output["training_metrics"]["AUC"] > 0.75
    m = XGBoostTrainer(dict(ntrees=10, seed=1)).fit(X, y, None, None, _info(8))
    assert m.output["training_metrics"]["AUC"] > 0.8
    # forest scoring kernel == torch traversal
    fr = m.forest
    a = fr.predict_raw(X[:, :5000])
    b = fr.predict_raw(X[:, :5000].cpu())
    assert torch.allclose(a.cpu(), b, atol=1e-5)
    Xo = torch.cat([X[:, :2000], X[:, :20] * 8], 1)
    m = IsolationForestTrainer(dict(ntrees=30, seed=1)).fit(Xo, None, None, None, _info(8, None))
    P = m._predict_tensor(Xo)
    assert float(P[-20:, 0].mean()) > float(P[:2000, 0].mean())


def test_xgboost_lossguide_on_gpu():
    """max_leaves pruning on the GPU builder: leaf count bound, GPU == CPU trees, margins == forest scoring."""
    from llama_github_io_amd.models.xgboost import XGBoostTrainer
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(8, 40000, device=dev, generator=g)
    y = (torch.rand(40000, device=dev, generator=g) < torch.sigmoid(2 * X[0] - X[1] * X[2])).float()
    prm = dict(ntrees=6, max_depth=6, seed=1, grow_policy="lossguide", max_leaves=9)
    tr = XGBoostTrainer(dict(prm))
    m = tr.fit(X, y, None, None, _info(8))
    assert all(t.n_leaves() <= 9 for t in m.forest.trees)
    raw = m.forest.predict_raw(X)
    assert torch.allclose(raw.reshape(-1).cpu(), tr.f[:, 0].cpu(), atol=1e-4)
    mc = XGBoostTrainer(dict(prm)).fit(X.cpu(), y.cpu(), None, None, _info(8))
    assert [t.n_leaves() for t in mc.forest.trees][:1] == [t.n_leaves() for t in m.forest.trees][:1]


def test_deeplearning_gpu_learns():
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(6, 20000, device=dev, generator=g)
    y = ((X[0] * X[1] + X[2]) > 0).float()
    m = DeepLearningTrainer(dict(hidden=[64, 64], epochs=3, seed=1)).fit(X, y, None, None, _info(6))
    assert m.output["training_metrics"]["AUC"] > 0.9


def test_fused_adadelta_matches_reference():
    from llama_github_io_amd.ops.dense import FlatParams
    torch.manual_seed(0)
    net_c = torch.nn.Sequential(torch.nn.Linear(37, 19), torch.nn.Linear(19, 3))
    net_g = torch.nn.Sequential(torch.nn.Linear(37, 19), torch.nn.Linear(19, 3)).to(dev)
    net_g.load_state_dict({k: v.to(dev) for k, v in net_c.state_dict().items()})
    fc, fg = FlatParams(net_c), FlatParams(net_g)
    x = torch.randn(64, 37)
    for _ in range(3):
        for net, f, xx in ((net_c, fc, x), (net_g, fg, x.to(dev))):
            f.zero_grad()
            net(xx).square().mean().backward()
            f.adadelta(0.99, 1e-8, l1=1e-4, l2=1e-3)
    assert torch.allclose(fc.p, fg.p.cpu(), atol=1e-6, rtol=1e-5)
    assert torch.allclose(fc.eg2, fg.eg2.cpu(), atol=1e-9, rtol=1e-4)


@pytest.mark.parametrize("wt_dtype", [torch.bfloat16, torch.float32])
def test_tiled_adadelta_with_transposed_copy(wt_dtype):
    """k_adadelta_tiles (64 x 64 weight tiles through LDS): master weights, bf16 shadow and the transposed copy of
    every layer (edge tiles included) against the fp32 reference update."""
    import numpy as np
    from llama_github_io_amd.ops.dense import FlatParams
    torch.manual_seed(1)
    dims = [100, 70, 130, 3]
    lins = [torch.nn.Linear(a, b) for a, b in zip(dims[:-1], dims[1:])]
    fc, fg = FlatParams(torch.nn.Sequential(*lins)), FlatParams(torch.nn.Sequential(*[
        torch.nn.Linear(a, b) for a, b in zip(dims[:-1], dims[1:])]).to(dev))
    fg.p.copy_(fc.p.to(dev))
    offs, o = [], 0
    for a, b in zip(dims[:-1], dims[1:]):
        offs.append(o)
        o += a * b
    assert o == fc.n_decay
    wt = torch.zeros(fc.n_decay, dtype=wt_dtype, device=dev)
    shadow = torch.zeros(fc.n_decay, dtype=torch.bfloat16, device=dev)
    wmap = (wt, np.array(offs + [o], np.int64), np.array(dims[:-1], np.int32), np.array(dims[1:], np.int32))
    for it in range(3):
        gr = torch.randn(fc.g.numel(), generator=torch.Generator().manual_seed(it))
        fc.g.copy_(gr)
        fg.g.copy_(gr.to(dev))
        fc.adadelta(0.99, 1e-8, l1=1e-4, l2=1e-3)
        fg.adadelta(0.99, 1e-8, l1=1e-4, l2=1e-3, shadow=shadow, wt=wmap)
    assert torch.allclose(fc.p, fg.p.cpu(), atol=1e-6, rtol=1e-5)
    assert torch.allclose(fc.edx2, fg.edx2.cpu(), atol=1e-9, rtol=1e-4)
    assert torch.equal(shadow.cpu(), fg.p[:o].cpu().bfloat16())
    for l, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        W = fg.p[offs[l]:offs[l] + a * b].view(b, a)
        assert torch.equal(wt[offs[l]:offs[l] + a * b].view(a, b).cpu(), W.t().to(wt_dtype).cpu()), l


@pytest.mark.parametrize("n,C", [(7, 0), (5000, 0), (9, 13), (3000, 4)])
def test_segment_sum_paths(n, C):
    from llama_github_io_amd.ops.segment import segment_sum
    g = torch.Generator(device=dev).manual_seed(n)
    N = 200000
    idx = torch.randint(0, n, (N,), device=dev, generator=g)
    v = torch.randn((N,) if C == 0 else (N, C), device=dev, generator=g)
    got = segment_sum(idx, v, n)
    ref = torch.zeros(got.shape, dtype=torch.float64).index_add_(0, idx.cpu(), v.cpu().double())
    assert torch.allclose(got.cpu(), ref, atol=1e-6, rtol=1e-6)


def test_kmeans_step_kernel():
    from llama_github_io_amd.ops.dense import kmeans_step
    g = torch.Generator(device=dev).manual_seed(3)
    X = torch.randn(100003, 11, device=dev, generator=g)
    C = torch.randn(6, 11, device=dev, generator=g)
    w = torch.rand(100003, device=dev, generator=g)
    a, d, sums, cnt = kmeans_step(X, C, w)
    D = ((X[:, None, :].double() - C[None].double()) ** 2).sum(-1)
    aref = D.argmin(1)
    assert (a == aref).float().mean() > 0.999
    ref = torch.zeros(6, 11, dtype=torch.float64, device=dev).index_add_(0, a, X.double() * w.double()[:, None])
    cref = torch.zeros(6, dtype=torch.float64, device=dev).index_add_(0, a, w.double())
    assert torch.allclose(sums, ref, rtol=1e-4, atol=1e-2) and torch.allclose(cnt, cref, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("N,K,P,weighted", [(100003, 10, 20, True), (4099, 37, 52, False), (20000, 64, 64, True),
                                             (777, 1, 4, False), (50001, 17, 36, True)])
def test_kmeans_mfma_lloyd_matches_fp32_reference(N, K, P, weighted, monkeypatch):
    """csrc/kmeans_mfma.hip (distance + centroid GEMMs on v_mfma_f32_16x16x4_f32) vs a plain PyTorch fp32/fp64
    reference of the same Lloyd step: argmin, min distance, per-center weighted sums and counts."""
    from llama_github_io_amd.ops.dense import _mfma_shape, kmeans_step
    monkeypatch.setenv("H2O_KMEANS_MFMA", "1")
    assert _mfma_shape(K, P) is not None
    g = torch.Generator(device=dev).manual_seed(N + K)
    X = torch.randn(N, P, device=dev, generator=g)
    C = torch.randn(K, P, device=dev, generator=g)
    w = torch.rand(N, device=dev, generator=g) if weighted else None
    a, d, sums, cnt = kmeans_step(X, C, w)
    D = ((X[:, None, :].double() - C[None].double()) ** 2).sum(-1)
    dref, aref = D.min(1)
    # disagreements only on numerical near-ties
    mism = a != aref
    if mism.any():
        gap = (D.gather(1, a[:, None])[:, 0] - dref)[mism]
        assert float(gap.max()) < 1e-3 * float(dref[mism].abs().max() + 1)
    assert torch.allclose(d.double(), D.gather(1, a[:, None])[:, 0], rtol=1e-4, atol=1e-3)
    wd = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
    ref = torch.zeros(K, P, dtype=torch.float64, device=dev).index_add_(0, a, X.double() * wd[:, None])
    cref = torch.zeros(K, dtype=torch.float64, device=dev).index_add_(0, a, wd)
    assert torch.allclose(sums, ref, rtol=1e-4, atol=1e-2) and torch.allclose(cnt, cref, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("extra", [{}, dict(activation="RectifierWithDropout", hidden_dropout_ratios=[0.3, 0.2]),
                                   dict(adaptive_rate=False, rate=0.01, momentum_start=0.5, momentum_stable=0.9,
                                        momentum_ramp=5000, max_w2=2.0, l2=1e-4)])
def test_deeplearning_graph_matches_eager(extra, monkeypatch):
    # the captured step (device step counter for the dropout hash, device rate / momentum scalars) replays
    # exactly what the eager loop computes step by step
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(6, 8192, device=dev, generator=g)
    y = ((X[0] * X[1] + X[2]) > 0).float()
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("H2O_DL_GRAPH", flag)
        m = DeepLearningTrainer(dict(dict(hidden=[32, 32], epochs=2, seed=3, mini_batch_size=512, score_interval=1e9,
                                          stopping_rounds=0), **extra)).fit(X, y, None, None, _info(6))
        res.append(torch.cat([q.detach().reshape(-1) for q in m.net.parameters()]).cpu())
    assert torch.allclose(res[0], res[1], atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("dist", ["gaussian", "bernoulli", "poisson", "gamma", "tweedie", "laplace", "quantile",
                                  "huber", "quasibinomial"])
def test_fused_gbm_step_matches_eager_path(dist, monkeypatch):
    # k_gbm_step (residuals + leaf terms + sampling + f update in one HIP pass) and k_leaf_values
    # == the PyTorch per-distribution path of GBMTrainer on the same device
    from llama_github_io_amd.models.gbm import GBMTrainer
    g = torch.Generator(device=dev).manual_seed(5)
    N, F = 20000, 6
    X = torch.randn(F, N, device=dev, generator=g)
    eta = 0.6 * X[0] - 0.4 * X[1] + 0.3 * X[2] * X[3]
    if dist in ("bernoulli", "quasibinomial"):
        y = (torch.rand(N, device=dev, generator=g) < torch.sigmoid(eta)).float()
        dom = ("0", "1")
    elif dist in ("poisson", "tweedie"):
        y = torch.poisson(torch.exp(eta), generator=g)
        dom = None
    elif dist == "gamma":
        y = torch.exp(eta) * torch.distributions.Gamma(2.0, 2.0).sample((N,)).to(dev)
        dom = None
    else:
        y = eta + 0.3 * torch.randn(N, device=dev, generator=g)
        dom = None
    params = dict(ntrees=8, max_depth=4, seed=3, distribution=dist, sample_rate=0.8)
    fused = GBMTrainer(dict(params)).fit(X, y, None, None, _info(F, dom))
    monkeypatch.setattr(GBMTrainer, "_fused", lambda self: False)
    eager = GBMTrainer(dict(params)).fit(X, y, None, None, _info(F, dom))
    a = fused.score_tensor(X).double().cpu()
    b = eager.score_tensor(X).double().cpu()
    # the row sampling masks come from different generators (hash in-kernel vs torch.rand): compare
    # model quality, and exact structure when sampling is off
    ta, tb = fused.output["training_metrics"], eager.output["training_metrics"]
    key = "logloss" if dom else "MSE"
    assert abs(ta[key] - tb[key]) <= 0.05 * abs(tb[key]) + 1e-3, (ta[key], tb[key])
    params["sample_rate"] = 1.0
    monkeypatch.undo()
    f1 = GBMTrainer(dict(params)).fit(X, y, None, None, _info(F, dom))
    monkeypatch.setattr(GBMTrainer, "_fused", lambda self: False)
    e1 = GBMTrainer(dict(params)).fit(X, y, None, None, _info(F, dom))
    np.testing.assert_allclose(f1.score_tensor(X).double().cpu().numpy(), e1.score_tensor(X).double().cpu().numpy(),
                               rtol=2e-4, atol=2e-5)
    _ = (a, b)


@pytest.mark.parametrize("N,P,R", [(1000, 7, 1), (70001, 51, 1), (5000, 130, 3), (33, 200, 8), (37, 13001, 2)])
def test_zbeta_matches_fp64(N, P, R):
    # GLM linear predictor: fp32 design read once, fp64 accumulation (k_zbeta) vs the fp64 matmul
    from llama_github_io_amd.ops.gram import zbeta
    g = torch.Generator(device=dev).manual_seed(N + P)
    Z = torch.randn(N, P, device=dev, generator=g)
    B = torch.randn(P, R, device=dev, generator=g, dtype=torch.float64)
    off = torch.randn(N, device=dev, generator=g, dtype=torch.float64)
    ref = Z.double() @ B + off[:, None]
    out = zbeta(Z, B, off)
    assert out.dtype == torch.float64 and torch.allclose(out, ref, rtol=1e-12, atol=1e-10)
    assert torch.allclose(zbeta(Z, B[:, 0]), Z.double() @ B[:, 0], rtol=1e-12, atol=1e-10)


@pytest.mark.parametrize("dtype", ["float32", "bf16"])
def test_deeplearning_explicit_step_matches_autograd_gpu(dtype, monkeypatch):
    # explicit MLP step (bf16 weight shadows from the fused ADADELTA, k_out_grad, epilogue bias grads) vs the
    # autograd step, both replayed from graphs
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(12, 16384, device=dev, generator=g)
    y = ((X[0] * X[1] + X[2]) > 0).float()
    res, aucs = [], []
    for flag in ("0", "1"):
        monkeypatch.setenv("H2O_DL_EXPLICIT", flag)
        m = DeepLearningTrainer(dict(hidden=[64, 64], epochs=2, seed=3, mini_batch_size=512, score_interval=1e9,
                                     stopping_rounds=0, compute_dtype=dtype)).fit(X, y, None, None, _info(12))
        assert m.output["training_step_explicit"] == (flag == "1")
        res.append(torch.cat([q.detach().reshape(-1) for q in m.net.parameters()]).cpu())
        aucs.append(m.output["training_metrics"]["AUC"])
    if dtype == "float32":
        assert torch.allclose(res[0], res[1], atol=1e-4, rtol=1e-3)
    else:   # bf16 GEMMs: the two paths round differently; both must learn equally well
        assert abs(aucs[0] - aucs[1]) < 0.02 and min(aucs) > 0.88


@pytest.mark.parametrize("standardize", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,cat", [(10001, True), (10000, False)])
def test_expander_hip_matches_cpu(standardize, dtype, N, cat):
    # k_num_stats / k_num_transform (NaN fill, centring, scaling, transpose) vs the PyTorch path; N % 4 == 0
    # without categoricals takes the 16-byte read / write paths
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.datainfo import Expander
    g = torch.Generator().manual_seed(4)
    F = 70
    X = torch.randn(F, N, generator=g) * 3 + 1
    X[2, ::7] = float("nan")
    iscat = np.zeros(F, np.int32)
    doms = [None] * F
    if cat:
        X[5] = torch.randint(0, 4, (N,), generator=g).float()
        X[5, ::11] = float("nan")
        iscat[5] = 1
        doms[5] = ["a", "b", "c", "d"]
    info = DataInfo([f"x{i}" for i in range(F)], iscat, doms, "y", None)
    w = torch.rand(N, generator=g).double()
    ec = Expander(info, standardize=standardize).fit(X, w)
    eg = Expander(info, standardize=standardize).fit(X.to(dev), w.to(dev))
    assert torch.allclose(ec.num_mean, eg.num_mean.cpu(), rtol=1e-9, atol=1e-9)
    assert torch.allclose(ec.num_sd, eg.num_sd.cpu(), rtol=1e-9, atol=1e-9)
    Zc = ec.transform(X, dtype=torch.float32)
    Zg = eg.transform(X.to(dev), dtype=dtype).float().cpu()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert torch.allclose(Zc, Zg, rtol=tol, atol=tol)


@pytest.mark.parametrize("F", [7, 50, 63, 64, 65])
@pytest.mark.parametrize("N", [10000, 10003, 129])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_expander_extra_column_matches_cpu(F, N, dtype):
    # the whole-row layout with the constant extra (intercept) column: k_num_transform's contiguous-span store
    # (F + 1 <= 65 columns) and the strided-fill fallback (F > 64) against the PyTorch path
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.datainfo import Expander
    g = torch.Generator().manual_seed(F + N)
    X = torch.randn(F, N, generator=g) * 2 - 1
    X[0, ::5] = float("nan")
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", None)
    ec = Expander(info, standardize=True).fit(X, None)
    eg = Expander(info, standardize=True).fit(X.to(dev), None)
    Zc = ec.transform(X, dtype=torch.float32, extra=1.0)
    Zg = eg.transform(X.to(dev), dtype=dtype, extra=1.0).float().cpu()
    assert Zg.shape == (N, F + 1)
    assert bool((Zg[:, F] == 1.0).all())
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert torch.allclose(Zc, Zg, rtol=tol, atol=tol)


@pytest.mark.parametrize("init", ["Furthest", "PlusPlus", "Random"])
def test_kmeans_offset_data_matches_cpu(init):
    """standardize=False on columns offset by 1e4: the training space is centred, so the MFMA
    distance GEMM does not cancel; the device run (pipelined MFMA Lloyd step, device-side seeding,
    speculative convergence check) finds the same clustering as the CPU reference path."""
    from llama_github_io_amd.models.kmeans import KMeansTrainer
    g = torch.Generator().manual_seed(5)
    N, F = 60000, 6
    centers = torch.randn(4, F, generator=g) * 4
    lab = torch.randint(0, 4, (N,), generator=g)
    X = (centers[lab] + 0.3 * torch.randn(N, F, generator=g)).T.contiguous() + 1e4
    info = _info(F)
    info.response = None
    prm = dict(k=4, max_iterations=20, init=init, seed=7, standardize=False)
    mg = KMeansTrainer(prm).fit(X.to(dev), None, None, None, info)
    mc = KMeansTrainer(prm).fit(X, None, None, None, info)
    cg = np.array(mg.output["centers"])
    cc = np.array(mc.output["centers"])
    np.testing.assert_allclose(cg, cc, rtol=0, atol=1e-3)
    assert mg.output["iterations"] == mc.output["iterations"]
    tg, tc = mg.output["training_metrics"]["tot_withinss"], mc.output["training_metrics"]["tot_withinss"]
    assert abs(tg - tc) <= 1e-6 * tc
    # the recovered centers are the generating ones (clusters are well separated)
    for c in cg:
        assert float(((centers.numpy() + 1e4 - c) ** 2).sum(1).min()) < 0.05


def test_kmeans_user_points_offset_padded_matches_cpu():
    """standardize=False, F=6 (padded to 8 columns on the GPU), data offset by 1e4, init=User with
    points in original space: the device run starts from the user's points, as the CPU run does."""
    from llama_github_io_amd.models.kmeans import KMeansTrainer
    g = torch.Generator().manual_seed(8)
    N, F = 40000, 6
    centers = torch.randn(4, F, generator=g) * 4
    lab = torch.randint(0, 4, (N,), generator=g)
    X = (centers[lab] + 0.3 * torch.randn(N, F, generator=g)).T.contiguous() + 1e4
    info = _info(F)
    info.response = None
    prm = dict(k=4, max_iterations=1, init="User", user_points=(centers + 1e4).numpy(), seed=7, standardize=False)
    mg = KMeansTrainer(prm).fit(X.to(dev), None, None, None, info)
    mc = KMeansTrainer(prm).fit(X, None, None, None, info)
    cg = np.array(mg.output["centers"])
    np.testing.assert_allclose(cg, np.array(mc.output["centers"]), rtol=0, atol=1e-3)
    np.testing.assert_allclose(cg, (centers + 1e4).numpy(), atol=0.05)


@pytest.mark.parametrize("n,idt,vdt", [(10, torch.int64, torch.float64), (3000, torch.int32, torch.float32),
                                       (16384, torch.int64, torch.float32), (1, torch.int32, torch.float64)])
def test_segment_sum_kernel_matches_index_add(n, idt, vdt):
    """csrc/segment_kernels.hip (LDS-privatised fp64 segment sums) vs the fp64 index_add reference."""
    from llama_github_io_amd.ops.segment import segment_sum
    g = torch.Generator().manual_seed(n)
    N = 1_234_567
    idx = torch.randint(0, n, (N,), generator=g).to(idt)
    v = torch.randn(N, generator=g).to(vdt)
    got = segment_sum(idx.to(dev), v.to(dev), n).cpu()
    ref = torch.zeros(n, dtype=torch.float64).index_add_(0, idx.long(), v.double())
    assert got.dtype == torch.float64 and torch.allclose(got, ref, rtol=1e-12, atol=1e-9)


def _fused_case(n_in, hidden, K, act, drops, regression, B, seed=0, f32=False, in_drop=0.0, maxout=False, ae=False):
    """One fused MFMA step (csrc/dl_kernels.hip) and the fp32 autograd gradient of the same weighted loss
    (bf16 path: weights and inputs rounded to bf16 like the kernels' operands; f32: the fp32 master weights and
    inputs, v_mfma_f32_16x16x4_f32; dropout masks from ops.dense._mask_ref)."""
    from llama_github_io_amd.models.deeplearning import MLP
    from llama_github_io_amd.ops import dl as dlops
    from llama_github_io_amd.ops.dense import FlatParams, _act, _mask_ref, step_seed
    g = torch.Generator(device="cpu").manual_seed(seed)
    actn = {1: "rectifier", 2: "tanh"}[act]
    net = MLP(n_in, hidden, K, actn, maxout, 0.0, drops, "UniformAdaptive", 1.0, g).to(dev)
    fp = FlatParams(net)
    with torch.no_grad():
        fp.p.add_(0.05 * torch.randn(fp.p.shape, generator=g).to(dev))   # non-trivial biases
    N = 3 * B
    Z = torch.randn(N, n_in, generator=g).to(dev).to(torch.float32 if f32 else torch.bfloat16)
    w = (torch.rand(N, generator=g) + 0.5).to(dev)
    y = torch.randn(N, generator=g).to(dev) if regression else torch.randint(0, K, (N,), generator=g).to(dev)
    ridx = torch.randperm(N, generator=g)[:B].to(dev)
    shadow = None if f32 else fp.p[: fp.n_decay].to(torch.bfloat16)
    wsrc = fp.p[: fp.n_decay] if f32 else shadow
    step_t = torch.full((1,), 7, dtype=torch.int64, device=dev)
    bases = [1234567 + 31 * i for i in range(len(hidden))]
    in_seed = 99991
    fs = dlops.FusedMLPStep(fp, list(net.hidden) + [net.out], act, drops, bases, Z, w, None if ae else y, regression,
                            B, shadow, step_t, fp.g, None, in_drop, in_seed, maxout, ae)
    fs.refresh_transposed()
    fp.g.zero_()
    fs.step(ridx)
    torch.cuda.synchronize()
    got = fp.g.clone()
    # fp32 autograd reference on the bf16-rounded operands
    Ws = [wsrc[(l_.weight.data_ptr() - fp.p.data_ptr()) // 4:][: l_.weight.numel()].float().view_as(l_.weight)
          .clone().requires_grad_(True) for l_ in list(net.hidden) + [net.out]]
    Bs = [l_.bias.detach().clone().requires_grad_(True) for l_ in list(net.hidden) + [net.out]]
    h = Z[ridx].float()
    if in_drop > 0:                  # input dropout: the kernels' hash mask over (batch row, input)
        m = _mask_ref((B, n_in), in_drop, step_seed(in_seed, 7), dev)
        h = torch.where(m, h / (1 - in_drop), torch.zeros_like(h))
        if not f32:                  # the bf16 kernels round the scaled inputs to bf16
            h = h.to(torch.bfloat16).float()
    for i in range(len(hidden)):
        if maxout:                   # two channels: weight / bias rows [0, u) and [u, 2u)
            z = h @ Ws[i].T + Bs[i]
            h = torch.maximum(z[:, :hidden[i]], z[:, hidden[i]:])
        else:
            h = _act(act, h @ Ws[i].T + Bs[i])
        if drops[i] > 0:
            m = _mask_ref((B, hidden[i]), drops[i], step_seed(bases[i], 7), dev)
            h = torch.where(m, h / (1 - drops[i]), torch.zeros_like(h))
    o = h @ Ws[-1].T + Bs[-1]
    wb = w[ridx]
    if ae:                           # reconstruction of the (undropped) inputs, quadratic loss / n_out
        loss = (wb[:, None] * (o - Z[ridx].float()) ** 2).sum() / o.shape[1] / wb.sum()
    elif regression:
        loss = (wb * 0.5 * (o[:, 0] - y[ridx]) ** 2).sum() / wb.sum()
    else:
        loss = (wb * torch.nn.functional.cross_entropy(o, y[ridx], reduction="none")).sum() / wb.sum()
    loss.backward()
    ref = torch.zeros_like(got)
    for l_, Wg, Bg in zip(list(net.hidden) + [net.out], Ws, Bs):
        ow = (l_.weight.data_ptr() - fp.p.data_ptr()) // 4
        ob = (l_.bias.data_ptr() - fp.p.data_ptr()) // 4
        ref[ow: ow + Wg.numel()] = Wg.grad.reshape(-1)
        ref[ob: ob + Bg.numel()] = Bg.grad
    # transposed shadow = transposed bf16 weights
    for i, l_ in enumerate(list(net.hidden) + [net.out]):
        ow = (l_.weight.data_ptr() - fp.p.data_ptr()) // 4
        n_o, n_i = l_.weight.shape
        assert torch.equal(fs.WT[ow: ow + n_o * n_i].view(n_i, n_o), wsrc[ow: ow + n_o * n_i].view(n_o, n_i).T)
    return got, ref


@pytest.mark.parametrize("n_in,hidden,K,act,drops,regression,B", [
    (784, [200, 200], 2, 1, [0.0, 0.0], False, 512),          # the BASELINE MLP shape
    (37, [48, 24], 3, 2, [0.0, 0.0], False, 200),            # ragged widths: scalar loads, padding rows
    (50, [64], 5, 1, [0.3], False, 256),                      # dropout (hash mask shared with the fwd/bwd kernels)
    (20, [40, 16, 8], 1, 2, [0.1, 0.0, 0.2], True, 128),      # regression, 3 hidden layers
])
def test_dl_fused_step_matches_fp32_autograd(n_in, hidden, K, act, drops, regression, B):
    got, ref = _fused_case(n_in, hidden, K, act, drops, regression, B)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 3e-2, rel
    assert float(torch.nn.functional.cosine_similarity(got, ref, dim=0)) > 0.999


@pytest.mark.parametrize("n_in,hidden,K,act,drops,regression,B", [
    (784, [200, 200], 2, 1, [0.0, 0.0], False, 512),          # the BASELINE MLP shape, default fp32 compute
    (37, [48, 24], 3, 2, [0.0, 0.0], False, 200),            # ragged widths: scalar loads, padding rows
    (50, [64], 5, 1, [0.3], False, 256),
    (20, [40, 16, 8], 1, 2, [0.1, 0.0, 0.2], True, 128),
])
def test_dl_fused_fp32_step_matches_fp32_autograd(n_in, hidden, K, act, drops, regression, B):
    """fp32 operands (compute_dtype='float32', the H2O default) on v_mfma_f32_16x16x4_f32: exact fp32 products,
    so only the summation order separates the kernels from autograd."""
    got, ref = _fused_case(n_in, hidden, K, act, drops, regression, B, f32=True)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 1e-4, rel


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("n_in,hidden,K,in_drop", [
    (60, [64, 32], 40, 0.0),         # K > 16: logit tile over the waves, one wave per row for the softmax
    (90, [48], 200, 0.2),            # 200 classes with input dropout
    (784, [200, 200], 2, 0.1),       # input dropout on the BASELINE shape
])
def test_dl_fused_step_wide_softmax_and_input_dropout(n_in, hidden, K, in_drop, f32):
    got, ref = _fused_case(n_in, hidden, K, 1, [0.0] * len(hidden), False, 256, f32=f32, in_drop=in_drop)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < (1e-4 if f32 else 3e-2), rel


def test_dl_trainer_uses_fused_step_and_learns(monkeypatch):
    """The trainer's graph-chunked loop runs the fused MFMA step (no library GEMM in the loop) and reaches
    the accuracy of the library-GEMM explicit step on the same data."""
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.rand(100, 60000, device=dev, generator=g)
    y = (X[:10].sum(0) > 5).float()
    for cd in ("bf16", "float32"):
        res = {}
        for flag in ("1", "0"):
            monkeypatch.setenv("H2O_DL_FUSED", flag)
            m = DeepLearningTrainer(dict(hidden=[64, 64], epochs=2, compute_dtype=cd, mini_batch_size=1024, seed=3,
                                         stopping_rounds=0, score_interval=1e9, standardize=False)).fit(
                X, y, None, None, _info(100))
            res[flag] = m
        assert res["1"].output["training_step_fused_mfma"] and not res["0"].output["training_step_fused_mfma"]
        a1, a0 = res["1"].output["training_metrics"]["AUC"], res["0"].output["training_metrics"]["AUC"]
        assert a1 > 0.9 and abs(a1 - a0) < 0.02, (cd, a1, a0)


@pytest.mark.parametrize("obj,extra", [("bernoulli", dict(reg_lambda=2.0, reg_alpha=0.5, max_delta_step=0.3)),
                                       ("gaussian", dict(reg_lambda=1.0))])
def test_xgboost_fused_step_matches_torch_path(obj, extra):
    """The fused XGBoost row step (k_gbm_step D_XGB_LOGISTIC / D_GAUSSIAN + k_leaf_values with lambda / alpha /
    max_delta_step) grows the same trees as the torch gradient path."""
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.xgboost import XGBoostTrainer
    g = torch.Generator().manual_seed(3)
    N, F = 20000, 6
    X = torch.randn(F, N, generator=g)
    if obj == "bernoulli":
        y = (torch.rand(N, generator=g) < torch.sigmoid(X[0] - X[1] + 0.5 * X[2] * X[3])).float()
        info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    else:
        y = X[0] * 2 + torch.sin(X[1]) + 0.1 * torch.randn(N, generator=g)
        info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", None)
    params = dict(ntrees=8, max_depth=4, learn_rate=0.3, seed=1, **extra)

    class TorchPath(XGBoostTrainer):
        def _fused(self):
            return False
    fused_tr = XGBoostTrainer(dict(params))
    mf = fused_tr.fit(X.cuda(), y.cuda(), None, None, info)
    assert fused_tr._fused()
    mt = TorchPath(dict(params)).fit(X.cuda(), y.cuda(), None, None, info)
    pf = mf._predict_tensor(X.cuda()).double().cpu()
    pt = mt._predict_tensor(X.cuda()).double().cpu()
    assert torch.allclose(pf, pt, rtol=2e-4, atol=2e-5), (pf - pt).abs().max()


@pytest.mark.parametrize("hidden", [[16, 16], [7]])
def test_deeplearning_reproducible_is_bit_identical(hidden):
    """reproducible=True: two seeded runs give bit-identical models (the fused step's fixed-order
    reductions, or autograd where the library-GEMM step would accumulate bias gradients atomically)."""
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    g = torch.Generator(device=dev).manual_seed(4)
    N, F = 20000, 12
    X = torch.randn(F, N, device=dev, generator=g)
    y = (X[0] - X[1] + 0.3 * torch.randn(N, device=dev, generator=g) > 0).float()
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    preds = []
    for _ in range(2):
        m = DeepLearningTrainer(dict(hidden=hidden, epochs=2, seed=7, reproducible=True, mini_batch_size=64,
                                     score_interval=1e9)).fit(X, y, None, None, info)
        preds.append(m.score_tensor(X).cpu())
    assert torch.equal(preds[0], preds[1])


def test_dl_trainer_fused_multinomial_input_dropout(monkeypatch):
    """30 classes with input dropout train through the fused step (wide softmax, input mask) and match the
    autograd path's accuracy (H2O_DL_FUSED=0)."""
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    g = torch.Generator(device=dev).manual_seed(2)
    F, N, K = 40, 40000, 30
    X = torch.rand(F, N, device=dev, generator=g)
    y = torch.clamp((X[0] * K).long(), 0, K - 1).float()
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", [str(i) for i in range(K)])
    acc = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O_DL_FUSED", flag)
        m = DeepLearningTrainer(dict(hidden=[64], epochs=8, input_dropout_ratio=0.1, mini_batch_size=512, seed=5,
                                     stopping_rounds=0, score_interval=1e9)).fit(X, y, None, None, info)
        assert bool(m.output["training_step_fused_mfma"]) == (flag == "1")
        acc[flag] = 1 - m.output["training_metrics"]["mean_per_class_error"]
    assert acc["1"] > 0.15 and abs(acc["1"] - acc["0"]) < 0.08, acc     # chance: 1/30


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("n_in,hidden,K,drops", [
    (784, [200, 200], 2, [0.0, 0.0]),   # Maxout on the BASELINE shape
    (37, [48, 24], 3, [0.2, 0.0]),      # ragged widths (channel blocks not multiples of 16), hidden dropout
    (20, [40, 16, 8], 30, [0.0, 0.1, 0.0]),
])
def test_dl_fused_step_maxout_matches_fp32_autograd(n_in, hidden, K, drops, f32):
    """Maxout hidden layers (Neurons.Maxout, 2 channels): the winning channel takes the gradient."""
    got, ref = _fused_case(n_in, hidden, K, 1, drops, False, 256, f32=f32, maxout=True)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < (1e-4 if f32 else 3e-2), rel


def test_dl_trainer_maxout_runs_fused(monkeypatch):
    """activation='Maxout' trains through the fused step and matches the autograd path's AUC."""
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    g = torch.Generator(device=dev).manual_seed(4)
    X = torch.rand(50, 30000, device=dev, generator=g)
    y = (X[:8].sum(0) > 4).float()
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O_DL_FUSED", flag)
        m = DeepLearningTrainer(dict(hidden=[32, 32], activation="Maxout", epochs=3, mini_batch_size=512, seed=2,
                                     stopping_rounds=0, score_interval=1e9)).fit(X, y, None, None, _info(50))
        res[flag] = m
    assert res["1"].output["training_step_fused_mfma"] and not res["0"].output["training_step_fused_mfma"]
    a1, a0 = res["1"].output["training_metrics"]["AUC"], res["0"].output["training_metrics"]["AUC"]
    assert a1 > 0.85 and abs(a1 - a0) < 0.05, (a1, a0)


@pytest.mark.parametrize("f32", [True])
@pytest.mark.parametrize("n_in,hidden,in_drop", [(12, [8], 0.0), (60, [32, 16, 32], 0.1), (120, [48], 0.0)])
def test_dl_fused_autoencoder_matches_fp32_autograd(n_in, hidden, in_drop, f32):
    """Autoencoder outputs (K = n_in, narrow and wide output paths) reconstruct the undropped inputs."""
    got, ref = _fused_case(n_in, hidden, n_in, 2, [0.0] * len(hidden), True, 256, f32=f32, in_drop=in_drop, ae=True)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 1e-4, rel


def test_dl_trainer_autoencoder_runs_fused(monkeypatch):
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    g = torch.Generator(device=dev).manual_seed(6)
    Zl = torch.randn(4, 20000, device=dev, generator=g)
    M = torch.randn(36, 4, device=dev, generator=g)
    X = torch.cat([Zl, M @ Zl], 0)                       # 40 columns of rank 4
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O_DL_FUSED", flag)
        m = DeepLearningTrainer(dict(hidden=[16, 4, 16], autoencoder=True, activation="Tanh", epochs=4,
                                     mini_batch_size=256, seed=1, stopping_rounds=0, score_interval=1e9)).fit(
            X, None, None, None, _info(40, None))
        res[flag] = m
    assert res["1"].output["training_step_fused_mfma"] and not res["0"].output["training_step_fused_mfma"]
    e1, e0 = res["1"].output["training_metrics"]["MSE"], res["0"].output["training_metrics"]["MSE"]
    assert e1 < 0.5 and abs(e1 - e0) < 0.25 * max(e0, e1), (e1, e0)


def test_tree_graph_replay_per_class_plans(monkeypatch):
    """Per-tree graph replay on a 3-class multinomial GBM (the classes share one launch plan, so one captured graph
    serves every tree): the trees equal the direct-launch ones exactly."""
    from llama_github_io_amd.models.gbm import GBMTrainer
    g = torch.Generator(device=dev).manual_seed(9)
    N, F = 30000, 5
    X = torch.randn(F, N, device=dev, generator=g)
    y = (X[0] > 0.3).float() + (X[1] + X[2] > 0.5).float()
    params = dict(ntrees=6, max_depth=4, seed=4, distribution="multinomial")
    monkeypatch.setenv("H2O_TREE_GRAPH", "1")
    tr = GBMTrainer(dict(params))
    a = tr.fit(X, y, None, None, _info(F, ("0", "1", "2")))
    gb = getattr(tr.builder, "inner", tr.builder)
    assert 1 <= len(gb._graphs) <= 3 and not gb.__dict__.get("_graph_off")
    monkeypatch.setenv("H2O_TREE_GRAPH", "0")
    b = GBMTrainer(dict(params)).fit(X, y, None, None, _info(F, ("0", "1", "2")))
    assert torch.equal(a.score_tensor(X).cpu(), b.score_tensor(X).cpu())
