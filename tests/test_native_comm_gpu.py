"""The row-sharded tree driver (``h2o_tree_dist``) on RCCL, rehearsed on one GPU.

RCCL refuses two ranks on one device, so a 1-GPU box runs the multi-GPU code path with a 1-RANK RCCL
communicator (``H2O_TREE_COMM_FORCE``): every kernel of the histogram exchange (k_hist_pack into the fp64 or fp32
wire format, all-reduce or feature-sliced reduce-scatter + rank-major candidate all-gather read in place, sibling
subtraction from the received slots, leaf-sum all-reduce) runs through ``ncclAllReduce`` / ``ncclReduceScatter`` /
``ncclAllGather`` on the compute stream. Multi-rank protocol correctness is pinned by the same native driver
under gloo at world 2/3 (``tests/test_distributed_gpu.py``). Oracle: :class:`RefTreeBuilder` (fp64 NumPy)."""
import os
import socket

import numpy as np
import pytest
import torch

from llama_github_io_amd.ops import tree as T
from llama_github_io_amd.ops.binning import apply_binning, fit_binning

pytestmark = pytest.mark.gpu

from test_tree_engine import _data  # noqa: E402


@pytest.fixture
def force_env(monkeypatch):
    def set_(mode, dtype="f32"):
        monkeypatch.setenv("H2O_TREE_COMM_FORCE", mode)
        monkeypatch.setenv("H2O_TREE_COMM_DTYPE", dtype)
    return set_


def test_rccl_one_rank_collectives(force_env):
    from llama_github_io_amd.parallel import rccl
    c = rccl.native_comm(force=True)
    assert c is not None and c.world == 1
    x = torch.arange(1000, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    c.collective(rccl.OP_ALLREDUCE, x, y, 1000, rccl.DT_F64)
    c.collective(rccl.OP_REDUCE_SCATTER, x.float(), y.float(), 1000, rccl.DT_F32)
    z = torch.empty(1000, dtype=torch.float32, device="cuda")
    c.collective(rccl.OP_ALLGATHER, x.float().contiguous(), z, 1000, rccl.DT_F32)
    torch.cuda.synchronize()
    assert torch.equal(y, x) and torch.equal(z, x.float())


def _leaf_paths(tl):
    """leaf id -> path string ('' root, 'L' / 'R' per level) of a TreeLevels, and node path -> (level, index)."""
    leaves, nodes = {}, {}

    def walk(d, i, path):
        nodes[path] = (d, i)
        dec = tl.decs[d][i]
        for side, arr in (("L", tl.child_l), ("R", tl.child_r)):
            c = int(arr[d][i])
            if c < 0:
                leaves[-1 - c] = path + ("" if dec["feat"] < 0 else side)
            else:
                walk(d + 1, c, path + side)
    walk(0, 0, "")
    return leaves, nodes


def _assert_same_tree_up_to_ties(tl_r, tl_g, lr, lg, rtol=1e-5, vectorized=False):
    """Tie-aware exact comparison of a tree grown from fp32-wire histograms with the fp64 reference tree:
    * wherever the two trees take different decisions, the two decisions have equal gain (a tie between equal-gain
      splits, which fp32 rounding of the exchanged sums may break differently), and
    * every row whose reference path does not pass through such a node reaches the leaf at the same path in both
      trees (identical routing below every non-tied node)."""
    leaves_r, nodes_r = _leaf_paths(tl_r)
    leaves_g, nodes_g = _leaf_paths(tl_g)
    tied = []
    for path, (d, i) in sorted(nodes_r.items(), key=lambda kv: len(kv[0])):
        if any(path.startswith(t) for t in tied):
            continue
        assert path in nodes_g, f"node {path!r} missing above any tie"
        dr, dg = tl_r.decs[d][i], tl_g.decs[nodes_g[path][0]][nodes_g[path][1]]
        if dr["feat"] == dg["feat"] and dr["bin"] == dg["bin"] and dr["na_left"] == dg["na_left"]:
            continue
        g = max(abs(float(dr["gain"])), abs(float(dg["gain"])), 1e-300)
        assert abs(float(dr["gain"]) - float(dg["gain"])) <= rtol * g, (path, dr["feat"], dg["feat"], dr["gain"],
                                                                         dg["gain"])
        tied.append(path)
    if vectorized:          # per-leaf codes instead of per-row path strings (100M-row trees)
        paths = sorted(set(leaves_r.values()) | set(leaves_g.values()))
        code = {q: i for i, q in enumerate(paths)}
        cr = np.array([code[leaves_r[k]] for k in range(len(leaves_r))], dtype=np.int64)
        cg = np.array([code[leaves_g[k]] for k in range(len(leaves_g))], dtype=np.int64)
        fr = np.array([not any(leaves_r[k].startswith(t) for t in tied) for k in range(len(leaves_r))])
        lr, lg = np.asarray(lr, dtype=np.int64), np.asarray(lg, dtype=np.int64)
        free = fr[lr]
        assert free.mean() > 0.5, "ties under the root"
        assert (cr[lr][free] == cg[lg][free]).all(), int((cr[lr][free] != cg[lg][free]).sum())
        return
    pr = np.array([leaves_r[int(k)] for k in lr], dtype=object)
    pg = np.array([leaves_g[int(k)] for k in lg], dtype=object)
    free = np.array([not any(p.startswith(t) for t in tied) for p in pr])
    assert free.mean() > 0.5, "ties under the root"      # the check must cover most rows to mean anything
    assert (pr[free] == pg[free]).all(), int((pr[free] != pg[free]).sum())


def _ref_and_gpu(depth, mode, dtype, force_env, seed=5, cat=True, N=20000):
    X, y, info = _data(N=N, cat=cat, seed=seed)
    b = fit_binning(X, info.iscat, info.nlevels, max_bins=64)
    bins = apply_binning(b, X)
    aux = torch.stack([torch.ones_like(y), y - y.mean(), y - y.mean(), torch.ones_like(y)], 1).contiguous()
    p = T.SplitParams(min_w=10)
    ref = T.RefTreeBuilder(bins, X.shape[0], b.nbins, b.iscat, None, depth, p)
    ref.build(aux, leaf_fn=lambda ls: (ls[:, 0] / ls[:, 1]).float())
    tl_r = ref.pop_levels()[0]
    force_env(mode, dtype)
    dev = torch.device("cuda", 0)
    gb = T.GpuTreeBuilder(bins.to(dev), X.shape[0], b.nbins, b.iscat, None, depth, p)
    return ref, tl_r, gb, aux.to(dev)


@pytest.mark.parametrize("depth,mode,dtype", [(6, "ar", "f64"), (5, "rs", "f64"), (7, "rs", "f64"), (6, "ar", "f32"),
                                              (6, "rs", "f32")])
def test_row_sharded_tree_on_rccl_matches_reference(depth, mode, dtype, force_env):
    """f64 wire: the decisions of the fp64 reference exactly. f32 wire (half the bytes): the same tree up to ties
    between equal-gain splits of one node (same rows either way), which fp32 rounding may break differently."""
    from llama_github_io_amd.parallel import rccl
    ref, tl_r, gb, aux = _ref_and_gpu(depth, mode, dtype, force_env)
    assert gb.dist_mode and isinstance(gb.transport, rccl.NativeComm)
    assert gb.sliced == (mode == "rs") and gb.cf32 == int(dtype == "f32")
    for _ in range(2):   # the second tree reuses every buffer (and the communicator)
        gb.build(aux, leaf_fn=lambda ls: (ls[:, 0] / ls[:, 1]).float())
        tl_g = gb.pop_levels()[0]
        assert tl_g.root_weight == pytest.approx(tl_r.root_weight)
        if dtype == "f32":
            _assert_same_tree_up_to_ties(tl_r, tl_g, ref.leaf_of_row.numpy(), gb.leaf_of_row.cpu().numpy())
            continue
        assert tl_g.n_leaves == tl_r.n_leaves
        for dr, dg in zip(tl_r.decs, tl_g.decs):
            assert np.array_equal(dr["feat"], dg["feat"])
            assert np.array_equal(dr["bin"], dg["bin"])
            np.testing.assert_allclose(dr["wl"], dg["wl"], rtol=1e-5)
        np.testing.assert_allclose(tl_r.leaf_values, tl_g.leaf_values, rtol=1e-4, atol=1e-6)
        assert torch.equal(ref.leaf_of_row, gb.leaf_of_row.cpu())


@pytest.mark.parametrize("mode", ["ar", "rs"])
def test_narrow_planar_tree_on_rccl_matches_reference(mode, force_env):
    """H2O's default histogram on wide bins (1016 edges per feature, planar rows): the narrow levels (column
    limits, low-entry reduce, one-plane routes, root-direction bytes, level-2 leaf-walk start) through the
    row-sharded driver on a 1-rank RCCL communicator, decision for decision against RefTreeBuilder."""
    from test_tree_engine import _edge_tab, _vr
    X, y, info = _data(N=30000, F=10, cat=True, seed=11)
    X = X.clone()
    X[1] = torch.exp(3 * X[1])              # heavy tail: the reference's node ranges (parent-observed, narrowed)
    b = fit_binning(X, info.iscat, info.nlevels, max_bins=1016)
    assert b.stride >= 64 and b.n_low == X.shape[0]
    bins = apply_binning(b, X)
    g = y - 0.5
    aux = torch.stack([torch.ones_like(y), g, g, torch.ones_like(y)], 1).contiguous()
    p = T.SplitParams(min_w=10, adapt_nbins=20, adapt_top=1024, edges=_edge_tab(b), vrange=_vr(b, X))
    ref = T.RefTreeBuilder(bins, b.F, b.nbins, b.iscat, None, 5, p)
    ref.set_feature_groups(b.vmap, b.n_low, b.n_mid)
    ref.build(aux, leaf_fn=lambda ls: (ls[:, 0] / ls[:, 1]).float())
    tl_r = ref.pop_levels()[0]
    force_env(mode, "f64")
    dev = torch.device("cuda", 0)
    gb = T.GpuTreeBuilder(apply_binning(b, X.to(dev), planar=True), b.F, b.nbins, b.iscat, None, 5, p)
    gb.set_feature_groups(b.vmap, b.n_low, b.n_mid)
    assert gb.dist_mode and gb.planar
    gb.build(aux.to(dev), leaf_fn=lambda ls: (ls[:, 0] / ls[:, 1]).float())
    tl_g = gb.pop_levels()[0]
    assert tl_g.n_leaves == tl_r.n_leaves
    for dr, dg in zip(tl_r.decs, tl_g.decs):
        assert np.array_equal(dr["feat"], dg["feat"]) and np.array_equal(dr["bin"], dg["bin"])
        np.testing.assert_allclose(dr["wl"], dg["wl"], rtol=1e-6)
    assert torch.equal(ref.leaf_of_row, gb.leaf_of_row.cpu())


def test_gbm_on_rccl_equals_single_process(force_env, monkeypatch):
    """A whole GBM (gradients, leaf values on device, prediction update) through the 1-rank RCCL driver."""
    from llama_github_io_amd.models.gbm import GBMTrainer
    X, y, info = _data(N=30000, cat=True, seed=9)
    dev = torch.device("cuda", 0)
    X, y = X.to(dev), y.to(dev)
    params = dict(ntrees=6, max_depth=5, seed=3)
    single = GBMTrainer(params).fit(X, y, None, None, info).forest.predict_raw(X)
    force_env("ar", "f64")
    tr = GBMTrainer(params)
    m = tr.fit(X, y, None, None, info)
    sharded = m.forest.predict_raw(X)
    assert torch.allclose(single, sharded, atol=1e-4, rtol=1e-4)


def test_tree_on_one_rank_nccl_process_group(force_env):
    """The communicator is created over a real (1-rank) ``nccl`` process group: the unique-id broadcast path."""
    import torch.distributed as dist
    from llama_github_io_amd.parallel import rccl
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        rccl.reset()
        ref, tl_r, gb, aux = _ref_and_gpu(6, "rs", "f64", force_env, seed=11)
        assert isinstance(gb.transport, rccl.NativeComm)
        gb.build(aux, leaf_fn=lambda ls: (ls[:, 0] / ls[:, 1]).float())
        tl_g = gb.pop_levels()[0]
        for dr, dg in zip(tl_r.decs, tl_g.decs):
            assert np.array_equal(dr["feat"], dg["feat"]) and np.array_equal(dr["bin"], dg["bin"])
        assert torch.equal(ref.leaf_of_row, gb.leaf_of_row.cpu())
    finally:
        rccl.reset()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_partial_f32_default_at_100m_rows(monkeypatch):
    """fp32 per-block partial histograms are the default for every N >= 1M (H2O_PARTIAL_F32): at 100M rows (the
    XGBoost BASELINE shape's row count) the tree equals the fp64-partials tree up to equal-gain ties, and rows are
    routed identically below every non-tied node."""
    N, F = 100_000_000, 8
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    bins = torch.randint(0, 250, (N, 32), generator=g, device=dev, dtype=torch.uint8)
    bins[:, F:] = 0
    y = ((bins[:, 0].float() - 125) / 70 - (bins[:, 1] > 130).float() + 0.5 * torch.sin(bins[:, 2].float() / 20) +
         torch.randn(N, generator=g, device=dev) > 0).float()
    aux = torch.stack([torch.ones_like(y), y - 0.5, y - 0.5, torch.full_like(y, 0.25)], 0).contiguous()
    p = T.SplitParams(min_w=10)
    nb = np.full(F, 250, np.int32)
    ic = np.zeros(F, np.int32)
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("H2O_PARTIAL_F32", flag)
        gb = T.GpuTreeBuilder(bins, F, nb, ic, None, 6, p)
        assert gb.pf32 == int(flag)
        gb.build(aux, soa=True, packed=True, unit=True, leaf_fn=lambda ls: (ls[:, 0] / ls[:, 1]).float())
        out.append((gb.pop_levels()[0], gb.leaf_of_row.cpu().numpy().copy()))
        del gb
        torch.cuda.empty_cache()
    (tl64, l64), (tl32, l32) = out
    _assert_same_tree_up_to_ties(tl64, tl32, l64, l32, vectorized=True)


def test_wide_categorical_group_on_rccl_matches_reference(force_env):
    """A 1000-level categorical group split through the row-sharded driver on a 1-rank RCCL communicator: the leader
    column's block derives the group's histograms from the exchanged build slots (Derive) and decides exactly as
    RefTreeBuilder's single sort over all levels."""
    from test_tree_engine import _wide_cat_data
    X, y, info = _wide_cat_data()
    b = fit_binning(X, info.iscat, info.nlevels, max_cat_bins=1024)
    bins = apply_binning(b, X)
    g = y - 0.5
    aux = torch.stack([torch.ones_like(y), g, g, torch.ones_like(y)], 1).contiguous()
    p = T.SplitParams(min_w=10)
    ref = T.RefTreeBuilder(bins, b.F, b.nbins, b.iscat, None, 5, p)
    ref.set_feature_groups(b.vmap)
    ref.set_cat_groups(b.gcat())
    ref.build(aux, leaf_fn=lambda ls: (ls[:, 0] / ls[:, 1]).float())
    tl_r = ref.pop_levels()[0]
    force_env("ar", "f64")
    dev = torch.device("cuda", 0)
    gb = T.GpuTreeBuilder(apply_binning(b, X.to(dev)), b.F, b.nbins, b.iscat, None, 5, p)
    gb.set_feature_groups(b.vmap)
    gb.set_cat_groups(b.gcat())
    assert gb.dist_mode
    gb.build(aux.to(dev), leaf_fn=lambda ls: (ls[:, 0] / ls[:, 1]).float())
    tl_g = gb.pop_levels()[0]
    assert tl_g.n_leaves == tl_r.n_leaves
    assert sum(int(c) == T.GROUP_CAT for d in tl_r.decs for c in d["is_cat"]) >= 2
    for dr, dg in zip(tl_r.decs, tl_g.decs):
        assert np.array_equal(dr["feat"], dg["feat"]) and np.array_equal(dr["bin"], dg["bin"])
        assert np.array_equal(dr["bits"], dg["bits"])
        np.testing.assert_allclose(dr["wl"], dg["wl"], rtol=1e-6)
    assert torch.equal(ref.leaf_of_row, gb.leaf_of_row.cpu())
