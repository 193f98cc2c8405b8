"""The reference's default histogram (AUTO = UniformAdaptive: per-node uniform re-binning, DTree.java:337-411,
DHistogram.java:226-297) as a NumPy oracle (ops/dhist_oracle.py), and the engine's AUTO lattice pinned to it on data
where the lattice can represent the reference's cut points (uniform / integer features): the first tree (same
residuals) must split on the same features with thresholds within a few thousandths of a standard deviation.
profiles/r5_default_histogram_report.md quantifies the divergence on heavy-tailed data."""
import math

import numpy as np
import pandas as pd
import pytest

from llama_github_io_amd.ops import dhist_oracle as O


def test_oracle_histogram_semantics():
    # find_maxEx: float max + ulp, integer max + 1 (DHistogram.java:454-459)
    assert O.find_max_ex(3.0, True) == 4.0
    assert O.find_max_ex(3.0, False) == 3.0 + math.ulp(3.0)
    # integer column whose range fits the bin count: unit bins (DHistogram.java:226-233)
    h = O.Hist.make(1024, 0.0, 8.0, True)
    assert h.nbins == 8 and h.step == 1.0
    h = O.Hist.make(20, 0.0, 1.0, False)
    assert h.nbins == 20 and h.bin_at(5) == pytest.approx(0.25)
    x = np.array([0.0, 0.049, 0.05, 0.999])
    assert h.bins_of(x).tolist() == [0, 0, 1, 19]
    # children: max(parent >> 1, nbins) bins over the PARENT's observed range, split column narrowed at splat
    rng = np.random.default_rng(0)
    X = rng.uniform(0, 1, size=(4000, 2))
    y = (X[:, 0] > 0.6).astype(float)
    f0, trees, splits = O.train_gbm(X, y, ntrees=1, max_depth=2)
    root = trees[0]
    assert root.feat == 0 and abs(root.splat - 0.6) < 1e-3
    lh = root.left.hists[0]
    assert lh.nbins == 512 and lh.max_ex == pytest.approx(root.splat) and lh.lo == pytest.approx(X[:, 0].min())


@pytest.mark.parametrize("kind", ["uniform", "integer"])
def test_engine_auto_tree0_matches_reference_algorithm(kind):
    import h2o
    from llama_github_io_amd.models import builder
    h2o.init(verbose=False)
    rng = np.random.default_rng(3)
    n = 50000
    if kind == "uniform":
        X = rng.uniform(-3, 3, size=(n, 6))
    else:
        X = np.column_stack([rng.poisson(3, n), rng.integers(0, 8, n), rng.poisson(15, n),
                             rng.uniform(-1, 1, n), rng.normal(size=n), rng.integers(0, 3, n)]).astype(float)
    # step effects: sharp optima, so both methods' argmax sits at the same cut up to the bin width (a smooth effect
    # has a flat SE optimum whose argmax moves with noise)
    lg = 2.5 * (X[:, 0] > 0.7) - 2.0 * (X[:, 1] < 1.5) * (X[:, 0] <= 0.7) + 1.5 * (X[:, 2] > 1.2) * (X[:, 0] > 0.7) \
        - 1.2 * (X[:, 3] > 0.4) * (X[:, 1] >= 1.5)
    y = (rng.random(n) < 1 / (1 + np.exp(-(lg - lg.mean())))).astype(float)
    _, trees, _ = O.train_gbm(X, y, ntrees=1, max_depth=4)
    cols = [f"x{i}" for i in range(X.shape[1])]
    df = pd.DataFrame(X, columns=cols)
    df["y"] = np.where(y > 0.5, "1", "0")
    fr = h2o.H2OFrame(df, column_types={"y": "enum"})
    m = builder.train("gbm", dict(ntrees=1, max_depth=4, min_rows=10, seed=1), x=cols, y="y", training_frame=fr)
    t = m.forest.trees[0]
    sd = X.std(0)

    def walk_ref(nd, path, out):
        if nd.left is not None:
            out[path] = (nd.feat, nd.splat)
            walk_ref(nd.left, path + "L", out)
            walk_ref(nd.right, path + "R", out)
        return out

    def walk_eng(i, path, out):
        if t.feat[i] >= 0:
            out[path] = (int(t.feat[i]), float(t.thr[i]))
            walk_eng(int(t.left[i]), path + "L", out)
            walk_eng(int(t.right[i]), path + "R", out)
        return out
    ref, eng = walk_ref(trees[0], "", {}), walk_eng(0, "", {})
    for path, (f, thr) in ref.items():
        if len(path) > 1:          # (deeper nodes of this target hold no signal: noise splits)
            continue
        assert path in eng and eng[path][0] == f, (path, ref[path], eng.get(path))
        assert abs(eng[path][1] - thr) / sd[f] < 0.01, (path, thr, eng[path][1])
