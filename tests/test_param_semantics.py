"""Parameters that used to be accepted as "hints" and now change the model or raise:
DeepLearning classification_stop / regression_stop / train_samples_per_iteration, XGBoost tree_method,
r2_stopping (deprecated in the reference: warns)."""
import warnings

import numpy as np
import pytest
import torch

from llama_github_io_amd.models import builder
from llama_github_io_amd.models.base import DataInfo
from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
from llama_github_io_amd.models.xgboost import XGBoostTrainer


def _sep(N=1200, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(3, N, generator=g)
    X[0] += torch.sign(X[0]) * 1.0             # a wide margin on x0: separable
    y = (X[0] > 0).float()
    info = DataInfo(["a", "b", "c"], np.zeros(3, np.int32), [None] * 3, "y", ["0", "1"])
    return X, y, info


def _dl(**kw):
    p = dict(hidden=[16], epochs=40, seed=1, mini_batch_size=32, score_interval=0.0, stopping_rounds=0,
             train_samples_per_iteration=0)
    p.update(kw)
    return DeepLearningTrainer(p)


def test_classification_stop_ends_training_on_training_accuracy():
    X, y, info = _sep()
    stopped = _dl().fit(X, y, None, None, info)                       # default 0: stop once error == 0
    full = _dl(classification_stop=-1).fit(X, y, None, None, info)    # -1 disables
    assert stopped.output["epochs"] < full.output["epochs"] == pytest.approx(40, rel=0.05)
    assert "stopped_early" in stopped.output


def test_regression_stop():
    g = torch.Generator().manual_seed(2)
    X = torch.randn(2, 800, generator=g)
    y = 0.5 * X[0]
    info = DataInfo(["a", "b"], np.zeros(2, np.int32), [None] * 2, "y", None)
    loose = _dl(regression_stop=0.05, epochs=30).fit(X, y, None, None, info)
    off = _dl(regression_stop=-1, epochs=30).fit(X, y, None, None, info)
    assert loose.output["epochs"] < off.output["epochs"]


def test_train_samples_per_iteration_sets_scoring_rounds():
    X, y, info = _sep()
    m1 = _dl(train_samples_per_iteration=0, epochs=4, classification_stop=-1).fit(X, y, None, None, info)
    m2 = _dl(train_samples_per_iteration=600, epochs=4, classification_stop=-1).fit(X, y, None, None, info)
    # score_interval 0: every iteration end is scored -> one per epoch vs two per epoch
    assert len(m1.output["scoring_history"]) == 4
    assert len(m2.output["scoring_history"]) == 8
    assert m2.output["actual_train_samples_per_iteration"] == 600
    with pytest.raises(ValueError):
        _dl(train_samples_per_iteration=-5).fit(X, y, None, None, info)


def test_xgboost_tree_method():
    g = torch.Generator().manual_seed(4)
    N = 3000
    Xc = torch.randint(0, 40, (2, N), generator=g).float()          # 40 distinct values: exact is expressible
    y = ((Xc[0] + Xc[1]) > 40).float()
    info = DataInfo(["a", "b"], np.zeros(2, np.int32), [None] * 2, "y", ["0", "1"])
    m = XGBoostTrainer(dict(ntrees=3, max_depth=3, tree_method="exact", seed=1)).fit(Xc, y, None, None, info)
    assert m.output["training_metrics"]["AUC"] > 0.9
    Xr = torch.randn(2, N, generator=g)                               # continuous: > 254 distinct values
    with pytest.raises(ValueError, match="exact"):
        XGBoostTrainer(dict(ntrees=2, tree_method="exact")).fit(Xr, y, None, None, info)
    with pytest.raises(ValueError):
        XGBoostTrainer(dict(ntrees=2, tree_method="gpu_magic")).fit(Xr, y, None, None, info)
    for tm in ("hist", "approx", "auto"):
        XGBoostTrainer(dict(ntrees=2, max_depth=2, tree_method=tm)).fit(Xr, y, None, None, info)


def test_r2_stopping_warns_like_the_reference():
    from llama_github_io_amd.models.params import validate
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        validate("gbm", dict(r2_stopping=0.5))
    assert any("no longer supported" in str(x.message) for x in w)
