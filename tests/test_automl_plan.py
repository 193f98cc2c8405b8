"""AutoML modeling plan (reference ai/h2o/automl/ModelingPlans.java TEN_LAYERED, modeling/*StepsProvider)
and the CV early-stopping semantics AutoML relies on (ModelBuilder.cv_computeAndSetOptimalParameters)."""
import math

import numpy as np
import pytest


def test_plan_groups_and_order():
    from llama_github_io_amd.automl import GRID_W, MODEL_W, _plan
    plan = _plan()
    groups = [g for _, _, g, _ in plan]
    assert groups == sorted(groups)
    g1 = [(a, s) for a, s, g, _ in plan if g == 1]
    assert g1 == [("xgboost", "def_2"), ("glm", "def_1"), ("gbm", "def_5"), ("stackedensemble", "best_of_family_1")]
    w = {(a, s): wt for a, s, _, wt in plan}
    assert w[("xgboost", "grid_1")] == 3 * GRID_W and w[("gbm", "grid_1")] == 2 * GRID_W
    assert w[("completion", "resume_best_grids")] == 2 * GRID_W and w[("gbm", "lr_annealing")] == MODEL_W
    assert ("deeplearning", "grid_3") in w and ("stackedensemble", "all_xglm") in w


def test_grid_spaces_and_tolerance():
    from llama_github_io_amd.automl import _grid_space, default_stopping_tolerance
    dl3 = _grid_space("deeplearning", "grid_3")
    assert [20, 20, 20] in dl3["hidden"] and all(len(r) == 3 for r in dl3["hidden_dropout_ratios"])
    assert _grid_space("gbm", "grid_1")["max_depth"] == list(range(3, 18))
    assert default_stopping_tolerance(100) == pytest.approx(0.05)
    assert default_stopping_tolerance(10_000_000) == pytest.approx(0.001)
    assert default_stopping_tolerance(10_000) == pytest.approx(0.01)


def test_cv_early_stopping_sets_main_model_length():
    import h2o
    from h2o.estimators import H2OGradientBoostingEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(1)
    n = 500
    a, b = rng.normal(size=n), rng.normal(size=n)
    y = np.where(a + b + rng.normal(size=n) > 0, "p", "q")
    fr = h2o.H2OFrame({"a": a.tolist(), "b": b.tolist(), "y": y.tolist()})
    fr["y"] = fr["y"].asfactor()
    m = H2OGradientBoostingEstimator(ntrees=2000, max_depth=6, nfolds=3, stopping_rounds=2, stopping_tolerance=0.01,
                                     score_tree_interval=5, seed=3)
    m.train(x=["a", "b"], y="y", training_frame=fr)
    cv_lens = [getattr(h2o.get_model(k), "_model", h2o.get_model(k)).output["ntrees"]
               for k in m._model.output["cross_validation_models"]]
    assert max(cv_lens) < 2000                                  # fold models stopped on their holdout
    assert m._model.output["ntrees"] == int(round(np.mean(cv_lens)))
