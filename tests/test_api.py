"""h2o-py compatible facade: frames, estimators, CV, grid, AutoML, persistence."""
import os

import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                            H2OIsolationForestEstimator, H2OKMeansEstimator, H2ORandomForestEstimator,
                            H2OXGBoostEstimator)


@pytest.fixture(scope="module")
def frames():
    h2o.init(verbose=False)
    rng = np.random.default_rng(0)
    n = 2000
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(["x", "y", "z"], n)})
    df["y"] = np.where(df.a + (df.c == "x") * 1.0 + rng.normal(size=n) * 0.5 > 0.3, "yes", "no")
    df["r"] = df.a * 2 + df.b + rng.normal(size=n) * 0.1
    fr = h2o.H2OFrame(df)
    tr, va = fr.split_frame([0.8], seed=1)
    return fr, tr, va


@pytest.mark.parametrize("E,kw", [(H2OGradientBoostingEstimator, dict(ntrees=10)), (H2ORandomForestEstimator, dict(ntrees=10)),
                                  (H2OXGBoostEstimator, dict(ntrees=10)), (H2OGeneralizedLinearEstimator, dict(family="binomial")),
                                  (H2ODeepLearningEstimator, dict(hidden=[10], epochs=2))])
def test_supervised_estimators_with_cv(frames, E, kw):
    fr, tr, va = frames
    m = E(seed=1, nfolds=3, keep_cross_validation_predictions=True, **kw)
    m.train(x=["a", "b", "c"], y="y", training_frame=tr, validation_frame=va)
    assert m.auc(valid=True) > 0.8
    assert abs(m.model_performance(va).auc() - m.auc(valid=True)) < 1e-9
    p = m.predict(va)
    assert p.names == ["predict", "no", "yes"] and p.nrows == va.nrows
    s = m.cross_validation_metrics_summary()
    assert "AUC" in s and len(s["AUC"]["values"]) == 3
    assert m.cross_validation_holdout_predictions().nrows == tr.nrows


def test_glm_regression_coefficients(frames):
    fr, tr, va = frames
    m = H2OGeneralizedLinearEstimator(lambda_=0)
    m.train(x=["a", "b"], y="r", training_frame=tr)
    c = m.coef()
    assert abs(c["a"] - 2) < 0.02 and abs(c["b"] - 1) < 0.02


def test_unsupervised(frames):
    fr, tr, va = frames
    k = H2OKMeansEstimator(k=3, seed=1)
    k.train(x=["a", "b"], training_frame=fr)
    assert len(k.centers()) == 3 and k.predict(fr).nrows == fr.nrows
    i = H2OIsolationForestEstimator(ntrees=20, seed=1)
    i.train(x=["a", "b"], training_frame=fr)
    assert i.predict(fr).names == ["predict", "mean_length"]


def test_grid_and_automl_and_persistence(frames, tmp_path):
    from h2o.automl import H2OAutoML
    from h2o.grid import H2OGridSearch
    fr, tr, va = frames
    g = H2OGridSearch(H2OGradientBoostingEstimator, dict(max_depth=[2, 4], ntrees=[5, 10]))
    g.train(x=["a", "b", "c"], y="y", training_frame=tr, validation_frame=va)
    t = g.get_grid(sort_by="auc").sorted_metric_table
    assert len(t) == 4 and t["auc"].is_monotonic_decreasing
    a = H2OAutoML(max_models=3, seed=1, nfolds=3, include_algos=["GLM", "GBM", "StackedEnsemble"])
    a.train(x=["a", "b", "c"], y="y", training_frame=tr)
    lb = a.leaderboard.as_data_frame()
    assert len(lb) >= 3 and lb["auc"].is_monotonic_decreasing
    path = h2o.save_model(a.leader._model, str(tmp_path), force=True)
    m2 = h2o.load_model(path)
    assert abs(m2.model_performance(va).auc() - a.leader.model_performance(va).auc()) < 1e-6


def test_frame_ops(frames, tmp_path):
    fr, tr, va = frames
    g = fr.group_by("c").count().mean("a").get_frame().as_data_frame()
    ref = fr.as_data_frame().groupby("c")["a"].agg(["count", "mean"])
    assert np.allclose(g["nrow"].values, ref["count"].values) and np.allclose(g["mean_a"].values, ref["mean"].values)
    p = str(tmp_path / "f.csv")
    h2o.export_file(fr, p)
    back = h2o.import_file(p)
    assert back.nrows == fr.nrows and back.types["c"] == "enum"
    assert np.allclose(back["a"].as_data_frame().values[:, 0], fr["a"].as_data_frame().values[:, 0])
    h2o.save_frame(fr, str(tmp_path / "bin"))
    b2 = h2o.load_frame("x", str(tmp_path / "bin"))
    assert b2.names == fr.names and b2.nrows == fr.nrows
    cf = h2o.create_frame(rows=100, cols=5, seed=1, has_response=True)
    assert cf.nrows == 100 and cf.ncols == 6
