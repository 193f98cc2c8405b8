"""h2o.explanation (h2o-py/h2o/explanation/_explain.py): tables behind every plot, and the figures."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator, H2ORandomForestEstimator


@pytest.fixture(scope="module")
def setup():
    h2o.init(verbose=False)
    rng = np.random.default_rng(0)
    n = 800
    d = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(list("xyz"), n)})
    d["y"] = d.a * 2 - d.b + (d.c == "x") + rng.normal(size=n) * 0.2
    d["g"] = np.where(rng.random(n) < 0.5, "m", "f")
    d["yb"] = np.where(d.y > 0, "1", "0")
    fr = h2o.H2OFrame(d, column_types={"c": "enum", "g": "enum", "yb": "enum"})
    gbm = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1)
    gbm.train(x=["a", "b", "c"], y="y", training_frame=fr)
    drf = H2ORandomForestEstimator(ntrees=10, max_depth=5, seed=1)
    drf.train(x=["a", "b", "c"], y="y", training_frame=fr)
    glm = H2OGeneralizedLinearEstimator()
    glm.train(x=["a", "b", "c"], y="y", training_frame=fr)
    return fr, [gbm, drf, glm]


def test_single_model_explain(setup):
    fr, (gbm, _, _) = setup
    ex = h2o.explain(gbm, fr)
    assert {"residual_analysis", "varimp", "shap_summary", "pdp", "ice"} <= set(ex)
    ss = ex["shap_summary"].data
    assert set(ss.feature) <= {"a", "b", "c"} and len(ss) == 3 * fr.nrows
    assert ex["pdp"]["a"].data.mean_response.is_monotonic_increasing
    assert ex["residual_analysis"].data.residual.abs().mean() < 1.0
    assert ex["shap_summary"].figure() is not None


def test_multi_model_explain_and_tables(setup):
    fr, models = setup
    vt = h2o.varimp(models)
    assert list(vt.index)[0] == "a" and vt.shape[1] == 3
    mc = h2o.model_correlation(models, fr)
    assert mc.shape == (3, 3) and np.allclose(np.diag(mc), 1.0) and (mc.to_numpy() > 0.8).all()
    ex = h2o.explain(models, fr)
    assert {"leaderboard", "varimp_heatmap", "model_correlation_heatmap", "pdp"} <= set(ex)
    assert ex["varimp_heatmap"].figure() is not None
    row = h2o.explain_row(models[0], fr, row_index=3)
    c = row["shap_explain_row"].data
    assert len(c) == 3
    # contributions + bias sum to the prediction (TreeSHAP local accuracy)
    pred = float(models[0].predict(fr).as_data_frame().iloc[3, 0])
    assert abs(c.contribution.sum() + row["shap_explain_row"].meta["bias"] - pred) < 1e-4
    lc = models[0].learning_curve_plot()
    assert lc.data is not None
    pf = h2o.pareto_front(pd.DataFrame({"model_id": ["m1", "m2", "m3"], "auc": [0.8, 0.9, 0.85],
                                         "predict_time_per_row_ms": [1.0, 3.0, 5.0]}), optimum="top left")
    assert list(pf.data.model_id) == ["m1", "m2"]
