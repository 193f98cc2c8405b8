"""H2OGridSearch surface of h2o-py/h2o/grid/grid_search.py: model ids / hyper names, per-model accessors
({model_id: value}), async start / join, sorted views and the Pareto front."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGradientBoostingEstimator, H2OGeneralizedLinearEstimator
from h2o.grid import H2OGridSearch


@pytest.fixture(scope="module")
def fr():
    h2o.init(verbose=False)
    rng = np.random.default_rng(3)
    d = pd.DataFrame({"a": rng.normal(size=600), "b": rng.normal(size=600)})
    d["y"] = np.where(d.a - 0.5 * d.b + rng.normal(size=600) * 0.5 > 0, "1", "0")
    return h2o.H2OFrame(d, column_types={"y": "enum"})


def test_grid_accessors(fr):
    g = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=5, seed=1), hyper_params={"max_depth": [2, 3, 4]})
    g.train(x=["a", "b"], y="y", training_frame=fr)
    assert g.key == g.grid_id and len(g.model_ids) == 3 and g.hyper_names == ["max_depth"]
    auc = g.auc()
    assert set(auc) == set(g.model_ids) and all(0.5 < v <= 1 for v in auc.values())
    assert set(g.logloss()) == set(g.model_ids) and set(g.rmse(train=True)) == set(g.model_ids)
    preds = g.predict(fr)
    assert all(p.nrows == fr.nrows for p in preds.values())
    perf = g.model_performance(fr)
    assert all(abs(perf[k].auc() - auc[k]) < 1e-9 for k in auc)
    assert set(g.varimp()) == set(g.model_ids)
    assert [m.model_id for m in g] == g.model_ids
    srt = g.get_grid(sort_by="auc", decreasing=True)
    assert srt.model_ids[0] == max(auc, key=auc.get)
    pf = g.pareto_front(x_metric="logloss", y_metric="AUC")
    assert len(pf.data) >= 1 and set(pf.data.model_id) <= set(g.model_ids)
    assert g.failed_params == [] and g.failed_raw_params == [] and g.failure_details == []


def test_grid_start_join_and_glm_accessors(fr):
    g = H2OGridSearch(H2OGeneralizedLinearEstimator(family="binomial"), hyper_params={"alpha": [0.0, 0.5]})
    g.start(x=["a", "b"], y="y", training_frame=fr)
    g.join()
    assert len(g) == 2
    co = g.coef()
    assert all(set(v) >= {"Intercept", "a", "b"} for v in co.values())
    assert set(g.null_deviance()) == set(g.model_ids) and set(g.aic()) == set(g.model_ids)


def test_grid_build_model(fr):
    g = H2OGridSearch(H2OGradientBoostingEstimator(seed=1), hyper_params={"max_depth": [2, 3]})
    g.build_model(dict(x=["a", "b"], y="y", training_frame=fr, ntrees=4))
    assert len(g) == 2 and all(m._m().params["ntrees"] == 4 for m in g)
    with pytest.raises(ValueError):
        g.build_model(dict(x=["a"], y="y", training_frame=None))


def test_automl_api_surface(fr, tmp_path):
    """h2o-py automl _base.py / _estimator.py / autoh2o.py surface: key, training_info, modeling_steps (re-injectable
    as modeling_plan), get_leaderboard extra columns, leader MOJO download, Pareto front."""
    from h2o.automl import H2OAutoML, get_leaderboard
    a = H2OAutoML(max_models=3, seed=1, exclude_algos=["DeepLearning", "StackedEnsemble"], nfolds=2)
    a.train(x=["a", "b"], y="y", training_frame=fr)
    assert a.key == a.project_name
    ti = a.training_info
    assert int(ti["stop_epoch"]) >= int(ti["start_epoch"])
    steps = a.modeling_steps
    assert steps and all(set(s) == {"name", "steps"} and s["steps"] for s in steps)
    lb = get_leaderboard(a, "ALL").as_data_frame()
    assert {"training_time_ms", "predict_time_per_row_ms", "algo"} <= set(lb.columns) and len(lb) == 3
    assert (lb["training_time_ms"] >= 0).all() and (lb["predict_time_per_row_ms"] > 0).all()
    assert list(a.get_leaderboard(["algo"]).as_data_frame().columns)[-1] == "algo"
    with pytest.raises(ValueError):
        get_leaderboard(a, "bogus")
    p = a.download_mojo(str(tmp_path))
    assert p.endswith(".zip")
    pf = a.pareto_front()
    assert len(pf.data) >= 1
    a2 = H2OAutoML(max_models=3, seed=1, nfolds=2, modeling_plan=steps)
    a2.train(x=["a", "b"], y="y", training_frame=fr)
    assert a2.modeling_steps == steps
