"""H2OAutoML options (reference ``ai/h2o/automl/AutoMLBuildSpec.java:181-194``, ``AutoML.java`` work
allocation, ``preprocessing/TargetEncoding.java``, ``hex/ensemble/StackedEnsemble.java`` blending driver):
each option either changes what AutoML builds or is refused — none is silently dropped."""
import os

import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.automl import H2OAutoML
from llama_github_io_amd import automl as A


@pytest.fixture(scope="module")
def fr():
    h2o.init(verbose=False)
    rng = np.random.default_rng(3)
    n = 900
    lev = np.array([f"L{i:02d}" for i in range(30)])
    cat = rng.choice(lev, n)
    eff = {l_: rng.normal() for l_ in lev}
    a = rng.normal(size=n)
    b = rng.normal(size=n)
    logit = 1.2 * a + np.array([eff[c] for c in cat]) * 1.5 - 0.3
    y = np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "yes", "no")
    return h2o.H2OFrame(pd.DataFrame({"a": a, "b": b, "hc": cat, "y": y}))


def _algos(aml):
    return [m.algo for m in aml._aml.models]


def test_unknown_option_is_refused():
    with pytest.raises(TypeError):
        H2OAutoML(max_models=1, not_an_option=3)


def test_modeling_plan_restricts_and_orders_steps(fr):
    plan = A.custom_plan([("GBM", ["def_1"]), {"name": "GLM", "alias": "defaults"}, ("XGBoost", [("def_2", 3, 5)])])
    assert [(a, s) for a, s, _, _ in plan] == [("glm", "def_1"), ("gbm", "def_1"), ("xgboost", "def_2")]
    assert plan[-1][2:] == (3, 5)                        # user group / weight
    aml = H2OAutoML(max_models=5, max_runtime_secs_per_model=3, seed=1, nfolds=3, modeling_plan=[("GBM", ["def_1"]), "GLM"])
    aml.train(x=["a", "b"], y="y", training_frame=fr)
    assert sorted(set(_algos(aml)) - {"stackedensemble"}) == ["gbm", "glm"]
    assert sum(1 for x in _algos(aml) if x == "gbm") == 1
    with pytest.raises(ValueError):
        A.custom_plan([("GBM", ["no_such_step"])])


def test_exploitation_ratio_rescales_exploitation_work():
    steps = [("gbm", "def_1", 1, 10), ("gbm", "grid_1", 4, 60), ("gbm", "lr_annealing", 6, 10),
             ("xgboost", "lr_search", 6, 30)]
    out = {s: w for _, s, _, w in A.exploitation_weights(steps, 0.2)}
    assert out["def_1"] == 10 and out["grid_1"] == 60
    # exploration 70 kept; total 70 / 0.8 = 88 -> 18 for exploitation, split 10:30
    assert out["lr_annealing"] + out["lr_search"] == 88 - 70
    zero = {s: w for _, s, _, w in A.exploitation_weights(steps, 0.0)}
    assert zero["lr_annealing"] == 0 and zero["lr_search"] == 0
    assert A.exploitation_weights(steps, -1) == steps
    with pytest.raises(ValueError):
        H2OAutoML(max_models=1, exploitation_ratio=1.5)


def test_exploitation_ratio_zero_skips_lr_annealing(fr):
    plan = [("GBM", ["def_1", "lr_annealing"])]
    a0 = H2OAutoML(max_models=3, max_runtime_secs_per_model=3, seed=1, nfolds=0, modeling_plan=plan, exploitation_ratio=0.0)
    a0.train(x=["a", "b"], y="y", training_frame=fr)
    assert not any("lr_annealing" in m.key for m in a0._aml.models)
    a1 = H2OAutoML(max_models=1, max_runtime_secs_per_model=3, seed=1, nfolds=0, modeling_plan=plan, exploitation_ratio=0.5)
    a1.train(x=["a", "b"], y="y", training_frame=fr)
    # exploitation ignores the model-count budget when the ratio is on (GBMExploitationStep)
    assert any("lr_annealing" in m.key for m in a1._aml.models)


def test_target_encoding_preprocessing(fr, tmp_path):
    aml = H2OAutoML(max_models=1, max_runtime_secs_per_model=3, seed=1, nfolds=3, include_algos=["GBM"], preprocessing=["target_encoding"])
    aml.train(x=["a", "b", "hc"], y="y", training_frame=fr)
    m = aml._aml.models[0]
    assert m.preprocessors and m.preprocessors[0].algo == "targetencoder"
    assert "hc_te" in m.info.x and "hc" not in m.info.x
    assert m.params.get("fold_column") == "y_te_fold" and not m.params.get("nfolds")
    p = aml.leader.predict(fr)                           # raw frame: encoded by the model's preprocessor
    assert p.nrows == fr.nrows
    with pytest.raises(ValueError):
        m_path = aml.leader.download_mojo(str(tmp_path))  # noqa: F841
    with pytest.raises(ValueError):
        H2OAutoML(max_models=1, preprocessing=["pca"])


def test_monotone_constraints_reach_tree_models(fr):
    aml = H2OAutoML(max_models=2, max_runtime_secs_per_model=3, seed=1, nfolds=0, include_algos=["GBM", "GLM"], monotone_constraints={"a": 1})
    aml.train(x=["a", "b"], y="y", training_frame=fr)
    gbms = [m for m in aml._aml.models if m.algo == "gbm"]
    glms = [m for m in aml._aml.models if m.algo == "glm"]
    assert gbms and all(m.params.get("monotone_constraints") == {"a": 1} for m in gbms)
    assert glms and all(not m.params.get("monotone_constraints") for m in glms)   # GLM has no such parameter
    # increasing in `a`: predictions on a grid of a never decrease
    grid = h2o.H2OFrame(pd.DataFrame({"a": np.linspace(-3, 3, 50), "b": np.zeros(50)}))
    p1 = gbms[0].predict(grid).as_data_frame()["yes"].values
    assert np.all(np.diff(p1) >= -1e-7)


def test_balance_classes_reaches_models(fr):
    aml = H2OAutoML(max_models=1, max_runtime_secs_per_model=3, seed=1, nfolds=0, include_algos=["GBM"], balance_classes=True,
                    max_after_balance_size=2.0)
    aml.train(x=["a", "b"], y="y", training_frame=fr)
    m = aml._aml.models[0]
    assert m.params.get("balance_classes") is True and m.params.get("max_after_balance_size") == 2.0
    assert m.output.get("model_class_distrib") is not None


def test_keep_cv_predictions_and_checkpoints(fr, tmp_path):
    d = str(tmp_path / "ck")
    aml = H2OAutoML(max_models=2, max_runtime_secs_per_model=3, seed=1, nfolds=3, include_algos=["GBM", "GLM"], export_checkpoints_dir=d)
    aml.train(x=["a", "b"], y="y", training_frame=fr)
    assert all("cross_validation_holdout_predictions_frame_id" not in m.output for m in aml._aml.models)
    assert sorted(os.listdir(d)) == sorted(m.key for m in aml._aml.models)
    kept = H2OAutoML(max_models=2, max_runtime_secs_per_model=3, seed=1, nfolds=3, include_algos=["GBM", "GLM"], keep_cross_validation_predictions=True)
    kept.train(x=["a", "b"], y="y", training_frame=fr)
    base = [m for m in kept._aml.models if m.algo != "stackedensemble"]
    assert all(m.output.get("cross_validation_holdout_predictions_frame_id") for m in base)


def test_blending_frame_trains_blended_ensembles(fr):
    tr, bl = fr.split_frame([0.7], seed=2)
    aml = H2OAutoML(max_models=2, max_runtime_secs_per_model=3, seed=1, nfolds=0, include_algos=["GBM", "GLM", "StackedEnsemble"])
    aml.train(x=["a", "b"], y="y", training_frame=tr, blending_frame=bl)
    ses = [m for m in aml._aml.models if m.algo == "stackedensemble"]
    assert ses and all(m.output["stacking_strategy"] == "blending" for m in ses)
    assert ses[0].model_performance(bl).auc() > 0.6
