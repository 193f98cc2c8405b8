"""ModelBase surface of the in-process estimators (reference ``h2o-py/h2o/model/model_base.py`` and
``h2o-py/h2o/model/extensions``): every accessor returns the model's real values, not placeholders."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                            H2OPrincipalComponentAnalysisEstimator)


@pytest.fixture(scope="module")
def fr():
    h2o.init(verbose=False)
    rng = np.random.default_rng(7)
    n = 600
    a, b = rng.normal(size=n), rng.normal(size=n)
    g = rng.choice(["m", "f"], n)
    y = np.where(1.5 * a - b + (g == "m") * 0.5 + rng.normal(size=n) > 0, "yes", "no")
    r = 2 * a + np.abs(b) + rng.normal(size=n) * 0.3 + 5
    return h2o.H2OFrame(pd.DataFrame({"a": a, "b": b, "g": g, "y": y, "r": r}))


@pytest.fixture(scope="module")
def gbm(fr):
    m = H2OGradientBoostingEstimator(ntrees=6, max_depth=3, seed=1, nfolds=3, sample_rate=0.7,
                                     keep_cross_validation_predictions=True, keep_cross_validation_fold_assignment=True)
    m.train(x=["a", "b", "g"], y="y", training_frame=fr)
    return m


def test_metric_accessors_and_bookkeeping(gbm):
    auc = gbm.auc()
    assert abs(gbm.gini() - (2 * auc - 1)) < 1e-12
    both = gbm.gini(train=True, xval=True)
    assert set(both) == {"train", "xval"} and both["train"] == gbm.gini()
    assert gbm.pr_auc() == gbm.aucpr()
    assert gbm.type == "classifier" and gbm.ntrees_actual == 6 and gbm.is_cross_validated()
    assert gbm.full_parameters["ntrees"]["actual_value"] == 6
    assert gbm.run_time >= 0 and gbm.summary() is not None
    assert len(gbm.score_history()) >= 1
    gbm.show()


def test_cross_validation_accessors(gbm, fr):
    keys = gbm.xval_keys()
    assert len(keys) == 3 and [m.key for m in gbm.get_xval_models()] == keys
    fa = gbm.cross_validation_fold_assignment().as_data_frame()["fold_assignment"].to_numpy()
    preds = gbm.cross_validation_predictions()
    assert len(preds) == 3
    ho = gbm.cross_validation_holdout_predictions().as_data_frame()["yes"].to_numpy()
    tot = sum(p.as_data_frame()["yes"].to_numpy() for p in preds)
    assert np.allclose(tot, ho)                        # each row is predicted by exactly its fold's model
    for i, p in enumerate(preds):
        assert np.all(p.as_data_frame()["yes"].to_numpy()[fa != i] == 0)


def test_tree_path_accessors(gbm, fr):
    ff = gbm.feature_frequencies(fr).as_data_frame()
    assert list(ff.columns) == ["a", "b", "g"] and (ff.to_numpy() >= 0).all()
    # every row walks every tree to a leaf: path lengths between 1 and max_depth per tree
    per_row = ff.to_numpy().sum(1)
    assert per_row.min() >= 6 and per_row.max() <= 6 * 3
    rta = gbm.row_to_tree_assignment(fr).as_data_frame()
    assert rta.shape == (fr.nrows, 7)
    frac = rta.iloc[:, 1:].to_numpy().mean()
    assert 0.6 < frac < 0.8                            # sample_rate = 0.7


def test_explanations_and_plots(gbm, fr, tmp_path):
    pi = gbm.permutation_importance(fr, use_pandas=True)
    assert pi.iloc[0]["Variable"] == "a"
    gbm.varimp_plot(save_plot_path=str(tmp_path / "vi.png"))
    gbm.scoring_history_plot(save_plot_path=str(tmp_path / "sh.png"))
    gbm.fair_roc_plot(fr, "g", None, "yes", save_plot_path=str(tmp_path / "roc.png"))
    gbm.fair_pr_plot(fr, "g", None, "yes")
    assert (tmp_path / "roc.png").exists()
    pva = gbm.predicted_vs_actual_by_variable(fr, gbm.predict(fr), "g")
    assert list(pva["level"]) == ["f", "m"] and pva["count"].sum() == fr.nrows
    rep = gbm.inspect_model_fairness(fr, ["g"], None, "yes")
    assert rep is not None


def test_glm_coefficient_family(fr, tmp_path):
    m = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0.0, compute_p_values=True,
                                      generate_variable_inflation_factors=True)
    m.train(x=["a", "b"], y="r", training_frame=fr)
    c = m.coef()
    assert abs(c["a"] - 2.0) < 0.2 and set(m.coef_norm()) == set(c)
    t = m.coef_with_p_values()
    assert list(t["names"]) == list(c) and (t["p_value"] >= 0).all()
    assert m.residual_deviance() < m.null_deviance()
    assert m.residual_degrees_of_freedom() == fr.nrows - 3
    assert m.aic() is not None and m.mean_residual_deviance() > 0 and m.rmsle() > 0
    assert set(m.get_variable_inflation_factors()) >= {"a", "b"}
    m.std_coef_plot(save_plot_path=str(tmp_path / "coef.png"))


def test_deeplearning_and_pca_internals(fr):
    dl = H2ODeepLearningEstimator(hidden=[5], epochs=2, seed=1, reproducible=True)
    dl.train(x=["a", "b", "g"], y="r", training_frame=fr)
    assert dl.biases(0).nrows == 5 and dl.weights(0).ncols in (3, 4)
    assert len(dl.normsub()) == 2 and len(dl.normmul()) == 2 and dl.respmul() and dl.respsub()
    assert dl.catoffsets()[-1] >= 1
    p = H2OPrincipalComponentAnalysisEstimator(k=2, transform="STANDARDIZE")
    p.train(x=["a", "b"], training_frame=fr)
    rot = p.rotation()
    assert rot.shape == (2, 2)
