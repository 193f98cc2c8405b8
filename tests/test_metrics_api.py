"""h2o-py model-metrics surface on the engine's ModelMetrics (h2o-py/h2o/model/metrics/binomial.py et al.):
metric() / F1() / accuracy() ... with thresholds, find_threshold_by_max_metric, confusion_matrix, roc, gains_lift,
and the multinomial / clustering / regression scalars."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGradientBoostingEstimator, H2OKMeansEstimator, H2OGeneralizedLinearEstimator


@pytest.fixture(scope="module")
def fr():
    h2o.init(verbose=False)
    rng = np.random.default_rng(7)
    d = pd.DataFrame({"a": rng.normal(size=800), "b": rng.normal(size=800)})
    d["y"] = np.where(d.a + rng.normal(size=800) * 0.7 > 0, "1", "0")
    d["m"] = np.where(d.b > 0.5, "p", np.where(d.b < -0.5, "q", "s"))
    d["r"] = d.a * 2 + rng.normal(size=800)
    return h2o.H2OFrame(d, column_types={"y": "enum", "m": "enum"})


def test_binomial_threshold_api(fr):
    m = H2OGradientBoostingEstimator(ntrees=5, seed=1)
    m.train(x=["a", "b"], y="y", training_frame=fr)
    perf = m.model_performance(fr)
    t = perf.find_threshold_by_max_metric("f1")
    f1 = perf.F1()
    assert f1[0][0] == t and f1.value == max(perf.metric("f1", "all").value)
    acc = perf.accuracy([0.5])
    assert len(acc) == 1 and 0.5 < acc.value[0] <= 1
    assert abs(perf.error(0.5).value - (1 - perf.accuracy(0.5).value)) < 1e-12
    cm = perf.confusion_matrix()
    assert cm.to_list()[0][0] + cm.to_list()[0][1] + cm.to_list()[1][0] + cm.to_list()[1][1] == fr.nrows
    # the F1-optimal confusion matrix reproduces that F1
    (tn, fp), (fn, tp) = cm.to_list()
    assert abs(2 * tp / (2 * tp + fp + fn) - f1.value) < 1e-9
    cms = perf.confusion_matrix(metrics=["accuracy", "precision"])
    assert len(cms) == 2
    fprs, tprs = perf.roc()
    assert len(fprs) == len(tprs) == len(perf.thresholds) and all(0 <= v <= 1 for v in fprs + tprs)
    assert perf.recall(0.5).value == perf.tpr(0.5).value == perf.sensitivity(0.5).value
    assert abs(perf.specificity(0.5).value + perf.fpr(0.5).value - 1) < 1e-12
    gl = perf.gains_lift()
    assert list(gl.columns)[:2] == ["group", "cumulative_data_fraction"] and len(gl) == 16
    assert perf.n() == fr.nrows
    with pytest.raises(ValueError):
        perf.metric("bogus")


def test_multinomial_clustering_regression_scalars(fr):
    m = H2OGradientBoostingEstimator(ntrees=5, seed=1)
    m.train(x=["a", "b"], y="m", training_frame=fr)
    cm = m.model_performance(fr).confusion_matrix()
    assert len(cm.to_list()) == 3 and sum(map(sum, cm.to_list())) == fr.nrows
    assert list(cm.table.columns)[-2:] == ["Error", "Rate"]
    k = H2OKMeansEstimator(k=3, seed=1)
    k.train(x=["a", "b"], training_frame=fr)
    pk = k.model_performance(fr)
    assert abs(pk.totss() - (pk.tot_withinss() + pk.betweenss())) < 1e-6 * pk.totss()
    g = H2OGeneralizedLinearEstimator(lambda_=0)
    g.train(x=["a", "b"], y="r", training_frame=fr)
    pg = g.model_performance(fr)
    assert pg.residual_deviance() is not None and pg.null_deviance() >= pg.residual_deviance()


def test_glm_frame_deviance_matches_training(fr):
    g = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0)
    g.train(x=["a", "b"], y="r", training_frame=fr)
    out = g._m().output
    pg = g.model_performance(fr)
    assert abs(pg.residual_deviance() - out["residual_deviance"]) < 1e-6 * out["residual_deviance"]
    assert abs(pg.null_deviance() - out["null_deviance"]) < 1e-6 * out["null_deviance"]
    assert pg.residual_degrees_of_freedom() == out["residual_degrees_of_freedom"]
    assert abs(pg.aic() - out["aic"]) < 1e-6 * abs(out["aic"])


def test_model_level_metric_delegation(fr):
    """H2OBinomialModel accessors (model/models/binomial.py): training metrics by default, a dict for several."""
    tr, va = fr.split_frame([0.7], seed=2)
    m = H2OGradientBoostingEstimator(ntrees=5, seed=1)
    m.train(x=["a", "b"], y="y", training_frame=tr, validation_frame=va)
    assert m.F1().value == m.model_performance(train=True).F1().value
    both = m.F1(train=True, valid=True)
    assert set(both) == {"train", "valid"}
    assert m.find_threshold_by_max_metric("f1", valid=True) == m.model_performance(valid=True).find_threshold_by_max_metric("f1")
    cm = m.confusion_matrix(valid=True)
    assert sum(map(sum, cm.to_list())) == va.nrows
    assert sum(map(sum, m.confusion_matrix(va).to_list())) == va.nrows
    f, t = m.roc()
    ks = m.kolmogorov_smirnov()
    assert 0 < ks <= 1 and abs(ks - max(abs(b - a) for a, b in zip(f, t))) < 1e-12
    assert 0 <= m.mean_per_class_error() <= 1 and len(m.gains_lift()) == 16


def test_kmeans_model_accessors(fr):
    k = H2OKMeansEstimator(k=3, seed=1)
    k.train(x=["a", "b"], training_frame=fr)
    cs = k.centroid_stats()
    assert list(cs.columns) == ["centroid", "size", "within_cluster_sum_of_squares"] and cs["size"].sum() == fr.nrows
    assert k.num_iterations() >= 1 and abs(sum(k.withinss()) - k.tot_withinss()) < 1e-6 * k.tot_withinss()
