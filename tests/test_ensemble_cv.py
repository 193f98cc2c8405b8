"""Stacked Ensemble / AutoML leaderboard use out-of-fold metrics (StackedEnsembleStepsProvider.java:146:
metalearner_nfolds = AutoML nfolds; the SE's cross-validation metrics are the metalearner's own CV)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def frame():
    import h2o
    h2o.init(verbose=False)
    rng = np.random.default_rng(3)
    n = 600
    X = rng.normal(size=(n, 5))
    y = np.where(rng.random(n) < 1 / (1 + np.exp(-(X[:, 0] - X[:, 1] + 0.5 * X[:, 2] * X[:, 3]))), "a", "b")
    import pandas as pd
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(5)])
    df["y"] = y
    return h2o.H2OFrame(df, column_types={"y": "enum"})


def test_se_cv_metrics_are_out_of_fold(frame):
    from llama_github_io_amd.models import builder
    base = []
    for algo, p in (("gbm", dict(ntrees=10, max_depth=3, seed=1)), ("glm", dict(family="binomial"))):
        base.append(builder.train(algo, dict(p, nfolds=3, fold_assignment="Modulo", keep_cross_validation_predictions=True),
                                  x=[f"x{i}" for i in range(5)], y="y", training_frame=frame))
    se = builder.train("stackedensemble", dict(base_models=[m.key for m in base], metalearner_nfolds=3, seed=2),
                       x=[f"x{i}" for i in range(5)], y="y", training_frame=frame)
    cv = se.output["cross_validation_metrics"]
    meta = se.meta
    assert cv is not None and cv is meta.output["cross_validation_metrics"]
    # the out-of-fold AUC differs from (and is not above) the metalearner's in-sample AUC
    assert cv["AUC"] != meta.output["training_metrics"]["AUC"]
    assert cv["AUC"] <= meta.output["training_metrics"]["AUC"] + 1e-9
    # without metalearner CV there is no cross-validation estimate at all (never the training fit)
    se0 = builder.train("stackedensemble", dict(base_models=[m.key for m in base], seed=2),
                        x=[f"x{i}" for i in range(5)], y="y", training_frame=frame)
    assert se0.output["cross_validation_metrics"] is None


def test_se_logit_transform_and_levelone(frame):
    from llama_github_io_amd.core import dkv
    from llama_github_io_amd.models import builder
    base = [builder.train("gbm", dict(ntrees=5, max_depth=2, seed=s, nfolds=3, fold_assignment="Modulo",
                                      keep_cross_validation_predictions=True),
                          x=[f"x{i}" for i in range(5)], y="y", training_frame=frame) for s in (1, 2)]
    se = builder.train("stackedensemble", dict(base_models=[m.key for m in base], metalearner_transform="Logit",
                                               keep_levelone_frame=True), x=[f"x{i}" for i in range(5)], y="y",
                       training_frame=frame)
    l1 = dkv.get(se.output["levelone_frame_id"])
    assert l1.ncols == 3 and l1.nrows == frame.nrows
    p = se.predict(frame).as_data_frame()
    assert np.all((p.iloc[:, 1] >= 0) & (p.iloc[:, 1] <= 1))


def test_automl_leaderboard_uses_se_cv(frame):
    from h2o.automl import H2OAutoML
    a = H2OAutoML(max_models=2, seed=1, nfolds=3, include_algos=["GLM", "GBM", "StackedEnsemble"])
    a.train(y="y", training_frame=frame)
    ses = [m for m in a._aml.models if m.algo == "stackedensemble"]
    assert ses
    for se in ses:
        cvm = se.output["cross_validation_metrics"]
        assert cvm is se.meta.output["cross_validation_metrics"]
        assert cvm is not se.output["training_metrics"]
