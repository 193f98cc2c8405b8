"""h2o-py submodules users import directly: h2o.cross_validation (fold iterators), h2o.scoring.make_leaderboard,
h2o.persist, h2o.information_retrieval.tf_idf, h2o.two_dim_table, h2o.model, h2o.backend.H2OLocalServer."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGradientBoostingEstimator, H2OGeneralizedLinearEstimator


@pytest.fixture(scope="module")
def fr():
    h2o.init(verbose=False)
    rng = np.random.default_rng(11)
    d = pd.DataFrame({"a": rng.normal(size=500), "b": rng.normal(size=500)})
    d["y"] = np.where(d.a + rng.normal(size=500) * 0.5 > 0, "1", "0")
    return h2o.H2OFrame(d, column_types={"y": "enum"})


def test_fold_iterators(fr):
    from h2o.cross_validation import H2OKFold, H2OStratifiedKFold
    kf = H2OKFold(fr, n_folds=4, seed=1)
    assert len(kf) == 4
    tot = 0
    for train, test in kf:
        tr, te = train.as_data_frame().iloc[:, 0].to_numpy(), test.as_data_frame().iloc[:, 0].to_numpy()
        assert np.all(tr + te == 1)
        tot += te.sum()
    assert tot == fr.nrows
    sk = H2OStratifiedKFold(fr["y"], n_folds=3, seed=1)
    assert sum(t.as_data_frame().iloc[:, 0].sum() for _, t in sk) == fr.nrows


def test_make_leaderboard(fr):
    g = H2OGradientBoostingEstimator(ntrees=5, seed=1)
    g.train(x=["a", "b"], y="y", training_frame=fr)
    l = H2OGeneralizedLinearEstimator(family="binomial")
    l.train(x=["a", "b"], y="y", training_frame=fr)
    lb = h2o.make_leaderboard([g, l], fr, extra_columns="ALL").as_data_frame()
    assert set(lb.model_id) == {g.model_id, l.model_id}
    assert {"auc", "logloss", "training_time_ms", "predict_time_per_row_ms", "algo"} <= set(lb.columns)
    assert lb.auc.is_monotonic_decreasing
    lb2 = h2o.make_leaderboard([g.model_id, l.model_id], scoring_data="train").as_data_frame()
    assert abs(lb2.set_index("model_id").auc[g.model_id] - g.auc()) < 1e-12
    with pytest.raises(ValueError):
        h2o.make_leaderboard(g, scoring_data="bogus")


def test_misc_modules(fr):
    from h2o.persist import remove_s3_credentials, set_s3_credentials
    assert callable(set_s3_credentials) and callable(remove_s3_credentials)
    from h2o.two_dim_table import H2OTwoDimTable
    t = H2OTwoDimTable("T", col_header=["x", "y"], cell_values=[[1, 2], [3, 4]])
    assert t["y"] == [2, 4] and t.as_data_frame().shape == (2, 2) and len(t) == 2
    from h2o.model import ConfusionMatrix, H2OBinomialModelMetrics, ModelBase
    g = H2OGradientBoostingEstimator(ntrees=3, seed=1)
    g.train(x=["a", "b"], y="y", training_frame=fr)
    assert isinstance(g, ModelBase) and isinstance(g.model_performance(fr), H2OBinomialModelMetrics)
    assert isinstance(g.confusion_matrix(), ConfusionMatrix)
    from h2o.information_retrieval import tf_idf
    docs = h2o.H2OFrame(pd.DataFrame({"id": [0, 1], "text": ["a b a", "b c"]}), column_types={"text": "string"})
    out = tf_idf(docs, 0, 1).as_data_frame()
    assert len(out) == 4


def test_local_server_roundtrip():
    from h2o.backend import H2OLocalServer
    srv = H2OLocalServer.start(verbose=False)
    try:
        assert srv.is_running()
        import requests
        r = requests.get(srv.url + "/3/Cloud", timeout=30)
        assert r.status_code == 200 and "cloud_name" in r.json()
    finally:
        srv.shutdown()
    assert not srv.is_running()
