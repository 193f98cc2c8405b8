"""Custom metrics / custom GBM distribution (water/udf/*) and segment models (hex/segments/*)."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator


@pytest.fixture(scope="module")
def df():
    h2o.init(verbose=False)
    rng = np.random.default_rng(7)
    n = 900
    d = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "seg": rng.choice(["s1", "s2", "s3"], n)})
    d["r"] = 2 * d.a - d.b + (d.seg == "s2") * 3 + rng.normal(size=n) * 0.2
    d["y"] = np.where(d.a + rng.normal(size=n) * 0.5 > 0, "1", "0")
    return h2o.H2OFrame(d, column_types={"seg": "enum", "y": "enum"})


class CustomMae:
    def map(self, pred, act, w, o, model):
        return [w * abs(act[0] - pred[0]), w]

    def reduce(self, l, r):
        return [l[0] + r[0], l[1] + r[1]]

    def metric(self, l):
        return l[0] / l[1]


class ScalarOnlyMae(CustomMae):
    def map(self, pred, act, w, o, model):
        import math
        return [w * math.fabs(act[0] - pred[0]), w]


class CustomGaussian:
    def link(self):
        return "identity"

    def init(self, w, o, y):
        return [w * (y - o), w]

    def gradient(self, y, f):
        return y - f

    def gamma(self, w, y, z, f):
        return [w * z, w]


@pytest.mark.parametrize("cls", [CustomMae, ScalarOnlyMae])
def test_custom_metric_matches_mae(df, cls):
    ref = h2o.upload_custom_metric(cls, func_name=f"mae_{cls.__name__}")
    assert ref.startswith("python:mae_")
    m = H2OGradientBoostingEstimator(ntrees=5, seed=1, custom_metric_func=ref)
    m.train(x=["a", "b", "seg"], y="r", training_frame=df)
    tm = m._model.output["training_metrics"]
    assert tm["custom_metric_name"] == f"mae_{cls.__name__}"
    assert tm["custom_metric_value"] == pytest.approx(tm["mae"], rel=1e-6)


MAE_SRC = '''
class CustomMaeFunc:
    def map(self, pred, act, w, o, model):
        return [abs(act[0] - pred[0]), 1]

    def reduce(self, l, r):
        return [l[0] + r[0], l[1] + r[1]]

    def metric(self, l):
        return l[0] / l[1]
'''


def test_custom_metric_from_source_string(df):
    # h2o.py:upload_custom_metric string form: class source + class_name
    ref = h2o.upload_custom_metric(MAE_SRC, class_name="CustomMaeFunc", func_name="mae_src")
    assert ref == "python:mae_src=metrics.CustomMaeFuncWrapper"
    m = H2OGradientBoostingEstimator(ntrees=5, seed=1, custom_metric_func=ref)
    m.train(x=["a", "b", "seg"], y="r", training_frame=df)
    tm = m._model.output["training_metrics"]
    assert tm["custom_metric_value"] == pytest.approx(tm["mae"], rel=1e-6)
    with pytest.raises(ValueError):
        h2o.upload_custom_metric(MAE_SRC)


def test_custom_distribution_equals_gaussian(df):
    ref = h2o.upload_custom_distribution(CustomGaussian, func_name="custom_gaussian")
    kw = dict(ntrees=6, max_depth=3, seed=1)
    c = H2OGradientBoostingEstimator(distribution="custom", custom_distribution_func=ref, **kw)
    c.train(x=["a", "b", "seg"], y="r", training_frame=df)
    g = H2OGradientBoostingEstimator(distribution="gaussian", **kw)
    g.train(x=["a", "b", "seg"], y="r", training_frame=df)
    pc = c.predict(df).as_data_frame().values[:, 0]
    pg = g.predict(df).as_data_frame().values[:, 0]
    np.testing.assert_allclose(pc, pg, rtol=1e-5, atol=1e-5)


def test_segment_models(df):
    est = H2OGeneralizedLinearEstimator(family="gaussian", segment_columns=["seg"])
    sm = est.train_segments(x=["a", "b"], y="r", training_frame=df, parallelism=2)
    tab = sm.as_frame().as_data_frame()
    assert sorted(tab["seg"].tolist()) == ["s1", "s2", "s3"]
    assert (tab["status"] == "SUCCEEDED").all()
    for m, s in zip(sm.models(), tab["seg"]):
        assert m.coef()["a"] == pytest.approx(2.0, abs=0.1)
    # a segment that cannot train is reported, not raised
    bad = H2OGeneralizedLinearEstimator(family="binomial", segment_columns="seg")
    sm2 = bad.train_segments(x=["a", "b"], y="r", training_frame=df)
    assert (sm2.as_frame().as_data_frame()["status"] == "FAILED").all()


def test_grep_model(tmp_path):
    from h2o.estimators import H2OGrepEstimator
    from llama_github_io_amd.models import grep as G
    h2o.init(verbose=False)
    text = "alpha beta\ngamma alphabet\nalpha"
    p = tmp_path / "t.txt"
    p.write_text(text)
    g = H2OGrepEstimator(regex="alpha[a-z]*", path=str(p))
    g.train()
    assert g._model.matches() == ["alpha", "alphabet", "alpha"]
    assert g._model.offsets() == [m.start() for m in __import__("re").finditer("alpha[a-z]*", text)]
    # chunk boundaries: a match straddling two chunks is reported exactly once
    old = G._CHUNK
    try:
        G._CHUNK = 7
        m, o = G.grep_text(text, "alpha[a-z]*")
        assert m == ["alpha", "alphabet", "alpha"]
    finally:
        G._CHUNK = old


def test_grid_recovery_resumes_without_retraining(df, tmp_path, monkeypatch):
    from h2o.grid import H2OGridSearch
    from llama_github_io_amd import grid as G
    from llama_github_io_amd.models import builder
    rdir = str(tmp_path / "rec")
    calls = []
    real = builder.train

    def crashing(algo, p, *a, **k):
        calls.append(p["max_depth"])
        if len(calls) == 3:
            raise KeyboardInterrupt("simulated node loss")
        return real(algo, p, *a, **k)
    monkeypatch.setattr(G.builder, "train", crashing)
    gs = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=3, seed=1), {"max_depth": [2, 3, 4, 5]},
                       grid_id="rec_grid", recovery_dir=rdir)
    with pytest.raises(KeyboardInterrupt):
        G.grid_search("gbm", {"max_depth": [2, 3, 4, 5]}, dict(ntrees=3, seed=1), ["a", "b"], "r", df,
                      grid_id="rec_grid", recovery_dir=rdir)
    import json, os
    meta = json.load(open(os.path.join(rdir, "recovery.json")))
    assert [m["hyper"] for m in meta["models"]] == [[2], [3]]
    from llama_github_io_amd.core import dkv
    dkv.remove("rec_grid")
    monkeypatch.setattr(G.builder, "train", lambda algo, p, *a, **k: (calls.append(p["max_depth"]), real(algo, p, *a, **k))[1])
    calls.clear()
    g = h2o.resume(rdir)
    assert calls == [4, 5]                       # finished models were loaded, not retrained
    assert sorted(h[0] for h in g.hyper_values) == [2, 3, 4, 5]
    assert not os.path.exists(rdir)              # cleaned up on success
    _ = gs


class MaxAbsError:
    """Non-additive reduce (max): the vectorised path must fold with reduce, never sum."""
    def map(self, pred, act, w, o, model):
        import numpy as _np
        return [_np.abs(_np.asarray(act[0]) - _np.asarray(pred[0]))]

    def reduce(self, l, r):
        import numpy as _np
        return [_np.maximum(l[0], r[0])]

    def metric(self, l):
        return l[0]


def test_custom_metric_non_additive_reduce(df):
    ref = h2o.upload_custom_metric(MaxAbsError, func_name="maxerr")
    m = H2OGradientBoostingEstimator(ntrees=3, seed=1, custom_metric_func=ref)
    m.train(x=["a", "b", "seg"], y="r", training_frame=df)
    tm = m._model.output["training_metrics"]
    p = m.predict(df).as_data_frame().iloc[:, 0].values
    r = df["r"].as_data_frame().iloc[:, 0].values
    assert tm["custom_metric_value"] == pytest.approx(float(np.max(np.abs(r - p))), rel=1e-5)
