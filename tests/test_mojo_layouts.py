"""Reference-layout MOJOs (DeepLearning, PCA, Word2Vec, Isotonic, StackedEnsemble): the exported zip
holds the reference keys/blobs and ``h2o.import_mojo`` scores exactly like the original model."""
import zipfile

import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                            H2OIsotonicRegressionEstimator, H2OPrincipalComponentAnalysisEstimator,
                            H2OStackedEnsembleEstimator, H2OWord2vecEstimator)
from llama_github_io_amd.mojo.reader import parse_mojo


@pytest.fixture(scope="module")
def df():
    h2o.init(verbose=False)
    rng = np.random.default_rng(3)
    n = 800
    a = rng.normal(size=n)
    a[rng.random(n) < 0.05] = np.nan
    c = rng.choice(list("pqrs"), n).astype(object)
    c[rng.random(n) < 0.05] = None
    d = pd.DataFrame({"a": a, "c": c, "b": rng.normal(size=n), "k": rng.choice(list("uv"), n)})
    d["y"] = np.where(np.nan_to_num(d.a) - d.b + (d.c == "p") + rng.normal(size=n) * 0.3 > 0, "1", "0")
    d["m"] = rng.choice(["m0", "m1", "m2"], n)
    d["r"] = np.sin(np.nan_to_num(d.a)) * 2 + d.b + rng.normal(size=n) * 0.1
    return h2o.H2OFrame(d, column_types={"y": "enum", "c": "enum", "k": "enum", "m": "enum"})


def _roundtrip(est, df, tmp_path):
    path = est.download_mojo(str(tmp_path))
    g = h2o.import_mojo(path)
    return path, est.predict(df).as_data_frame(), g.predict(df).as_data_frame()


@pytest.mark.parametrize("kw,y", [
    (dict(hidden=[8, 6], activation="Rectifier"), "y"),
    (dict(hidden=[7], activation="Tanh", use_all_factor_levels=False), "m"),
    (dict(hidden=[5, 4], activation="Maxout"), "y"),
    (dict(hidden=[6], activation="ExpRectifier"), "r"),
    (dict(hidden=[6], activation="RectifierWithDropout", hidden_dropout_ratios=[0.2]), "r"),
])
def test_deeplearning_mojo_reference_layout(df, tmp_path, kw, y):
    m = H2ODeepLearningEstimator(epochs=2, seed=1, reproducible=True, **kw)
    m.train(x=["a", "c", "b", "k"], y=y, training_frame=df)
    path, a, b = _roundtrip(m, df, tmp_path)
    mj = parse_mojo(path)
    ki = mj["info"]
    # reference keys (DeepLearningMojoWriter.writeModelData), categoricals first in [columns]
    for key in ("nums", "cats", "cat_offsets", "norm_mul", "norm_sub", "activation", "neural_network_sizes",
                "weight_layer0", "bias_layer0", "hidden_dropout_ratios", "distribution", "mean_imputation"):
        assert key in ki, key
    assert mj["columns"][:2] == ["c", "k"] and int(ki["cats"]) == 2
    cols = [c for c in a.columns]
    for c in cols:
        if c == "predict" and y != "r":
            assert (a[c].astype(str) == b[c].astype(str)).mean() > 0.99
        else:
            np.testing.assert_allclose(a[c].astype(float).values, b[c].astype(float).values, rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("transform", ["NONE", "DEMEAN", "STANDARDIZE"])
def test_pca_mojo_reference_layout(df, tmp_path, transform):
    p = H2OPrincipalComponentAnalysisEstimator(k=3, transform=transform, use_all_factor_levels=True)
    p.train(x=["b", "c", "k"], training_frame=df)
    path = p.download_mojo(str(tmp_path))
    with zipfile.ZipFile(path) as z:
        assert "eigenvectors_raw" in z.namelist()
    g = h2o.import_mojo(path)
    ok = ~df.as_data_frame()["c"].isna().values       # NA categoricals: reference skips, training imputes
    a = p.predict(df).as_data_frame().values[ok]
    b = g.predict(df).as_data_frame().values[ok]
    np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)


def test_word2vec_mojo(tmp_path):
    h2o.init(verbose=False)
    rng = np.random.default_rng(0)
    words = []
    for i in range(400):
        words += list(rng.choice(["cat", "dog", "cow"] if i % 2 else ["one", "two", "six"], 5)) + [None]
    fr = h2o.H2OFrame(pd.DataFrame({"w": words}), column_types={"w": "string"})
    w2v = H2OWord2vecEstimator(vec_size=6, min_word_freq=1, epochs=2, seed=1, sent_sample_rate=0)
    w2v.train(training_frame=fr)
    path = w2v.download_mojo(str(tmp_path))
    mj = parse_mojo(path)
    assert int(mj["info"]["vec_size"]) == 6 and len(mj["files"]["vectors"]) == int(mj["info"]["vocab_size"]) * 6 * 4
    g = h2o.import_mojo(path)
    assert g.find_synonyms("cat", 2) == pytest.approx(w2v._model.find_synonyms("cat", 2), rel=1e-5)


def test_isotonic_mojo(df, tmp_path):
    m = H2OIsotonicRegressionEstimator(out_of_bounds="clip")
    m.train(x=["b"], y="r", training_frame=df)
    path, a, b = _roundtrip(m, df, tmp_path)
    assert "calib/thresholds_x" in parse_mojo(path)["files"]
    np.testing.assert_allclose(a.values.astype(float), b.values.astype(float), rtol=1e-6, atol=1e-9)


def test_stacked_ensemble_nested_mojo(df, tmp_path):
    x = ["a", "c", "b", "k"]
    kw = dict(nfolds=3, fold_assignment="Modulo", keep_cross_validation_predictions=True, seed=1)
    g1 = H2OGradientBoostingEstimator(ntrees=5, **kw)
    g1.train(x=x, y="y", training_frame=df)
    g2 = H2OGeneralizedLinearEstimator(family="binomial", **kw)
    g2.train(x=x, y="y", training_frame=df)
    se = H2OStackedEnsembleEstimator(base_models=[g1, g2])
    se.train(x=x, y="y", training_frame=df)
    path, a, b = _roundtrip(se, df, tmp_path)
    ki = parse_mojo(path)["info"]
    assert int(ki["submodel_count"]) == 3 and int(ki["base_models_num"]) == 2
    with zipfile.ZipFile(path) as z:
        assert any(n.startswith("models/") and n.endswith("model.ini") for n in z.namelist())
    np.testing.assert_allclose(a["1"].values, b["1"].values, rtol=1e-5, atol=1e-6)
    # labels agree except where p1 sits on the default threshold itself (the max-F1 threshold is one of the
    # training predictions; a 1-ulp difference in p1 may land on either side)
    thr = se._model.default_threshold()
    diff = (a["predict"] != b["predict"]).values & (np.abs(a["1"].values.astype(float) - thr) > 1e-6)
    assert diff.sum() == 0


def test_extended_isolation_forest_mojo(df, tmp_path):
    from h2o.estimators import H2OExtendedIsolationForestEstimator
    m = H2OExtendedIsolationForestEstimator(ntrees=7, sample_size=64, extension_level=1, seed=3)
    m.train(x=["b", "r"], training_frame=df)
    path, a, b = _roundtrip(m, df, tmp_path)
    assert "trees/t06.bin" in parse_mojo(path)["files"]
    np.testing.assert_allclose(a.values.astype(float), b.values.astype(float), rtol=1e-6, atol=1e-9)


# ------------------------------------------------------------------------------------------------ XGBoost
@pytest.mark.parametrize("kind", ["binomial", "regression", "multinomial"])
def test_xgboost_mojo_booster_bytes(tmp_path, kind):
    import struct
    import zipfile
    import h2o
    import pandas as pd
    from h2o.estimators import H2OXGBoostEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(7)
    n = 1500
    df = pd.DataFrame(rng.normal(size=(n, 4)), columns=list("abcd"))
    df.loc[rng.random(n) < 0.05, "b"] = np.nan
    s = df.a.fillna(0) - 0.5 * df.b.fillna(0) + 0.3 * df.c
    if kind == "binomial":
        df["y"] = np.where(s + rng.normal(0, 0.5, n) > 0, "p", "n")
    elif kind == "multinomial":
        df["y"] = np.digitize(s, [-0.5, 0.5]).astype(str)
    else:
        df["y"] = s + rng.normal(0, 0.1, n)
    types = {"y": "enum"} if kind != "regression" else None
    fr = h2o.H2OFrame(df, column_types=types)
    m = H2OXGBoostEstimator(ntrees=8, max_depth=4, seed=3)
    m.train(x=list("abcd"), y="y", training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    with zipfile.ZipFile(path) as z:
        ini = z.read("model.ini").decode()
        bb = z.read("boosterBytes")
        assert b"0 a q" in z.read("feature_map")
    assert "algo = xgboost" in ini and "nums = 4" in ini and "use_java_scoring_by_default = true" in ini
    (bs, nf, ncls) = struct.unpack_from("<fIi", bb, 0)
    assert nf == 4 and ncls == (3 if kind == "multinomial" else 0)
    objlen = struct.unpack_from("<Q", bb, 136)[0]
    assert bb[144:144 + objlen].decode() == {"binomial": "binary:logistic", "regression": "reg:squarederror",
                                             "multinomial": "multi:softprob"}[kind]
    g = h2o.import_mojo(path)
    a = m.predict(fr).as_data_frame().iloc[:, -1].values.astype(float)
    b = g.predict(fr).as_data_frame().iloc[:, -1].values.astype(float)
    np.testing.assert_allclose(b, a, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("strata", [False, True])
def test_coxph_mojo_reference_layout(tmp_path, strata):
    from h2o.estimators import H2OCoxProportionalHazardsEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(5)
    n = 600
    x = rng.normal(size=n)
    g = rng.choice(list("abc"), n)
    s = rng.choice(["s0", "s1"], n)
    T = rng.exponential(1 / np.exp(0.7 * x + (g == "b") * 0.5))
    C = rng.exponential(2.0, n)
    # the stop column first: the scorer must pick the predictors, not the frame's first columns
    d = pd.DataFrame({"time": np.minimum(T, C), "x": x, "g": g, "s": s, "event": (T <= C).astype(int)})
    fr = h2o.H2OFrame(d, column_types={"g": "enum", "s": "enum"})
    kw = dict(stop_column="time")
    if strata:
        kw["stratify_by"] = ["s"]
    m = H2OCoxProportionalHazardsEstimator(**kw)
    m.train(x=["time", "x", "g", "s"] if strata else ["time", "x", "g"], y="event", training_frame=fr)
    assert abs(m._model.output["coefficients"]["x"] - 0.7) < 0.2
    path, a, b = _roundtrip(m, fr, tmp_path)
    mj = parse_mojo(path)
    ki = mj["info"]
    assert ki["algo"] == "coxph" and "coef" in ki and "x_mean_num" in mj["files"]
    assert int(ki["strata_count"]) == (2 if strata else 0)
    cols = mj["columns"]
    assert cols[: (2 if strata else 1)] == (["s", "g"] if strata else ["g"])
    assert np.allclose(a.values.astype(float), b.values.astype(float), atol=1e-5)
    # lp is centred per stratum (CoxPHModel.java:405 _lpBase[stratum]): mean 0 inside every stratum
    lp = a.values.astype(float).reshape(-1)
    groups = d["s"].values if strata else np.zeros(n)
    for gval in np.unique(groups):
        assert abs(float(lp[groups == gval].mean())) < 1e-6
    if strata:
        xm = np.frombuffer(mj["files"]["x_mean_num"], dtype=">f8")
        assert xm.size == 2 and xm[0] != xm[1]          # a real design-mean row per stratum


def test_coxph_rejects_na_strata():
    from h2o.estimators import H2OCoxProportionalHazardsEstimator
    h2o.init(verbose=False)
    d = pd.DataFrame({"time": [1.0, 2, 3, 4, 5, 6], "x": [0.1, 0.5, -0.2, 0.3, 1.0, -1.0],
                      "s": ["a", None, "b", "a", "b", "a"], "event": [1, 0, 1, 1, 0, 1]})
    fr = h2o.H2OFrame(d, column_types={"s": "enum"})
    m = H2OCoxProportionalHazardsEstimator(stop_column="time", stratify_by=["s"])
    with pytest.raises(Exception, match="missing"):
        m.train(x=["time", "x", "s"], y="event", training_frame=fr)


@pytest.mark.parametrize("y,blending", [("y", True), ("r", False), ("m", True)])
def test_target_encoder_mojo_reference_layout(df, tmp_path, y, blending):
    from h2o.estimators import H2OTargetEncoderEstimator
    te = H2OTargetEncoderEstimator(blending=blending, inflection_point=5, smoothing=3)
    te.train(x=["k", "m"] if y != "m" else ["k"], y=y, training_frame=df)
    path = te.download_mojo(str(tmp_path))
    mj = parse_mojo(path)
    f = mj["files"]
    assert mj["info"]["algo"] == "targetencoder"
    em = f["feature_engineering/target_encoding/encoding_map.ini"].decode()
    assert em.startswith("[k]\n0 = ")
    assert "[from]\nk\n[to]\n" in f["feature_engineering/target_encoding/input_output_columns_map.ini"].decode()
    g = h2o.import_mojo(path)
    a = te.transform(df).as_data_frame()
    b = g.transform(df).as_data_frame()
    tecols = [c for c in a.columns if c.endswith("_te")]
    assert tecols and list(b[tecols].columns) == tecols
    assert np.allclose(a[tecols].values.astype(float), b[tecols].values.astype(float), atol=1e-9)
