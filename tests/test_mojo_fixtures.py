"""MOJO scoring parity against every fixture shipped with the reference genmodel tests
(``h2o-genmodel/src/test/resources/hex/genmodel/algos/*`` and the XGBoost extension's zips), with
the outputs the reference's own Java tests pin (``h2o-genmodel/src/test/java/hex/genmodel/algos/**``).
The fixture files are read as data (zip / ini / binary blobs); where a Java test pins numbers they
are asserted here, taken from the reference test source at run time when they are long tables.
Tests without pinned numbers in the reference say "parity unpinned" and check the documented
semantics instead. Skipped when the reference checkout is absent."""
import math
import os
import re
import tempfile
import zipfile

import numpy as np
import pytest
import torch

REF = "/root/reference"
ALG = os.path.join(REF, "h2o-genmodel/src/test/resources/hex/genmodel/algos")
JTEST = os.path.join(REF, "h2o-genmodel/src/test/java/hex/genmodel/algos")
XGB = os.path.join(REF, "h2o-genmodel-extensions/xgboost/src/test/resources/hex/genmodel/algos/xgboost")

pytestmark = pytest.mark.skipif(not os.path.isdir(ALG), reason="reference checkout not mounted")


def _zipdir(d):
    z = tempfile.mktemp(suffix=".zip")
    with zipfile.ZipFile(z, "w") as zf:
        for root, _, files in os.walk(d):
            for f in files:
                full = os.path.join(root, f)
                zf.write(full, os.path.relpath(full, d))
    return z


def _load(rel):
    import h2o
    p = os.path.join(ALG, rel)
    m = h2o.import_mojo(_zipdir(p) if os.path.isdir(p) else p)
    return getattr(m, "_model", m)


def _score0(m, rows):
    """genmodel ``score0`` input: raw doubles in model column order (categoricals = level index)."""
    X = torch.tensor(rows, dtype=torch.float64).T.contiguous().float()
    return m._predict_tensor(X, None).double()


def _predict_row(m, row: dict, types=None):
    import h2o
    import pandas as pd
    fr = h2o.H2OFrame(pd.DataFrame({k: [v] for k, v in row.items()}), column_types=types)
    return m.predict(fr).as_data_frame()


def _java_arrays(path, name):
    """``double[][] name = new double[][]{ new double[]{...}, ... };`` from a reference Java test."""
    src = open(path).read()
    block = re.search(r"double\[\]\[\]\s+" + name + r"\s*=\s*new double\[\]\[\]\s*\{(.*?)\};", src, re.S).group(1)
    rows = re.findall(r"new double\[\]\s*\{([^}]*)\}", block)
    conv = {"Double.NaN": "nan"}
    return [[float(conv.get(v.strip(), v.strip())) for v in r.split(",")] for r in rows]


# ---------------------------------------------------------------------------------- stacked ensembles
def test_se_binomial_pinned():
    # StackedEnsembleBinomialMojoTest.testPredictBinomialProstate
    m = _load("ensemble/binomial.zip")
    p = _predict_row(m, dict(AGE=65, RACE="1", DPROS=2, DCAPS=1, PSA=1.4, VOL=0, GLEASON=6), {"RACE": "enum"})
    assert str(p["predict"][0]) == "0"
    assert np.allclose(p[["0", "1"]].values[0], [0.8222695, 0.1777305], atol=1e-5)


def test_se_multinomial_pinned():
    m = _load("ensemble/multinomial.zip")
    p = _predict_row(m, dict(CAPSULE="0", AGE=65, DPROS=2, DCAPS=1, PSA=1.4, VOL=0, GLEASON=6), {"CAPSULE": "enum"})
    assert str(p["predict"][0]) == "1"
    assert np.allclose(p.iloc[0, 1:].values.astype(float), [0.006592327, 0.901237, 0.09217069], atol=1e-5)


def test_se_regression_pinned():
    m = _load("ensemble/regression.zip")
    p = _predict_row(m, dict(CAPSULE="0", RACE="1", DPROS=2, DCAPS=1, PSA=1.4, VOL=0, GLEASON=6),
                     {"CAPSULE": "enum", "RACE": "enum"})
    assert abs(p["predict"][0] - 66.29695) < 1e-5


def test_se_without_useless_base_models():
    # 27 base-model slots, only #6 present; missing columns of the row are NA
    m = _load("ensemble/binomial_without_useless_models.zip")
    assert len(m.base) == 27 and [i for i, b in enumerate(m.base) if b is not None] == [6]
    p = _predict_row(m, dict(AGE=65))
    assert str(p["predict"][0]) == "1"


def test_se_titanic_row_reordering():
    m = _load("ensemble/binomial_titanic.zip")
    row = {"pclass": 1.0, "survived": 1.0, "name": "Allison, Master. Hudson Trevor", "sex": "male", "age": 0.9167,
           "sibsp": 1.0, "parch": 2.0, "ticket": 113781.0, "fare": 151.55, "cabin": "C22 C26", "embarked": "S",
           "boat": 11.0, "body": float("nan"), "home.dest": "Montreal, PQ / Chesterville, ON"}
    types = {k: "enum" for k, v in row.items() if isinstance(v, str)}
    p = _predict_row(m, row, types)
    assert str(p["predict"][0]) != "" and abs(float(p.iloc[0, 1]) + float(p.iloc[0, 2]) - 1) < 1e-6


# ---------------------------------------------------------------------------------- tree models
def test_gbm_calibrated_pinned():
    # GbmMojoModelTest.testScore0 / testPredict: 2-class "multinomial" GBM with one tree per iteration,
    # Platt calibration
    m = _load("gbm/calibrated")
    row = [18.7, 1.51, 1.003, 132.53, 1.15, 0.2, 1.153, 8.3, 0.34, 0.0, 0.0]
    P = _score0(m, [row])[0]
    assert np.allclose(P.numpy(), [0.5416688, 0.4583312], atol=1e-5)
    cal = m._calibrated(P[None].float())
    assert np.allclose([float(cal._col("cal_p0").data[0]), float(cal._col("cal_p1").data[0])],
                       [0.3920402, 0.6079598], atol=1e-5)
    assert P[1] > m.default_threshold()           # label 1


def test_gbm_variable_importance_fixture_scores():
    m = _load("gbm/gbm_variable_importance.zip")        # parity unpinned: decodes and scores finite
    X = torch.zeros(m.info.F, 4)
    P = m._predict_tensor(X, None)
    assert torch.isfinite(P).all()


def test_isolation_forest_fixture():
    # IsolationForestMojoModelTest pins no numbers (leaf assignments only): parity unpinned. The score
    # follows IsolationForestMojoModel.unifyPreds: (max_path - sum) / (max_path - min_path), not clamped
    # (this far-out row scores above 1), and the mean length is sum / ntrees.
    m = _load("isofor")
    P = _score0(m, [[1, 2, 3, 4, 5, 6, 7, 8, 9]])[0]
    mn, mx = float(m.mojo_info["min_path_length"]), float(m.mojo_info["max_path_length"])
    tot = float(P[1]) * m.ntrees
    assert abs(float(P[0]) - (mx - tot) / (mx - mn)) < 1e-5 and P[1] > 0


def test_extended_isolation_forest_fixture():
    # ExtendedIsolationForestMojoModelTest: score = 2^(-mean path / c(sample_size)), zero-padded tree blobs
    m = _load("isoforextended")
    P = _score0(m, [[3.0, 3.0]])[0]
    n = 256
    c = 2 * (math.log(n - 1) + 0.5772156649) - 2 * (n - 1) / n
    assert abs(float(P[0]) - 2 ** (-float(P[1]) / c)) < 1e-4


@pytest.mark.parametrize("zname", ["xgboost.zip", "xgboost_java.zip"])
def test_xgboost_fixtures(zname):
    import h2o
    m = h2o.import_mojo(os.path.join(XGB, zname))
    m = getattr(m, "_model", m)
    if zname == "xgboost_java.zip":
        # XGBoostJavaMojoModelTest.testConvertWithWeights: root weight of tree 0 = 380 prostate rows
        assert m.forest.trees[0].cover[0] == 380
        prostate = h2o.import_file(os.path.join(REF, "h2o-py/h2o/h2o_data/prostate.csv"))
        pred = m.predict(prostate).as_data_frame()["predict"].values
        age = prostate["AGE"].as_data_frame()["AGE"].values
        assert np.corrcoef(pred, age)[0, 1] > 0.5            # a regression on AGE, fitted
    else:
        X = torch.zeros(m.info.F, 3)
        P = m._predict_tensor(X, None)
        assert P.shape == (3, len(m.info.response_domain)) and torch.allclose(P.sum(1), torch.ones(3), atol=1e-5)


# ---------------------------------------------------------------------------------- linear / clustering
def test_glm_prostate_pinned():
    # GlmMojoModelTest.testScore0 (MOJO 1.0 without an ``algo`` key; NA AGE mean-imputed)
    jt = os.path.join(JTEST, "glm/GlmMojoModelTest.java")
    data, exp = _java_arrays(jt, "data"), _java_arrays(jt, "expPreds")
    m = _load("glm/prostate")
    P = _score0(m, data).numpy()
    E = np.array(exp)
    assert np.abs(P - E[:, 1:]).max() < 1e-6
    thr = m.default_threshold()
    assert ((P[:, 1] >= thr).astype(float) == E[:, 0]).all()


def test_glm_multinomial_pinned():
    jt = os.path.join(JTEST, "glm/GlmMultinomialMojoModelTest.java")
    data, exp = _java_arrays(jt, "data"), _java_arrays(jt, "expPreds")
    m = _load("glm/multinomial")
    P = _score0(m, data).numpy()
    E = np.array(exp)
    assert np.abs(P - E[:, 1:]).max() < 1e-6
    assert (P.argmax(1) == E[:, 0]).all()


def test_kmeans_pinned():
    # KMeansMojoModelTest: rows 0..2 fall in clusters 0..2; distances follow GenModel.KMeans_distance
    # (standardised numerics, 0/1 categorical mismatch)
    m = _load("kmeans")
    rows = [[2.0, 1.0, 22.0, 1.0, 0.0], [2.0, 1.0, 2.0, 3.0, 1.0], [2.0, 0.0, 27.0, 0.0, 2.0]]
    assert _score0(m, rows).numpy().tolist() == [0.0, 1.0, 2.0]
    D = m.kmeans_distances(torch.tensor(rows).T.float()).numpy()
    for i, r in enumerate(rows):
        z = [r[0], r[1]] + [(r[j] - m.means[j]) * m.mults[j] for j in range(2, 5)]
        c = m.centers.numpy()
        exp = [sum((z[j] != c[k][j]) if j < 2 else (z[j] - c[k][j]) ** 2 for j in range(5)) for k in range(3)]
        assert np.allclose(D[i], exp, atol=1e-9)


def test_svm_pinned():
    # SvmMojoModelTest: zeros -> label 1, ones -> label 0
    m = _load("svm")
    P = _score0(m, [[0.0] * 6, [1.0] * 6])
    labels = (P[:, 1] > P[:, 0]).long().tolist()
    assert labels == [1, 0]


def test_glrm_row_data_and_factors():
    # GlrmMojoModelTest.testConvertUnseenEnumsToNA: an unseen level of a permuted categorical -> NaN.
    # The X factors themselves come from a seeded random start in the reference: parity unpinned; the
    # solved factors must reconstruct the numeric columns better than x = 0.
    from llama_github_io_amd.mojo import algos as A
    m = _load("glrm")
    st = m.glrm
    rows = [[0.0, 1.0, 5.0, 2.0, 741, 912, 5.0, 79.0, 82.0, 447.0, 1.0, 1.0],
            [0.0, 1.0, 9.0, 6.0, 729.0, 847.0, 5.0, 79.0, 82.0, 447.0, 0.0, -1],
            [0.0, 1.0, 10.0, 0.0, 749.0, 922.0, 5.0, 79.0, 82.0, 447.0, 1.0, 1.0]]
    perm, nlev = st["perm"], st["nlev"]
    for r in range(3):
        rows[r][perm[r]] = nlev[r] + 10.0
        a = A.glrm_row_data(st, torch.tensor([rows[r]]).T)[0]
        assert math.isnan(float(a[r]))
    x = A.score_glrm(st, torch.tensor([rows[0]]).T.float()).double()
    Y = st["Y"]
    nc = st["cat_off"][-1]
    nums = torch.tensor([rows[0][perm[i]] for i in range(st["ncats"], len(perm))], dtype=torch.float64)
    rec = (x @ Y)[0, nc:nc + st["nnums"]]
    assert ((rec - nums) ** 2).sum() < (nums ** 2).sum()


def test_word2vec_pinned():
    # Word2VecMojoModelTest.testTransform0
    m = _load("word2vec")
    w = m.inner
    assert w.vectors.shape[1] == 3
    assert np.allclose(w.vectors[w.vocab["a"]].numpy(), [0.0, 1.0, 0.2], atol=1e-4)
    assert np.allclose(w.vectors[w.vocab["b"]].numpy(), [1.0, 0.0, 0.8], atol=1e-4)
    assert "c" not in w.vocab


def test_pipeline_fixtures_load():
    # MojoPipelineBuilderTest inputs (kmeans + glm sub-models): parity unpinned, they decode and score
    import h2o
    for z in ("glm_model.zip", "kmeans_model.zip"):
        m = h2o.import_mojo(os.path.join(ALG, "pipeline", z))
        m = getattr(m, "_model", m)
        P = m._predict_tensor(torch.zeros(m.info.F, 2), None)
        assert P.shape[0] == 2


def test_glrm_mojo_reference_layout_roundtrip(tmp_path):
    """Our GLRM written in the GlrmMojoWriter layout reads back through the same reader that scores the
    reference fixture; the solved X factors reconstruct the (standardised) rows like the trained X."""
    import h2o
    from h2o.estimators import H2OGeneralizedLowRankEstimator
    from llama_github_io_amd.mojo.reader import parse_mojo
    h2o.init(verbose=False)
    rng = np.random.default_rng(5)
    n = 300
    U = rng.normal(size=(n, 2))
    V = rng.normal(size=(2, 4))
    A = U @ V + rng.normal(size=(n, 4)) * 0.01
    cat = np.where(U[:, 0] > 0, "hi", "lo")
    fr = h2o.H2OFrame({"x0": A[:, 0].tolist(), "x1": A[:, 1].tolist(), "x2": A[:, 2].tolist(),
                       "x3": A[:, 3].tolist(), "c": cat.tolist()}, column_types={"c": "enum"})
    m = H2OGeneralizedLowRankEstimator(k=3, transform="STANDARDIZE", seed=1, max_iterations=200)
    m.train(training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    mj = parse_mojo(path)
    assert mj["info"]["algo"] == "glrm" and "losses" in mj["files"] and "archetypes" in mj["files"]
    g = h2o.import_mojo(path)
    g = getattr(g, "_model", g)
    X, _ = fr.model_matrix(g.info)
    x = g._predict_tensor(X, None).double()                  # [n, k] factors
    st = g.glrm
    nc = st["cat_off"][-1]
    rec = (x @ st["Y"])[:, nc:]
    Z = (torch.tensor(A) - torch.tensor(st["norm_sub"])) * torch.tensor(st["norm_mul"])
    assert float(((rec - Z) ** 2).mean()) < 0.05
