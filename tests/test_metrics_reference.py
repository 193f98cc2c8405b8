"""Metrics and core algorithms against independent references (scikit-learn / NumPy / SciPy), the
CPU counterpart of the reference's AUC2Test / ConfusionMatrixTest / GainsLiftTest / GLMTest / KMeansTest /
PCATest suites. H2O's AUC uses 400 threshold bins (AUC2.java), so AUC agreement is to ~1e-3."""
import numpy as np
import pytest
import torch
from sklearn import metrics as skm

from llama_github_io_amd import metrics as mm


@pytest.fixture(scope="module")
def binom():
    rng = np.random.default_rng(0)
    n = 5000
    y = (rng.random(n) < 0.35).astype(np.float64)
    p = np.clip(0.25 + 0.4 * y + rng.normal(0, 0.2, n), 0.001, 0.999)
    w = rng.uniform(0.5, 2.0, n)
    return y, p, w


def test_binomial_auc_logloss_mse(binom):
    y, p, _ = binom
    m = mm.binomial_metrics(torch.tensor(y), torch.tensor(p), None, ["0", "1"])
    assert m["AUC"] == pytest.approx(skm.roc_auc_score(y, p), abs=2e-3)
    assert m["Gini"] == pytest.approx(2 * m["AUC"] - 1, abs=1e-12)
    assert m["logloss"] == pytest.approx(skm.log_loss(y, p), rel=1e-9)
    assert m["MSE"] == pytest.approx(np.mean((y - p) ** 2), rel=1e-9)
    assert m["pr_auc"] == pytest.approx(skm.average_precision_score(y, p), abs=2e-2)


def test_binomial_weighted(binom):
    y, p, w = binom
    m = mm.binomial_metrics(torch.tensor(y), torch.tensor(p), torch.tensor(w), ["0", "1"])
    assert m["logloss"] == pytest.approx(skm.log_loss(y, p, sample_weight=w), rel=1e-9)
    assert m["AUC"] == pytest.approx(skm.roc_auc_score(y, p, sample_weight=w), abs=2e-3)


def test_confusion_matrix_at_max_f1(binom):
    y, p, _ = binom
    m = mm.binomial_metrics(torch.tensor(y), torch.tensor(p), None, ["0", "1"])
    thr = m["max_f1_threshold"]
    pred = (p >= thr).astype(int)
    cm = skm.confusion_matrix(y.astype(int), pred)
    ours = np.asarray(m["cm"]["table"] if isinstance(m["cm"], dict) and "table" in m["cm"] else m["cm"])
    assert ours.shape[0] >= 2
    assert np.array_equal(np.asarray(ours)[:2, :2].astype(int), cm)
    best_f1 = max(skm.f1_score(y, (p >= t).astype(int)) for t in np.unique(np.round(p, 3)))
    assert skm.f1_score(y, pred) == pytest.approx(best_f1, abs=1e-2)


def test_gains_lift_table(binom):
    y, p, _ = binom
    m = mm.binomial_metrics(torch.tensor(y), torch.tensor(p), None, ["0", "1"])
    gl = m["gains_lift_table"]
    rows = gl if isinstance(gl, list) else gl.get("rows", gl)
    cum_cap = [r["cumulative_capture_rate"] for r in rows] if isinstance(rows, list) and isinstance(rows[0], dict) \
        else list(np.asarray(gl["cumulative_capture_rate"]))
    assert cum_cap[-1] == pytest.approx(1.0, abs=1e-9)
    assert all(b >= a - 1e-12 for a, b in zip(cum_cap, cum_cap[1:]))


def test_regression_metrics():
    rng = np.random.default_rng(1)
    y = rng.gamma(2.0, 2.0, 3000)
    p = y + rng.normal(0, 0.5, 3000)
    p = np.abs(p)
    m = mm.regression_metrics(torch.tensor(y), torch.tensor(p), None, None)
    assert m["MSE"] == pytest.approx(skm.mean_squared_error(y, p), rel=1e-9)
    assert m["mae"] == pytest.approx(skm.mean_absolute_error(y, p), rel=1e-9)
    assert m["r2"] == pytest.approx(skm.r2_score(y, p), rel=1e-6)
    assert m["rmsle"] == pytest.approx(np.sqrt(skm.mean_squared_log_error(y, p)), rel=1e-6)


def test_multinomial_metrics():
    rng = np.random.default_rng(2)
    n, K = 4000, 4
    y = rng.integers(0, K, n)
    logits = rng.normal(size=(n, K))
    logits[np.arange(n), y] += 1.5
    P = np.exp(logits) / np.exp(logits).sum(1, keepdims=True)
    m = mm.multinomial_metrics(torch.tensor(y, dtype=torch.float64), torch.tensor(P), None, list("abcd"))
    assert m["logloss"] == pytest.approx(skm.log_loss(y, P), rel=1e-9)
    pred = P.argmax(1)
    per_class_err = np.mean([np.mean(pred[y == k] != k) for k in range(K)])
    assert m["mean_per_class_error"] == pytest.approx(per_class_err, abs=1e-9)
    hr = m["hit_ratio_table"]
    top1 = hr[0]["hit_ratio"] if isinstance(hr, list) and isinstance(hr[0], dict) else hr[0]
    assert top1 == pytest.approx(np.mean(pred == y), abs=1e-9)


# ------------------------------------------------------------------------------------------------ algorithms
def test_glm_gaussian_and_binomial_match_sklearn():
    from sklearn.linear_model import LogisticRegression
    import h2o
    import pandas as pd
    from h2o.estimators import H2OGeneralizedLinearEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(3)
    n = 3000
    X = rng.normal(size=(n, 4))
    yr = X @ np.array([1.0, -2.0, 0.5, 0.0]) + 0.3 + rng.normal(0, 0.1, n)
    yb = (rng.random(n) < 1 / (1 + np.exp(-(X @ np.array([1.0, -1.0, 0.5, 0.2]))))).astype(int)
    df = pd.DataFrame(X, columns=list("abcd"))
    df["yr"], df["yb"] = yr, yb.astype(str)
    fr = h2o.H2OFrame(df, column_types={"yb": "enum"})
    g = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0, standardize=False)
    g.train(x=list("abcd"), y="yr", training_frame=fr)
    A = np.column_stack([X, np.ones(n)])
    ols = np.linalg.lstsq(A, yr, rcond=None)[0]
    c = g.coef()
    np.testing.assert_allclose([c["a"], c["b"], c["c"], c["d"], c["Intercept"]], ols, rtol=1e-5, atol=1e-6)
    b = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0)
    b.train(x=list("abcd"), y="yb", training_frame=fr)
    sk = LogisticRegression(C=1e12, max_iter=2000, tol=1e-10).fit(X, yb)
    cb = b.coef()
    np.testing.assert_allclose([cb["a"], cb["b"], cb["c"], cb["d"]], sk.coef_[0], rtol=2e-3, atol=2e-3)
    assert cb["Intercept"] == pytest.approx(sk.intercept_[0], abs=2e-3)


def test_kmeans_matches_sklearn_objective():
    from sklearn.cluster import KMeans
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.kmeans import KMeansTrainer
    rng = np.random.default_rng(4)
    centers = np.array([[0, 0], [5, 5], [0, 6], [7, 0]], dtype=float)
    X = np.concatenate([c + rng.normal(0, 0.5, (500, 2)) for c in centers])
    info = DataInfo(["x0", "x1"], np.zeros(2, np.int32), [None, None], None, None)
    m = KMeansTrainer(dict(k=4, seed=1, standardize=False, init="PlusPlus")).fit(
        torch.tensor(X.T, dtype=torch.float32), None, None, None, info)
    sk = KMeans(4, n_init=10, random_state=0).fit(X)
    ours = m.output["training_metrics"]["tot_withinss"]
    assert ours == pytest.approx(sk.inertia_, rel=1e-3)


def test_pca_matches_numpy_svd():
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.pca import PCATrainer
    rng = np.random.default_rng(5)
    X = rng.normal(size=(800, 5)) @ rng.normal(size=(5, 5))
    info = DataInfo([f"x{i}" for i in range(5)], np.zeros(5, np.int32), [None] * 5, None, None)
    m = PCATrainer(dict(k=3, transform="DEMEAN")).fit(torch.tensor(X.T, dtype=torch.float32), None, None, None, info)
    Xc = X - X.mean(0)
    _, s, Vt = np.linalg.svd(Xc, full_matrices=False)
    V = m.V.double().cpu().numpy()
    for j in range(3):                              # eigenvectors up to sign
        assert abs(abs(float(V[:, j] @ Vt[j])) - 1.0) < 1e-4
    sd = np.asarray(m.output["importance"]["standard_deviation"][:3]) if isinstance(m.output["importance"], dict) \
        else None
    if sd is not None:
        np.testing.assert_allclose(sd, s[:3] / np.sqrt(len(X) - 1), rtol=1e-4)


def test_naive_bayes_matches_sklearn():
    from sklearn.naive_bayes import GaussianNB
    import h2o
    import pandas as pd
    from h2o.estimators import H2ONaiveBayesEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(6)
    n = 2000
    y = rng.integers(0, 2, n)
    X = rng.normal(size=(n, 3)) + y[:, None] * np.array([1.0, -0.5, 0.2])
    df = pd.DataFrame(X, columns=list("abc"))
    df["y"] = y.astype(str)
    fr = h2o.H2OFrame(df, column_types={"y": "enum"})
    nb = H2ONaiveBayesEstimator()
    nb.train(x=list("abc"), y="y", training_frame=fr)
    ours = nb.predict(fr).as_data_frame()["1"].values
    sk = GaussianNB(var_smoothing=0).fit(X, y).predict_proba(X)[:, 1]
    # H2O uses the unbiased (n-1) variance; sklearn the biased one: agreement to a few 1e-3
    np.testing.assert_allclose(ours, sk, atol=5e-3)


def test_lattice_threshold_table_tracks_exact_scores(binom):
    """The threshold table / max-F1 threshold come from the 2^18-bin score lattice in every process layout
    (identical single vs sharded). Thresholds are bin maxima, so the criteria sit within one lattice bin of
    the exact distinct-score optimum (parity with AUC2's 400 merging bins is unpinned: no reference fixture)."""
    y, p, _ = binom
    m = mm.binomial_metrics(torch.tensor(y), torch.tensor(p), None, ["0", "1"])
    order = np.argsort(-p, kind="stable")
    ps, ys = p[order], y[order]
    tp, fp = np.cumsum(ys), np.cumsum(1 - ys)
    last = np.r_[ps[1:] != ps[:-1], True]                   # one point per distinct score
    f1 = 2 * tp[last] / (tp[last] + fp[last] + ys.sum())
    best = float(f1.max())
    row = max(m["thresholds_and_metric_scores"], key=lambda r: r["f1"])
    assert row["f1"] == pytest.approx(best, abs=2e-3)
    assert abs(m["max_f1_threshold"] - float(ps[last][f1.argmax()])) < 0.02
    # every reported threshold is an observed score
    assert all(np.any(np.isclose(p, r["threshold"], rtol=0, atol=1e-12)) for r in m["thresholds_and_metric_scores"])


def test_lattice_auc_for_large_frames_is_close_to_exact(monkeypatch):
    """Frames of >= LATTICE_AUC_ROWS rows take AUC from the 2^18-bin score lattice (no full sort)."""
    import numpy as np
    import sklearn.metrics as skm
    import torch
    from llama_github_io_amd import metrics as M
    rng = np.random.default_rng(3)
    n = 200_000
    p = rng.random(n)
    y = (rng.random(n) < p).astype(np.float64)
    monkeypatch.setattr(M, "LATTICE_AUC_ROWS", 1000)
    m = M.binomial_metrics(torch.tensor(y), torch.tensor(p))
    assert abs(m["AUC"] - skm.roc_auc_score(y, p)) < 1e-5
    assert abs(m["pr_auc"] - skm.average_precision_score(y, p)) < 2e-3
