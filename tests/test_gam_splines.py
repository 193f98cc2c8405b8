"""GAM smoother families (reference hex/gam/GamSplines/*, MatrixFrameUtils/Gen*GamOneColumn.java):
cubic regression (bs=0), thin plate (bs=1, several columns), monotone I-splines (bs=2), M-splines
(bs=3), and categorical linear predictors."""
import numpy as np
import pandas as pd
import pytest
import torch


@pytest.fixture(scope="module")
def data():
    import h2o
    h2o.init(verbose=False)
    rng = np.random.default_rng(7)
    n = 800
    a = rng.uniform(-3, 3, n)
    b = rng.uniform(-2, 2, n)
    c = rng.choice(["u", "v", "w"], n)
    shift = np.select([c == "u", c == "v"], [0.0, 1.0], -1.0)
    y = np.sin(a) + 0.5 * b ** 2 + shift + rng.normal(size=n) * 0.1
    ym = np.tanh(a) * 2 + rng.normal(size=n) * 0.2                  # monotone in a
    fr = h2o.H2OFrame({"a": a.tolist(), "b": b.tolist(), "c": c.tolist(), "y": y.tolist(), "ym": ym.tolist()})
    fr["c"] = fr["c"].asfactor()
    return fr, a, b, shift


def test_cr_basis_is_cardinal_with_linear_null_space():
    from llama_github_io_amd.models.gam import _cr_mats, cr_basis
    knots = torch.tensor([0.0, 0.7, 1.5, 2.0, 3.3, 4.0], dtype=torch.float64)
    F, S = _cr_mats(knots)
    X = cr_basis(knots, knots, F)
    assert torch.allclose(X, torch.eye(6, dtype=torch.float64), atol=1e-12)    # beta = values at the knots
    assert torch.allclose(S @ torch.ones(6, dtype=torch.float64), torch.zeros(6, dtype=torch.float64), atol=1e-10)
    assert torch.allclose(S @ knots, torch.zeros(6, dtype=torch.float64), atol=1e-10)   # straight lines unpenalised


def test_cr_and_categorical_linear(data):
    from h2o.estimators import H2OGeneralizedAdditiveEstimator
    fr, a, b, shift = data
    m = H2OGeneralizedAdditiveEstimator(gam_columns=["a", "b"], num_knots=[8, 6], bs=[0, 0], family="gaussian")
    m.train(x=["c"], y="y", training_frame=fr)
    pred = m.predict(fr).as_data_frame()["predict"].values
    truth = np.sin(a) + 0.5 * b ** 2 + shift
    assert np.sqrt(np.mean((pred - truth - np.mean(pred - truth)) ** 2)) < 0.12


def test_thin_plate_two_columns(data):
    from h2o.estimators import H2OGeneralizedAdditiveEstimator
    fr, a, b, shift = data
    m = H2OGeneralizedAdditiveEstimator(gam_columns=[["a", "b"]], num_knots=[40], bs=[1], family="gaussian")
    m.train(x=["c"], y="y", training_frame=fr)
    pred = m.predict(fr).as_data_frame()["predict"].values
    truth = np.sin(a) + 0.5 * b ** 2 + shift
    assert np.corrcoef(pred, truth)[0, 1] > 0.97


def test_thin_plate_standardize_tp_gam_cols(data):
    """GAMModel._standardize_tp_gam_cols (GamUtilsThinPlateRegression: distances on sd-scaled coordinates): with one
    column on a 1000x larger scale the isotropic distance ignores the small column unless the columns are
    standardized, which recovers the fit."""
    import h2o
    from h2o.estimators import H2OGeneralizedAdditiveEstimator
    fr, a, b, shift = data
    fr2 = h2o.H2OFrame({"a": (a * 1000.0).tolist(), "b": b.tolist(), "y": (np.sin(a) + 0.5 * b ** 2).tolist()})
    preds = {}
    for flag in (False, True):
        m = H2OGeneralizedAdditiveEstimator(gam_columns=[["a", "b"]], num_knots=[40], bs=[1], family="gaussian",
                                            standardize_tp_gam_cols=flag)
        m.train(x=[], y="y", training_frame=fr2)
        preds[flag] = m.predict(fr2).as_data_frame()["predict"].values
    truth = np.sin(a) + 0.5 * b ** 2
    assert np.abs(preds[True] - preds[False]).max() > 1e-3
    assert np.corrcoef(preds[True], truth)[0, 1] > 0.97


def test_monotone_ispline(data):
    from h2o.estimators import H2OGeneralizedAdditiveEstimator
    import h2o
    fr, a, b, shift = data
    m = H2OGeneralizedAdditiveEstimator(gam_columns=["a"], num_knots=[8], bs=[2], spline_orders=[3], family="gaussian")
    m.train(x=[], y="ym", training_frame=fr)
    grid = np.linspace(-3, 3, 200)
    g = h2o.H2OFrame({"a": grid.tolist(), "b": [0.0] * 200, "c": ["u"] * 200}, column_types={"c": "enum"})
    p = m.predict(g).as_data_frame()["predict"].values
    assert (np.diff(p) >= -1e-9).all()                                   # non-negative coefficients: monotone
    assert np.corrcoef(p, np.tanh(grid) * 2)[0, 1] > 0.98


def test_mspline(data):
    from h2o.estimators import H2OGeneralizedAdditiveEstimator
    fr, a, b, shift = data
    m = H2OGeneralizedAdditiveEstimator(gam_columns=["a"], num_knots=[8], bs=[3], spline_orders=[3], family="gaussian")
    m.train(x=["c"], y="y", training_frame=fr)             # b**2 is left out: pred ~ sin(a) + shift + const
    pred = m.predict(fr).as_data_frame()["predict"].values
    assert np.corrcoef(pred, np.sin(a) + shift)[0, 1] > 0.95


def test_gam_passes_glm_options_through():
    """GAM's linear part honours the GLM options it shares (interactions, max_active_predictors,
    remove_collinear_columns, cold_start, objective_epsilon)."""
    import numpy as np
    import pandas as pd
    import h2o
    from h2o.estimators import H2OGeneralizedAdditiveEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(7)
    n = 2000
    d = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.normal(size=n)})
    d["c2"] = d["c"] * 2.0
    d["y"] = np.sin(d.a) + d.b * d.c + rng.normal(size=n) * 0.1
    fr = h2o.H2OFrame(d)
    base = dict(gam_columns=["a"], num_knots=[6], lambda_=0.0)
    m0 = H2OGeneralizedAdditiveEstimator(**base)
    m0.train(x=["a", "b", "c"], y="y", training_frame=fr)
    m1 = H2OGeneralizedAdditiveEstimator(interactions=["b", "c"], **base)
    m1.train(x=["a", "b", "c"], y="y", training_frame=fr)
    assert m1._model.output["training_metrics"]["MSE"] < 0.5 * m0._model.output["training_metrics"]["MSE"]
    m2 = H2OGeneralizedAdditiveEstimator(remove_collinear_columns=True, **base)
    m2.train(x=["a", "b", "c", "c2"], y="y", training_frame=fr)
    m3 = H2OGeneralizedAdditiveEstimator(cold_start=True, objective_epsilon=1e-6, **base)
    m3.train(x=["a", "b", "c"], y="y", training_frame=fr)


def test_gam_beta_constraints_prior_and_early_stopping():
    """GAM passes beta_constraints, prior and early_stopping to its GLM (GAM.java builds the GLM with the
    same parameters): a bounded linear coefficient is clipped, the prior moves the intercept, and early
    stopping shortens the lambda path."""
    import h2o
    from h2o.estimators import H2OGeneralizedAdditiveEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(4)
    n = 3000
    a, b = rng.normal(size=n), rng.uniform(-2, 2, n)
    yb = np.where(rng.random(n) < 1 / (1 + np.exp(-(1.5 * a + np.sin(2 * b)))), "1", "0")
    fr = h2o.H2OFrame(pd.DataFrame({"a": a, "b": b, "y": yb}))
    base = dict(family="binomial", gam_columns=["b"], num_knots=[6], lambda_=0.0)
    free = H2OGeneralizedAdditiveEstimator(**base)
    free.train(x=["a", "b"], y="y", training_frame=fr)
    assert free._model.output["coefficients"]["a"] > 1.0
    bc = h2o.H2OFrame(pd.DataFrame({"names": ["a"], "lower_bounds": [-10.0], "upper_bounds": [0.5]}))
    bounded = H2OGeneralizedAdditiveEstimator(beta_constraints=bc, **base)
    bounded.train(x=["a", "b"], y="y", training_frame=fr)
    assert abs(bounded._model.output["coefficients"]["a"] - 0.5) < 1e-6
    pr = H2OGeneralizedAdditiveEstimator(prior=0.2, **base)
    pr.train(x=["a", "b"], y="y", training_frame=fr)
    assert pr._model.output["coefficients"]["Intercept"] < free._model.output["coefficients"]["Intercept"] - 0.3
    ls = dict(family="binomial", gam_columns=["b"], num_knots=[6], lambda_search=True, nlambdas=40)
    es = H2OGeneralizedAdditiveEstimator(early_stopping=True, **ls)
    es.train(x=["a", "b"], y="y", training_frame=fr)
    noes = H2OGeneralizedAdditiveEstimator(early_stopping=False, **ls)
    noes.train(x=["a", "b"], y="y", training_frame=fr)
    assert len(noes._model.glm.output["lambda"]) == 40
    assert len(es._model.glm.output["lambda"]) <= 40


@pytest.mark.parametrize("family,bs", [("binomial", [0, 2]), ("gaussian", [3, 0])])
def test_gam_mojo_reference_layout_roundtrip(tmp_path, family, bs):
    """GAM MOJO in the GAMMojoWriter layout (model.ini keys, knots / zTranspose / _binvD blobs, sorted
    smoother order): the imported generic model reproduces the GAM's predictions."""
    import zipfile
    import h2o
    from h2o.estimators import H2OGeneralizedAdditiveEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(9)
    n = 1500
    a, b, c = rng.normal(size=n), rng.uniform(-2, 2, n), rng.uniform(0, 3, n)
    g = rng.choice(["u", "v", "w"], n)
    eta = 0.8 * a + np.sin(2 * b) + 0.3 * c ** 2 + (g == "v") * 0.5
    y = np.where(rng.random(n) < 1 / (1 + np.exp(-eta)), "1", "0") if family == "binomial" else eta + 0.2 * rng.normal(size=n)
    a[::37] = np.nan
    b[::41] = np.nan
    fr = h2o.H2OFrame(pd.DataFrame({"a": a, "b": b, "c": c, "g": g, "y": y}))
    m = H2OGeneralizedAdditiveEstimator(family=family, gam_columns=["b", "c"], bs=bs, num_knots=[6, 5],
                                        spline_orders=[3, 3], lambda_=1e-4)
    m.train(x=["a", "g", "b", "c"], y="y", training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    with zipfile.ZipFile(path) as z:
        names = set(z.namelist())
        ini = z.read("model.ini").decode()
    assert {"knots", "zTranspose", "gam_columns_sorted", "gamColNamesCenter", "_names_no_centering"} <= names
    assert "beta_center = " in ini and "bs_sorted = " in ini and "num_CS_col = 1" in ini
    gen = h2o.import_mojo(path)
    p1 = m.predict(fr).as_data_frame()
    p2 = gen.predict(fr).as_data_frame()
    col = "1" if family == "binomial" else "predict"
    assert np.allclose(p1[col].to_numpy(), p2[col].to_numpy(), atol=1e-6)
