"""GLM parameters that change the model (reference ``hex/glm/GLM.java``): ``checkpoint`` (IRLSM restart
from a previous model, GLM.java:1310-1318 / buildModel) and ``fix_tweedie_variance_power=False`` (ML
estimation of the Tweedie power and dispersion, GLM.java updateTweediePandPhi, GLMModel.java:725)."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGeneralizedLinearEstimator


@pytest.fixture(scope="module")
def bin_frame():
    h2o.init(verbose=False)
    rng = np.random.default_rng(11)
    n = 2000
    X = rng.normal(size=(n, 3))
    eta = 0.4 + X @ np.array([1.2, -0.8, 0.3])
    y = np.where(rng.random(n) < 1 / (1 + np.exp(-eta)), "1", "0")
    return h2o.H2OFrame(pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "y": y}))


def test_checkpoint_continues_irlsm(bin_frame):
    x = ["a", "b", "c"]
    full = H2OGeneralizedLinearEstimator(family="binomial", solver="IRLSM", lambda_=0.0, max_iterations=50, beta_epsilon=1e-8)
    full.train(x=x, y="y", training_frame=bin_frame)
    short = H2OGeneralizedLinearEstimator(family="binomial", solver="IRLSM", lambda_=0.0, max_iterations=1)
    short.train(x=x, y="y", training_frame=bin_frame)
    assert short._model.output["iterations"] == 1
    c0 = short.coef()
    assert abs(c0["a"] - full.coef()["a"]) > 1e-3            # one IRLS step is not converged
    cont = H2OGeneralizedLinearEstimator(family="binomial", solver="IRLSM", lambda_=0.0, max_iterations=50,
                                         beta_epsilon=1e-8, checkpoint=short.model_id)
    cont.train(x=x, y="y", training_frame=bin_frame)
    for k, v in full.coef().items():
        assert abs(cont.coef()[k] - v) < 1e-6
    assert cont._model.output["iterations"] > 1 and cont._model.output["checkpoint"] == short.model_id
    with pytest.raises(ValueError, match="IRLSM"):
        H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0, checkpoint=short.model_id).train(
            x=x, y="y", training_frame=bin_frame)
    with pytest.raises(ValueError, match="family"):
        H2OGeneralizedLinearEstimator(family="poisson", solver="IRLSM", checkpoint=short.model_id).train(
            x=["a", "b", "c"], y="a", training_frame=bin_frame)
    with pytest.raises(ValueError, match="max_iterations"):
        H2OGeneralizedLinearEstimator(family="binomial", solver="IRLSM", lambda_=0.0, max_iterations=1,
                                      checkpoint=short.model_id).train(x=x, y="y", training_frame=bin_frame)


def _tweedie_sample(rng, mu, phi, p):
    lam = mu ** (2 - p) / (phi * (2 - p))
    shape = (2 - p) / (p - 1)
    scale = phi * (p - 1) * mu ** (p - 1)
    n = rng.poisson(lam)
    return np.array([rng.gamma(shape, s, k).sum() if k else 0.0 for k, s in zip(n, scale)])


def test_tweedie_power_and_dispersion_estimated():
    h2o.init(verbose=False)
    rng = np.random.default_rng(5)
    n = 6000
    x = rng.normal(size=n)
    mu = np.exp(0.5 + 0.6 * x)
    y = _tweedie_sample(rng, mu, phi=1.5, p=1.4)
    fr = h2o.H2OFrame(pd.DataFrame({"x": x, "y": y}))
    m = H2OGeneralizedLinearEstimator(family="tweedie", link="tweedie", tweedie_variance_power=1.7, tweedie_link_power=0,
                                      lambda_=0.0, fix_tweedie_variance_power=False, dispersion_parameter_method="ml")
    m.train(x=["x"], y="y", training_frame=fr)
    o = m._model.output
    assert abs(o["tweedie_variance_power"] - 1.4) < 0.08, o["tweedie_variance_power"]
    assert abs(o["dispersion"] - 1.5) < 0.3, o["dispersion"]
    assert abs(m.coef()["x"] - 0.6) < 0.06
    fixed = H2OGeneralizedLinearEstimator(family="tweedie", link="tweedie", tweedie_variance_power=1.7,
                                          tweedie_link_power=0, lambda_=0.0)
    fixed.train(x=["x"], y="y", training_frame=fr)
    assert "tweedie_variance_power" not in fixed._model.output or fixed._model.output["tweedie_variance_power"] == 1.7
    with pytest.raises(ValueError, match="ml"):
        H2OGeneralizedLinearEstimator(family="tweedie", link="tweedie", tweedie_variance_power=1.5, tweedie_link_power=0,
                                      fix_tweedie_variance_power=False).train(x=["x"], y="y", training_frame=fr)


def test_modelselection_backward_p_values_threshold():
    """ModelSelection backward mode stops removing predictors once every p-value is <= p_values_threshold
    (ModelSelection.buildBackwardModels)."""
    from h2o.estimators import H2OModelSelectionEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(2)
    n = 1500
    X = rng.normal(size=(n, 5))
    y = 3 * X[:, 0] - 2 * X[:, 1] + 0.05 * X[:, 2] + rng.normal(size=n)
    fr = h2o.H2OFrame(pd.DataFrame({f"x{i}": X[:, i] for i in range(5)} | {"y": y}))
    full = H2OModelSelectionEstimator(mode="backward", min_predictor_number=1, family="gaussian")
    full.train(x=[f"x{i}" for i in range(5)], y="y", training_frame=fr)
    stop = H2OModelSelectionEstimator(mode="backward", min_predictor_number=1, family="gaussian", p_values_threshold=0.01)
    stop.train(x=[f"x{i}" for i in range(5)], y="y", training_frame=fr)
    sizes_full = [len(r["predictor_names"]) for r in full._model.output["result"]]
    sizes_stop = [len(r["predictor_names"]) for r in stop._model.output["result"]]
    assert min(sizes_full) == 1 and min(sizes_stop) == 2        # x0, x1 are both highly significant
    assert sorted(stop._model.output["result"][0]["predictor_names"]) == ["x0", "x1"]


def test_modelselection_and_anova_pass_glm_parameters():
    """ModelSelection / ANOVAGLM build their GLMs with the shared GLM parameters (beta_constraints, prior,
    remove_collinear_columns, ...); ANOVAGLM supports type 3 sums of squares only."""
    from h2o.estimators import H2OANOVAGLMEstimator, H2OModelSelectionEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(8)
    n = 1200
    X = rng.normal(size=(n, 3))
    y = 2 * X[:, 0] - X[:, 1] + rng.normal(size=n)
    fr = h2o.H2OFrame(pd.DataFrame({"x0": X[:, 0], "x1": X[:, 1], "x2": X[:, 2], "y": y}))
    bc = h2o.H2OFrame(pd.DataFrame({"names": ["x0"], "lower_bounds": [-5.0], "upper_bounds": [1.0]}))
    ms = H2OModelSelectionEstimator(mode="maxr", max_predictor_number=2, beta_constraints=bc)
    ms.train(x=["x0", "x1", "x2"], y="y", training_frame=fr)
    assert abs(ms._model.coef(2)["x0"] - 1.0) < 1e-6
    yb = np.where(rng.random(n) < 1 / (1 + np.exp(-X[:, 0])), "1", "0")
    frb = h2o.H2OFrame(pd.DataFrame({"x0": X[:, 0], "x1": X[:, 1], "y": yb}))
    a0 = H2OANOVAGLMEstimator(family="binomial", highest_interaction_term=1)
    a0.train(x=["x0", "x1"], y="y", training_frame=frb)
    a1 = H2OANOVAGLMEstimator(family="binomial", highest_interaction_term=1, prior=0.1)
    a1.train(x=["x0", "x1"], y="y", training_frame=frb)
    i0 = a0._model.full.output["coefficients"]["Intercept"]
    i1 = a1._model.full.output["coefficients"]["Intercept"]
    assert i1 < i0 - 1.0
    with pytest.raises(ValueError, match="type 3"):
        H2OANOVAGLMEstimator(family="binomial", type=1).train(x=["x0", "x1"], y="y", training_frame=frb)
