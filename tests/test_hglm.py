"""HGLM (GLM HGLM=True, gaussian/gaussian random intercepts) against a direct mixed-model reference:
the converged fixed effects / random effects must satisfy Henderson's mixed-model equations at the
estimated variance components, and recover the simulated variance components."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGeneralizedLinearEstimator


@pytest.fixture(scope="module")
def data():
    h2o.init(verbose=False)
    rng = np.random.default_rng(11)
    G, n_per = 40, 60
    g = np.repeat(np.arange(G), n_per)
    u = rng.normal(0, 1.5, G)                       # sigma_u^2 = 2.25
    x = rng.normal(size=G * n_per)
    y = 1.0 + 2.0 * x + u[g] + rng.normal(0, 0.7, G * n_per)   # sigma_e^2 = 0.49
    d = pd.DataFrame({"x": x, "grp": [f"g{k:02d}" for k in g], "y": y})
    return h2o.H2OFrame(d, column_types={"grp": "enum"}), u


def test_hglm_recovers_components_and_satisfies_mme(data):
    fr, u_true = data
    m = H2OGeneralizedLinearEstimator(family="gaussian", HGLM=True, random_columns=["grp"], rand_family=["gaussian"],
                                      standardize=False)
    m.train(x=["x", "grp"], y="y", training_frame=fr)
    out = m._model.output
    assert out["converge"]
    assert out["coefficients"]["x"] == pytest.approx(2.0, abs=0.05)
    assert out["varfix"] == pytest.approx(0.49, rel=0.1)
    assert out["varranef"][0] == pytest.approx(2.25, rel=0.5)
    ub = np.array(out["ubeta"])
    assert np.corrcoef(ub, u_true)[0, 1] > 0.98
    # Henderson MME at the reported components: [X'X X'Z; Z'X Z'Z + lam I][b; u] = [X'y; Z'y]
    df = fr.as_data_frame()
    X = np.column_stack([df["x"].values, np.ones(len(df))])
    Z = pd.get_dummies(df["grp"]).values.astype(float)
    lam = out["varfix"] / out["varranef"][0]
    A = np.block([[X.T @ X, X.T @ Z], [Z.T @ X, Z.T @ Z + lam * np.eye(Z.shape[1])]])
    rhs = np.concatenate([X.T @ df["y"].values, Z.T @ df["y"].values])
    sol = np.linalg.solve(A, rhs)
    np.testing.assert_allclose(sol[:1], [out["coefficients"]["x"]], rtol=1e-6)
    np.testing.assert_allclose(sol[2:], ub, rtol=1e-5, atol=1e-8)
    # predictions include the random intercepts
    pred = m.predict(fr).as_data_frame().values[:, 0]
    np.testing.assert_allclose(pred, X @ sol[:2] + Z @ sol[2:], rtol=1e-5, atol=1e-5)
    assert set(m._model.coefs_random()) == {f"grp.g{k:02d}" for k in range(40)}
    assert np.isfinite(out["hlik"])


def test_hglm_requires_gaussian(data):
    fr, _ = data
    with pytest.raises(Exception):
        H2OGeneralizedLinearEstimator(family="poisson", HGLM=True, random_columns=["grp"]).train(
            x=["x", "grp"], y="y", training_frame=fr)


def test_hglm_rand_link_identity_accepted_others_refused(data):
    """GLMModel.java:534-548: rand_link may name identity / family_default per random column (the same model as the
    default); any other link, or a list of the wrong length, is refused with the reference's message."""
    fr, _ = data
    kw = dict(family="gaussian", HGLM=True, random_columns=["grp"], rand_family=["gaussian"], standardize=False)
    a = H2OGeneralizedLinearEstimator(**kw)
    a.train(x=["x", "grp"], y="y", training_frame=fr)
    b = H2OGeneralizedLinearEstimator(rand_link=["identity"], **kw)
    b.train(x=["x", "grp"], y="y", training_frame=fr)
    assert b._model.output["coefficients"]["x"] == pytest.approx(a._model.output["coefficients"]["x"], rel=1e-12)
    np.testing.assert_allclose(b._model.output["ubeta"], a._model.output["ubeta"], rtol=1e-12)
    with pytest.raises(Exception, match="identity link"):
        H2OGeneralizedLinearEstimator(rand_link=["log"], **kw).train(x=["x", "grp"], y="y", training_frame=fr)
    with pytest.raises(Exception, match="same length"):
        H2OGeneralizedLinearEstimator(rand_link=["identity", "identity"], **kw).train(x=["x", "grp"], y="y",
                                                                                         training_frame=fr)
