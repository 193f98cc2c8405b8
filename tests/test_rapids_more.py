"""Rapids lambdas / ddply / apply, iSAX, grouped_permute, fairness metrics, calibration, tree weight
updates, RuleFit rule predictions and the other remaining primitives (reference: water/rapids/ast/prims/**,
h2o-algos rapids prims, hex/tree/CalibrationHelper.java)."""
import numpy as np
import pandas as pd
import pytest
import torch

import h2o
from llama_github_io_amd.rapids import Session


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2o.init(verbose=False)


def _sess():
    return Session()


def test_ddply_lambda_and_apply():
    df = pd.DataFrame({"g": ["a", "b", "a", "b", "a"], "v": [1.0, 2.0, 3.0, 4.0, 5.0]})
    fr = h2o.H2OFrame(df, column_types={"g": "enum"}, destination_frame="dd")
    s = _sess()
    out = s.exec("(ddply dd [0] {x . (mean (cols x 1) TRUE)})").as_data_frame()
    assert list(out.columns) == ["g", "ddply_C1"]
    got = dict(zip(out["g"], out["ddply_C1"]))
    assert got == {"a": 3.0, "b": 3.0}
    out2 = s.exec("(ddply dd [0] {x . (sum (cols x 1) TRUE)})").as_data_frame()
    assert dict(zip(out2["g"], out2["ddply_C1"])) == {"a": 9.0, "b": 6.0}
    num = h2o.H2OFrame(pd.DataFrame({"a": [1.0, 2.0, 3.0], "b": [10.0, 20.0, 30.0]}), destination_frame="ap")
    col_sums = s.exec("(apply ap 2 {x . (sum x TRUE)})").as_data_frame().values.ravel()
    np.testing.assert_allclose(col_sums, [6.0, 60.0])
    assert s.exec("(%/% 7 2)") == 3.0


def test_isax():
    rng = np.random.default_rng(0)
    X = np.cumsum(rng.normal(size=(6, 32)), axis=1)
    fr = h2o.H2OFrame(pd.DataFrame(X, columns=[f"t{i}" for i in range(32)]), destination_frame="ts")
    out = _sess().exec("(isax ts 4 8 0)").as_data_frame()
    assert list(out.columns) == ["iSax_index", "c0", "c1", "c2", "c3"]
    # reference symbol: count of N(0,1) 1/8-quantiles below the z-scored segment mean
    from scipy.stats import norm
    seg = X.reshape(6, 4, 8)
    m = seg.mean(2)
    sd = np.sqrt(((seg - m[:, :, None]) ** 2).sum((1, 2)) / 31)
    z = (m - X.mean(1)[:, None]) / sd[:, None]
    sym = (norm.ppf(np.arange(1, 8) / 8)[None, None, :] < z[:, :, None]).sum(2)
    np.testing.assert_array_equal(out[["c0", "c1", "c2", "c3"]].values, sym)
    assert out["iSax_index"][0] == "_".join(f"{v}^8" for v in sym[0])


def test_grouped_permute():
    df = pd.DataFrame({"grp": [1, 1, 1, 2, 2], "id": [10, 11, 12, 20, 21], "kind": ["D", "C", "C", "D", "C"],
                       "amt": [1.0, 2.0, 3.0, 4.0, 5.0]})
    h2o.H2OFrame(df, column_types={"kind": "enum"}, destination_frame="gp")
    out = _sess().exec("(grouped_permute gp 1 [0] 2 3)").as_data_frame()
    assert list(out.columns) == ["grp", "In", "Out", "InAmnt", "OutAmnt"]
    rows = sorted(map(tuple, out.values.tolist()))
    assert rows == [(1, 10, 11, 1.0, 2.0), (1, 10, 12, 1.0, 3.0), (2, 20, 21, 4.0, 5.0)]


@pytest.fixture(scope="module")
def binom_frame():
    rng = np.random.default_rng(1)
    n = 3000
    df = pd.DataFrame(rng.normal(size=(n, 3)), columns=list("abc"))
    df["grp"] = rng.choice(["m", "f", "x"], n)
    logit = df.a - df.b + (df.grp == "m") * 0.5
    df["y"] = np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "yes", "no")
    return h2o.H2OFrame(df, column_types={"grp": "enum", "y": "enum"}, destination_frame="fair")


def test_fairness_metrics(binom_frame):
    from h2o.estimators import H2OGradientBoostingEstimator
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1, model_id="fair_gbm")
    m.train(x=["a", "b", "c", "grp"], y="y", training_frame=binom_frame)
    res = m.fairness_metrics(binom_frame, ["grp"], ["m"], "yes")
    ov = res["overview"].as_data_frame()
    assert set(ov["grp"]) == {"m", "f", "x"}
    row = ov[ov.grp == "m"].iloc[0]
    assert row["AIR_selectedRatio"] == pytest.approx(1.0)
    assert row["total"] + ov[ov.grp != "m"]["total"].sum() == binom_frame.nrows
    for _, r in ov.iterrows():
        assert r["accuracy"] == pytest.approx((r["tp"] + r["tn"]) / r["total"])
        assert 0 <= r["p.value"] <= 1
    s = _sess()
    ov2 = s.exec('(fairnessMetrics fair_gbm fair ["grp"] ["m"] "yes")')["overview"].as_data_frame()
    np.testing.assert_allclose(ov2["auc"].values, ov["auc"].values)
    pred = m.predict(binom_frame)
    h2o.assign(pred[:, [2]], "fair_pred")
    pv = s.exec('(predicted.vs.actual.by.var fair_gbm fair "grp" fair_pred)').as_data_frame()
    assert pv.shape == (4, 3) and list(pv.columns) == ["grp", "yes", "actual"]
    df = binom_frame.as_data_frame()
    p1 = pred.as_data_frame()["yes"].values
    for lvl in ("m", "f", "x"):
        r = pv[pv.grp == lvl].iloc[0]
        assert r["yes"] == pytest.approx(p1[df.grp.values == lvl].mean(), rel=1e-6)
        assert r["actual"] == pytest.approx((df.y.values[df.grp.values == lvl] == "yes").mean(), rel=1e-6)


def test_calibration_platt_and_isotonic(binom_frame, tmp_path):
    from h2o.estimators import H2OGradientBoostingEstimator
    for method in ("PlattScaling", "IsotonicRegression"):
        m = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1, calibrate_model=True,
                                         calibration_frame=binom_frame, calibration_method=method)
        m.train(x=["a", "b", "c", "grp"], y="y", training_frame=binom_frame)
        p = m.predict(binom_frame).as_data_frame()
        assert list(p.columns)[-2:] == ["cal_p0", "cal_p1"]
        np.testing.assert_allclose(p.cal_p0 + p.cal_p1, 1.0, atol=1e-6)
        if method == "IsotonicRegression":       # monotone in p1
            o = np.argsort(p.yes.values, kind="stable")
            assert np.all(np.diff(p.cal_p1.values[o]) >= -1e-9)
        else:                                    # logistic in p0: monotone decreasing in p0
            o = np.argsort(p.no.values, kind="stable")
            assert np.all(np.diff(p.cal_p1.values[o]) <= 1e-9)
        path = h2o.save_model(m, str(tmp_path), force=True)
        m2 = h2o.load_model(path)
        p2 = m2.predict(binom_frame).as_data_frame()
        np.testing.assert_allclose(p2.cal_p1.values, p.cal_p1.values, rtol=1e-6)
        mojo = m.download_mojo(str(tmp_path))
        g = h2o.import_mojo(mojo)
        pg = g.predict(binom_frame).as_data_frame()
        np.testing.assert_allclose(pg.cal_p1.values, p.cal_p1.values, atol=1e-5)


def test_tree_update_weights_and_rules(binom_frame):
    from h2o.estimators import H2OGradientBoostingEstimator, H2ORuleFitEstimator
    df = binom_frame.as_data_frame()
    df["w"] = 2.0
    fr = h2o.H2OFrame(df, column_types={"grp": "enum", "y": "enum"})
    m = H2OGradientBoostingEstimator(ntrees=3, max_depth=2, seed=1, model_id="tw_gbm")
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    assert m.update_tree_weights(fr, "w") == "OK"
    t0 = m._model.forest.trees[0]
    assert t0.cover[0] == pytest.approx(2.0 * fr.nrows)
    assert all(abs(t0.cover[i] - t0.cover[t0.left[i]] - t0.cover[t0.right[i]]) < 1e-6
               for i in range(t0.n_nodes) if t0.feat[i] >= 0)
    rf = H2ORuleFitEstimator(max_rule_length=2, min_rule_length=1, rule_generation_ntrees=4, seed=1, model_id="rf_m")
    rf.train(x=["a", "b", "c"], y="y", training_frame=fr)
    ids = [r["variable"] for r in rf.rule_importance() if not r["variable"].startswith("linear.")][:3]
    pr = rf.predict_rules(fr, ids).as_data_frame()
    assert list(pr.columns) == ids
    assert set(np.unique(pr.values)) <= {0, 1}


def test_misc_prims(tmp_path):
    s = _sess()
    h2o.H2OFrame(pd.DataFrame({"x": [1.0, 2, 3, 4, 5], "y": [1.0, 3, 2, 4, 6]}), destination_frame="pv")
    out = s.exec("(isotonic.pav pv)").as_data_frame()
    assert np.all(np.diff(out["Y"].values) >= 0)
    assert s.exec('(testing.setreadforbidden ["a"])') == "OK"
    fr = h2o.H2OFrame(pd.DataFrame({"a": [1.0, 2.0, 3.0]}), destination_frame="si")
    s.exec("(scale_inplace si 1 1)")
    assert abs(fr.as_data_frame()["a"].mean()) < 1e-9
