"""Explanations: TreeSHAP additivity (contributions + bias == raw margin), PDP, H statistic."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGradientBoostingEstimator, H2ORandomForestEstimator, H2OXGBoostEstimator


@pytest.fixture(scope="module")
def fr():
    h2o.init(verbose=False)
    rng = np.random.default_rng(0)
    n = 1500
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(list("xyz"), n)})
    df.loc[::13, "b"] = np.nan
    df["y"] = np.where(df.a + (df.c == "x") + rng.normal(size=n) * 0.3 > 0, "1", "0")
    df["r"] = df.a * 2 + np.nan_to_num(df.b) * df.a
    return h2o.H2OFrame(df, column_types={"y": "enum"})


@pytest.mark.parametrize("E,y", [(H2OGradientBoostingEstimator, "y"), (H2OGradientBoostingEstimator, "r"),
                                 (H2OXGBoostEstimator, "y"), (H2ORandomForestEstimator, "r")])
def test_shap_additivity(fr, E, y):
    m = E(ntrees=8, seed=1, max_depth=5)
    m.train(x=["a", "b", "c"], y=y, training_frame=fr)
    c = m.predict_contributions(fr).as_data_frame()
    assert list(c.columns) == ["a", "b", "c", "BiasTerm"]
    mm = m._model
    raw = mm.forest.predict_raw(fr.model_matrix(mm.info)[0])[:, 0].double().numpy()
    if mm.algo == "drf":
        raw = raw / mm.ntrees_built()
    else:
        init = mm.init_f[0] if isinstance(mm.init_f, (list, tuple)) else mm.init_f
        raw = raw + init
    assert np.abs(c.sum(1).values - raw).max() < 1e-5
    assert c["a"].abs().mean() > c["c"].abs().mean() * 0.5


def test_pdp_and_h(fr):
    m = H2OGradientBoostingEstimator(ntrees=10, seed=1, max_depth=4)
    m.train(x=["a", "b", "c"], y="r", training_frame=fr)
    p = m.partial_plot(fr, ["a"], nbins=6)["a"]
    means = [r["mean_response"] for r in p]
    assert means[-1] > means[0]                 # r increases with a
    hab = m.h(fr, ["a", "b"])
    assert 0 < hab <= 1.5                        # a*b interaction is real
    fi = m.feature_interaction()
    assert len(fi) >= 3 and list(fi[0].columns)[:3] == ["Interaction", "Gain", "FScore"]
    assert set(fi[0]["Interaction"]) <= {"a", "b", "c"} and (fi[1]["Interaction"].str.count("[|]") == 1).all()
    assert sorted(fi[0]["Gain Rank"]) == list(range(1, len(fi[0]) + 1))
    p2 = m.partial_plot(fr, [], nbins=4, col_pairs_2dpdp=[["a", "b"]])["a|b"]
    assert len(p2) == 16 and {"value", "value2", "mean_response"} <= set(p2[0])
    ice = m.partial_plot(fr, ["a"], nbins=5, row_index=3)["a"]
    assert len(ice) == 5 and all(r["stddev_response"] == 0 for r in ice)
