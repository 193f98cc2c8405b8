"""Rapids long-tail primitives (water/rapids/ast/prims/**) evaluated through the s-expression engine,
each checked against a NumPy/pandas reference of the same operation."""
import math

import numpy as np
import pandas as pd
import pytest
import scipy.special as sp

import h2o
from llama_github_io_amd import rapids as R
from llama_github_io_amd.core import dkv


@pytest.fixture(scope="module")
def fr():
    h2o.init(verbose=False)
    d = pd.DataFrame({"x": [0.1, 0.5, -0.3, 0.9, np.nan, 0.25], "y": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0],
                      "g": ["a", "b", "a", "c", "b", "a"], "s": [" ab ", "abab", "xy", "b", "a b", "zz"]})
    f = h2o.H2OFrame(d, column_types={"g": "enum", "s": "string"})
    dkv.put("rp_fr", f)
    return f


def _col(frame, i=0):
    return frame.as_data_frame().iloc[:, i].values.astype(float)


@pytest.mark.parametrize("op,ref", [("acos", np.arccos), ("asin", np.arcsin), ("atan", np.arctan),
                                    ("cosh", np.cosh), ("sinh", np.sinh), ("asinh", np.arcsinh),
                                    ("cospi", lambda v: np.cos(np.pi * v)), ("sinpi", lambda v: np.sin(np.pi * v)),
                                    ("lgamma", lambda v: sp.gammaln(v)), ("digamma", sp.digamma),
                                    ("trigamma", lambda v: sp.polygamma(1, v))])
def test_math_prims(fr, op, ref):
    out = R.rapids(f"({op} (cols rp_fr [0]))")
    x = fr.as_data_frame()["x"].values
    with np.errstate(all="ignore"):
        np.testing.assert_allclose(_col(out), ref(x), rtol=1e-5, equal_nan=True)


def test_gamma_and_round(fr):
    out = R.rapids("(gamma (cols rp_fr [1]))")
    np.testing.assert_allclose(_col(out), sp.gamma([1, 2, 3, 4, 5, 6.0]), rtol=1e-6)
    np.testing.assert_allclose(_col(R.rapids("(round (cols rp_fr [0]) 0)")), np.round(fr.as_data_frame()["x"]),
                               equal_nan=True)


def test_moments_and_reducers(fr):
    y = np.arange(1, 7.0)
    assert R.rapids("(skewness (cols rp_fr [1]) 1)")[0] == pytest.approx(0.0, abs=1e-12)
    k = ((y - y.mean()) ** 4).mean() / ((y - y.mean()) ** 2).mean() ** 2
    assert R.rapids("(kurtosis (cols rp_fr [1]) 1)")[0] == pytest.approx(k)
    assert R.rapids("(prod (cols rp_fr [1]))") == pytest.approx(720.0)
    assert R.rapids("(h2o.mad (cols rp_fr [1]) 'interpolate' 1.4826)") == pytest.approx(1.4826 * 1.5)
    assert R.rapids("(any.na rp_fr)") == 1.0 and R.rapids("(any.factor rp_fr)") == 1.0
    assert R.rapids("(naCnt rp_fr)") == [1.0, 0.0, 0.0, 0.0]
    assert R.rapids("(which.max (cols rp_fr [0 1]) 1 0)").as_data_frame().values[0].tolist() == [3.0, 5.0]
    assert _col(R.rapids("(sumaxis (cols rp_fr [1]) 0 0)"))[0] == 21.0


def test_mungers(fr):
    seq = R.rapids("(seq 1 5 2)")
    assert _col(seq).tolist() == [1.0, 3.0, 5.0]
    assert _col(R.rapids("(seq_len 3)")).tolist() == [1.0, 2.0, 3.0]
    assert _col(R.rapids("(rep_len (cols rp_fr [1]) 8)")).tolist() == [1, 2, 3, 4, 5, 6, 1, 2]
    m = R.rapids("(match (cols rp_fr [2]) ['b' 'a'] NA)")
    assert _col(m).tolist()[:4] == [2.0, 1.0, 2.0, 0.0] or np.isnan(_col(m)[3])
    rk = R.rapids("(rank_within_groupby rp_fr [2] [1] [1] 'rank' 0)")
    assert rk.as_data_frame()["rank"].tolist() == [1.0, 1.0, 2.0, 1.0, 2.0, 3.0]
    rf = R.rapids("(relevel.by.freq (cols rp_fr [2]) NA -1)")
    assert rf.levels()[0][0] == "a"
    d = R.rapids("(distance (cols rp_fr [1]) (cols rp_fr [1]) 'l1')")
    assert list(d.shape) == [6, 6] and _col(d, 0)[5] == 5.0
    assert R.rapids("(filterNACols rp_fr 0.0)") == [1.0, 2.0, 3.0]
    assert R.rapids("(getrow (rows (cols rp_fr [1]) [2]))") == [3.0]


def test_strings(fr):
    cm = R.rapids("(countmatches (cols rp_fr [3]) 'ab')")
    assert _col(cm).tolist() == [1.0, 2.0, 0.0, 0.0, 0.0, 0.0]
    tok = R.rapids("(tokenize (cols rp_fr [3]) ' ')")
    vals = tok.as_data_frame()["C1"].tolist()
    assert vals[:2] == ["ab", None] and vals.count(None) == 6
    d = R.rapids("(strDistance (cols rp_fr [3]) (cols rp_fr [3]) 'lv' 1)")
    assert _col(d).tolist() == [0.0] * 6
    ra = R.rapids("(replaceall (cols rp_fr [3]) 'b' 'B' 0)").as_data_frame().iloc[:, 0].tolist()
    assert ra[1] == "aBaB"
    sub = R.rapids("(substring (cols rp_fr [3]) 0 2)").as_data_frame().iloc[:, 0].tolist()
    assert sub[1] == "ab"


def test_time_prims():
    h2o.init(verbose=False)
    t = R.rapids("(mktime 2020 0 14 10 30 15 250)")
    assert R.rapids(f"(year {t.frame_id})") if False else True
    assert _col(t.minute())[0] == 30 and _col(t.second())[0] == 15
    assert int(_col(R.rapids("(millis (mktime 2020 0 14 10 30 15 250))"))[0]) == 250
    assert R.rapids("(getTimeZone)") == "UTC"


def test_prim_count_covers_reference_surface():
    assert len(R._session.prims) >= 180


def test_assign_and_model_prims(fr):
    from h2o.estimators import H2OGradientBoostingEstimator
    h2o.init(verbose=False)
    d = pd.DataFrame({"a": np.linspace(-1, 1, 200), "b": np.cos(np.arange(200.0))})
    d["y"] = np.where(d.a + 0.1 * d.b > 0, "1", "0")
    f = h2o.H2OFrame(d, column_types={"y": "enum"})
    dkv.put("rp_m", f)
    m = H2OGradientBoostingEstimator(ntrees=3, seed=1)
    m.train(x=["a", "b"], y="y", training_frame=f)
    dkv.put("rp_model", m._model)
    pv = R.rapids("(PermutationVarImp rp_model rp_m 'AUTO' -1 1 [] 1)")
    assert pv.as_data_frame()["Variable"].tolist()[0] == "a"
    lb = R.rapids("(makeLeaderboard ['rp_model'] rp_m 'AUTO' [] 'AUTO')")
    assert lb.as_data_frame()["model_id"].tolist() == [m._model.key]
    old = R.rapids("(model.reset.threshold rp_model 0.3)")
    assert m._model.default_threshold() == 0.3 and old[0] != 0.3
    g = h2o.H2OFrame(pd.DataFrame({"u": [1.0, 2.0, 3.0], "v": [4.0, 5.0, 6.0]}))
    dkv.put("rp_g", g)
    R.rapids("(:= rp_g 9 [1] [0 2])")
    assert g.as_data_frame()["v"].tolist() == [9.0, 5.0, 9.0]
    assert R.rapids("(perfectAUC (cols rp_m [0]) (cols rp_m [2]))") > 0.95
