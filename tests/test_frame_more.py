"""The rest of the h2o-py H2OFrame surface (reference h2o-py/h2o/frame.py) against numpy/scipy/pandas."""
import ast
import math
import os

import numpy as np
import pytest
import scipy.special as sps


@pytest.fixture(scope="module")
def fr():
    import h2o
    h2o.init(verbose=False)
    return h2o.H2OFrame({"a": [0.1, 0.5, 0.9, float("nan"), 0.3], "b": [1.0, 2.0, 3.0, 4.0, 5.0],
                         "c": ["x", "y", "x", "z", "x"]}, column_types={"c": "enum"})


def _v(f):
    return f.as_data_frame().values.ravel().astype(float)


def test_every_reference_method_exists():
    ref = "/root/reference/h2o-py/h2o/frame.py"
    if not os.path.exists(ref):
        pytest.skip("reference not mounted")
    from llama_github_io_amd.frame import H2OFrame
    names = set()
    for n in ast.walk(ast.parse(open(ref).read())):
        if isinstance(n, ast.ClassDef) and n.name == "H2OFrame":
            names |= {b.name for b in n.body if isinstance(b, ast.FunctionDef) and not b.name.startswith("_")}
    inst = H2OFrame({"x": [1.0]})
    missing = sorted(m for m in names if not hasattr(inst, m))
    assert missing == [], missing


def test_special_functions(fr):
    a = np.array([0.1, 0.5, 0.9, np.nan, 0.3])
    b = np.arange(1, 6.0)
    np.testing.assert_allclose(_v(fr["a"].acos()), np.arccos(a), equal_nan=True)
    np.testing.assert_allclose(_v(fr["a"].atanh()), np.arctanh(a), equal_nan=True)
    np.testing.assert_allclose(_v(fr["b"].cospi()), np.cos(np.pi * b), atol=1e-12)
    np.testing.assert_allclose(_v(fr["b"].lgamma()), sps.gammaln(b))
    np.testing.assert_allclose(_v(fr["b"].digamma()), sps.digamma(b), rtol=1e-9)
    np.testing.assert_allclose(_v(fr["b"].trigamma()), sps.polygamma(1, b), rtol=1e-9)


def test_statistics(fr):
    b = np.arange(1, 6.0)
    assert fr["b"].prod() == pytest.approx(120.0)
    assert fr["b"].skewness()[0] == pytest.approx(0.0, abs=1e-12)
    k = ((b - b.mean()) ** 4).mean() / ((b - b.mean()) ** 2).mean() ** 2
    assert fr["b"].kurtosis()[0] == pytest.approx(k)
    assert _v(fr["b"].idxmax())[0] == 4 and _v(fr["b"].idxmin())[0] == 0
    assert fr.anyfactor() and fr["b"].any_na_rm() and fr.ischaracter() == [False, False, False]


def test_levels_and_matching(fr):
    c = fr["c"]
    assert c.categories() == ["x", "y", "z"]
    assert c.relevel_by_frequency().levels() == [["x", "y", "z"]]
    assert c.relevel_by_frequency(top_n=1).levels()[0][0] == "x"
    assert _v(c.isin(["y", "z"])).tolist() == [0, 1, 0, 1, 0]
    assert _v(c.match(["z", "x"])).tolist() == [2, 0, 2, 1, 2]
    assert c.append_levels(["w"]).levels()[0][-1] == "w"


def test_time_constructors():
    from llama_github_io_amd.frame import H2OFrame
    m = H2OFrame.moment(2020, 2, 29, 12, 30).as_data_frame().values[0, 0]
    assert str(m).startswith("2020-02-29T12:30")
    k = H2OFrame.mktime(2020, 1, 28).as_data_frame().values[0, 0]       # 0-based month and day
    assert str(k).startswith("2020-02-29")


def test_concat_rep_getrow_structure(fr, capsys):
    assert fr["a"].concat([fr["b"]], axis=1).ncols == 2
    assert fr["b"].rep_len(7).nrows == 7
    assert fr[0, :].getrow()[1] == 1.0
    fr.structure()
    assert "obs. of 3 variables" in capsys.readouterr().out


def test_frame_id_rename_refused_while_write_locked():
    """Renaming a frame a job holds write-locked fails and leaves exactly one live key (reference Rapids rename)."""
    import pytest
    from llama_github_io_amd.core import dkv
    from llama_github_io_amd.frame import H2OFrame
    fr = H2OFrame({"a": [1.0, 2.0]}, destination_frame="locked_src")
    with dkv.write_lock("locked_src"):
        with pytest.raises(RuntimeError):
            fr.frame_id = "locked_dst"
        assert fr.frame_id == "locked_src" and dkv.get("locked_src") is fr and not dkv.contains("locked_dst")
    fr.frame_id = "locked_dst"
    assert dkv.get("locked_dst") is fr and not dkv.contains("locked_src")


def test_impute_by_group_matches_pandas():
    """h2o.impute with groupByCols (AstImpute.java:205-257): NAs take their group's mean / median / mode; a group
    with no observed value keeps its NAs; NA keys are a group of their own."""
    import numpy as np
    import pandas as pd
    from llama_github_io_amd.frame import H2OFrame
    from llama_github_io_amd.rapids import rapids
    rng = np.random.default_rng(3)
    n = 300
    df = pd.DataFrame({"g": rng.choice(["a", "b", "c", None], n), "h": rng.integers(0, 3, n).astype(float),
                       "x": rng.normal(size=n), "e": rng.choice(["u", "v", "w"], n)})
    df.loc[rng.random(n) < 0.2, "x"] = np.nan
    df.loc[df.g == "c", "x"] = np.nan                                  # a group with nothing to impute from
    df.loc[rng.random(n) < 0.2, "e"] = None
    for method in ("mean", "median"):
        fr = H2OFrame(df.copy())
        fr.impute("x", method, by=["g", "h"])
        got = fr.as_data_frame()["x"].to_numpy()
        key = df.g.fillna("NA") + "|" + df.h.astype(str)
        agg = df.x.groupby(key).transform(method)
        want = df.x.fillna(agg).to_numpy()
        np.testing.assert_allclose(got, want, rtol=1e-12, equal_nan=True)
        assert np.isnan(got[(df.g == "c").to_numpy()]).all()
    fr = H2OFrame(df.copy())
    fr.impute("e", "mode", by=["h"])
    got = fr.as_data_frame()["e"]
    for hv in (0.0, 1.0, 2.0):
        m = (df.h == hv).to_numpy()
        mode = df.e[m].value_counts().sort_index().idxmax()             # ties: the smallest level, as torch.mode
        assert (got[m & df.e.isna().to_numpy()] == mode).all()
    # through Rapids (Flow's imputeColumn cell): column 2 by columns [0 1]
    fr = H2OFrame(df.copy(), destination_frame="imp_by")
    rapids('(h2o.impute imp_by 2 "mean" "interpolate" [0 1] _ _)')
    assert np.isnan(fr.as_data_frame()["x"].to_numpy()).sum() == int((df.g == "c").sum())
