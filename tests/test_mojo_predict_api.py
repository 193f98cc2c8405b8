"""h2o.mojo_predict_csv / mojo_predict_pandas (reference h2o-py/h2o/utils/shared_utils.py:442-580, which drive
hex.genmodel.tools.PredictCsv in a JVM; here the native MOJO reader scores) and h2o.get_automl
(h2o-py/h2o/automl/autoh2o.py:13). Parity with the in-process model's predictions is the check."""
import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import H2OGradientBoostingEstimator


@pytest.fixture(scope="module")
def data():
    rng = np.random.default_rng(3)
    n = 600
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n),
                       "c": rng.choice(["x", "y", "z"], n)})
    df["y"] = np.where(df.a + (df.c == "y") + 0.3 * rng.normal(size=n) > 0.5, "yes", "no")
    return df


def test_mojo_predict_csv_and_pandas(data, tmp_path):
    fr = h2o.H2OFrame(data, column_types={"c": "enum", "y": "enum"})
    m = H2OGradientBoostingEstimator(ntrees=6, max_depth=3, seed=1)
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    ref = m.predict(fr).as_data_frame()
    inp = tmp_path / "in.csv"
    data[["a", "b", "c"]].to_csv(inp, index=False)
    rows = h2o.mojo_predict_csv(str(inp), path)
    assert (tmp_path / "prediction.csv").exists()
    assert list(rows[0].keys()) == list(ref.columns)
    assert [r["predict"] for r in rows] == list(ref["predict"].astype(str))
    assert np.allclose([float(r["yes"]) for r in rows], ref["yes"].to_numpy(), atol=1e-6)
    out = h2o.mojo_predict_pandas(data[["a", "b", "c"]], path)
    assert np.allclose(out["yes"].to_numpy(), ref["yes"].to_numpy(), atol=1e-6)
    contrib = h2o.mojo_predict_pandas(data[["a", "b", "c"]].head(20), path, predict_contributions=True)
    assert "BiasTerm" in contrib.columns


def test_mojo_predict_csv_invalid_numbers(data, tmp_path):
    fr = h2o.H2OFrame(data, column_types={"c": "enum", "y": "enum"})
    m = H2OGradientBoostingEstimator(ntrees=3, max_depth=2, seed=1)
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    bad = data[["a", "b", "c"]].head(5).astype({"a": object})
    bad.loc[2, "a"] = "oops"
    inp = tmp_path / "bad.csv"
    bad.to_csv(inp, index=False)
    with pytest.raises(ValueError):
        h2o.mojo_predict_csv(str(inp), path, str(tmp_path / "o.csv"))
    rows = h2o.mojo_predict_csv(str(inp), path, str(tmp_path / "o.csv"), setInvNumNA=True)
    assert len(rows) == 5
    with pytest.raises(RuntimeError):
        h2o.mojo_predict_csv(str(tmp_path / "missing.csv"), path)


def test_get_automl(data):
    from h2o.automl import H2OAutoML
    fr = h2o.H2OFrame(data, column_types={"c": "enum", "y": "enum"})
    aml = H2OAutoML(max_models=2, nfolds=0, seed=1, project_name="gaml_proj", include_algos=["GLM", "GBM"])
    aml.train(x=["a", "b", "c"], y="y", training_frame=fr)
    got = h2o.get_automl("gaml_proj")
    assert got.project_name == "gaml_proj"
    assert got.leader.model_id == aml.leader.model_id
    assert got.leaderboard.as_data_frame().shape == aml.leaderboard.as_data_frame().shape
    with pytest.raises(ValueError):
        h2o.get_automl("no_such_project")


def test_frame_id_setter_renames_dkv_entry():
    fr = h2o.H2OFrame(pd.DataFrame({"a": [1.0, 2.0, 3.0]}))
    old = fr.frame_id
    fr.frame_id = "renamed_frame_x"
    assert fr.frame_id == "renamed_frame_x"
    assert h2o.get_frame("renamed_frame_x") is not None
    assert old not in [str(k) for k in h2o.ls()["key"]]
