"""Top-level h2o-py functions beyond estimators (reference: h2o-py/h2o/h2o.py): REST passthrough, SQL import,
grid save/load, timezone / expression-optimisation switches, logs, network test."""
import os
import sqlite3

import numpy as np
import pandas as pd
import pytest

import h2o


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2o.init(verbose=False)


def test_reference_surface_present():
    for name in ("api", "cluster_info", "connection", "demo", "download_all_logs", "download_csv",
                 "enable_expr_optimizations", "estimate_cluster_mem", "frame", "get_timezone", "import_frame",
                 "import_hive_table", "import_sql_select", "import_sql_table", "is_expr_optimizations_enabled",
                 "lazy_import", "list_timezones", "load_dataset", "load_grid", "log_and_echo", "models",
                 "network_test", "parse", "rapids", "save_grid", "set_timezone", "version_check"):
        assert callable(getattr(h2o, name)), name


def test_switches_and_estimates():
    h2o.set_timezone("America/Los_Angeles")
    assert h2o.get_timezone() == "America/Los_Angeles"
    h2o.set_timezone("UTC")
    h2o.enable_expr_optimizations(False)
    assert not h2o.is_expr_optimizations_enabled()
    h2o.enable_expr_optimizations(True)
    assert h2o.estimate_cluster_mem(10, 1_000_000) > h2o.estimate_cluster_mem(10, 1000)
    tz = h2o.list_timezones()
    assert tz.nrows > 100


def test_sql_import(tmp_path):
    db = str(tmp_path / "t.db")
    with sqlite3.connect(db) as con:
        con.execute("create table t (a real, b text, c integer)")
        con.executemany("insert into t values (?,?,?)", [(i * 0.5, "xy"[i % 2], i) for i in range(50)])
    fr = h2o.import_sql_table("jdbc:sqlite:" + db, "t", columns=["a", "c"])
    assert fr.nrows == 50 and fr.names == ["a", "c"]
    np.testing.assert_allclose(fr.as_data_frame()["a"].values, np.arange(50) * 0.5)
    sel = h2o.import_sql_select("jdbc:sqlite:" + db, "select c from t where c >= 40")
    assert sel.nrows == 10
    with pytest.raises(NotImplementedError):
        h2o.import_sql_table("jdbc:postgresql://x/db", "t")


def test_frame_models_rapids_api(tmp_path):
    df = pd.DataFrame({"x": np.arange(20.0), "y": np.arange(20.0) * 2})
    fr = h2o.H2OFrame(df)
    meta = h2o.frame(fr.frame_id)
    assert meta["frames"][0]["rows"] == 20
    out = h2o.api("GET /3/Cloud")
    assert isinstance(out, dict)
    p = h2o.download_csv(fr, str(tmp_path / "f.csv"))
    assert os.path.exists(p)
    assert str(tmp_path / "f.csv") in h2o.lazy_import(str(tmp_path), pattern=r"\.csv$")
    z = h2o.download_all_logs(str(tmp_path))
    assert z.endswith(".zip") and os.path.getsize(z) > 0
    rows = h2o.network_test()
    assert rows and rows[0]["ranks"] >= 1


def test_save_load_grid(tmp_path):
    from h2o.estimators import H2OGradientBoostingEstimator
    from h2o.grid import H2OGridSearch
    rng = np.random.default_rng(0)
    df = pd.DataFrame(rng.normal(size=(400, 3)), columns=list("abc"))
    df["y"] = df.a * 2 + rng.normal(0, 0.1, 400)
    fr = h2o.H2OFrame(df)
    gs = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=5), {"max_depth": [2, 3]}, grid_id="g_saved")
    gs.train(x=list("abc"), y="y", training_frame=fr)
    path = h2o.save_grid(str(tmp_path / "grid"), "g_saved")
    h2o.remove("g_saved")
    g2 = h2o.load_grid(path)
    assert len(g2.models) == 2
    pa = gs.models[0].predict(fr).as_data_frame().values
    pb = g2.models[0].predict(fr).as_data_frame().values
    np.testing.assert_allclose(pa, pb, rtol=1e-6)
