"""Wire compatibility: the UNMODIFIED h2o-py client of the reference snapshot
(``/root/reference/h2o-py``, pure Python) drives this framework's REST server over HTTP.

Covers the client paths a user hits first (reference ``h2o-py/h2o/h2o.py`` connect/import_file,
``estimator_base.py`` train/predict/model_performance, ``grid/grid_search.py``,
``automl/_estimator.py`` train + leaderboard/event-log fetch, ``expr.py`` Rapids ASTs). The
client is loaded from the reference tree in a subprocess so it never mixes with this repo's own
``h2o`` facade. Skipped when the reference tree is absent."""
import os
import socket
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest

REF = "/root/reference/h2o-py"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "h2o")), reason="reference h2o-py not present")

CLIENT = textwrap.dedent("""
    import sys
    sys.path.insert(0, %(ref)r)
    import h2o
    h2o.connect(url="http://127.0.0.1:%(port)d", verbose=False, strict_version_check=False)
    fr = h2o.import_file(%(csv)r)
    assert fr.nrow == 400 and fr.ncol == 6, fr.dim
    assert fr.types["cat"] == "enum" and fr["cat"].levels()[0] == ["a", "b", "c"]
    print("MEAN", fr["x0"].mean()[0])
    from h2o.estimators import (H2OGradientBoostingEstimator, H2OGeneralizedLinearEstimator,
                                H2ODeepLearningEstimator, H2OKMeansEstimator)
    m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1, nfolds=2)
    m.train(x=["x0", "x1", "x2", "cat"], y="yb", training_frame=fr)
    print("AUC", m.auc(), m.auc(xval=True))
    vi = m.varimp()
    assert vi[0][0] in ("x0", "x1", "x2", "cat")
    perf = m.model_performance(fr)
    cm = perf.confusion_matrix()
    assert cm is not None
    p = m.predict(fr)
    assert p.ncol == 3 and p.nrow == 400
    g = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0)
    g.train(x=["x0", "x1"], y="yr", training_frame=fr)
    print("COEF", g.coef()["x0"], g.coef()["x1"])
    dl = H2ODeepLearningEstimator(hidden=[16], epochs=10, seed=1, initial_weight_distribution="uniform_adaptive",
                                  activation="rectifier", missing_values_handling="mean_imputation")
    dl.train(x=["x0", "x1", "x2"], y="yr", training_frame=fr)
    print("DLRMSE", dl.rmse())
    dl2 = H2ODeepLearningEstimator(hidden=[8], epochs=1, seed=1, activation="tanh_with_dropout")
    dl2.train(x=["x0", "x1", "x2"], y="yb", training_frame=fr)
    assert dl2.logloss() > 0
    km = H2OKMeansEstimator(k=2, seed=1, init="plus_plus")
    km.train(x=["x0", "x1"], training_frame=fr)
    assert len(km.centers()) == 2
    tr, te = fr.split_frame([0.75], seed=1)
    assert tr.nrow + te.nrow == 400
    sub = fr[fr["x0"] > 0, ["x0", "cat"]]
    assert sub.ncol == 2 and 0 < sub.nrow < 400
    from h2o.grid import H2OGridSearch
    gs = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=2), hyper_params={"max_depth": [2, 3]})
    gs.train(x=["x0", "x1"], y="yb", training_frame=fr)
    assert len(gs.get_grid(sort_by="auc", decreasing=True).model_ids) == 2
    from h2o.automl import H2OAutoML
    aml = H2OAutoML(max_models=1, seed=1, nfolds=2, include_algos=["GLM"])
    aml.train(x=["x0", "x1", "x2"], y="yb", training_frame=fr)
    lb = aml.leaderboard
    assert lb.nrow >= 1 and "auc" in lb.columns, lb.columns
    print("DONE")
""")


CLIENT2 = textwrap.dedent("""
    import os, sys, tempfile
    sys.path.insert(0, %(ref)r)
    import h2o
    h2o.connect(url="http://127.0.0.1:%(port)d", verbose=False, strict_version_check=False)
    fr = h2o.import_file(%(csv)r)
    from h2o.estimators import H2OGradientBoostingEstimator, H2OGeneralizedLinearEstimator
    m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1)
    m.train(x=["x0", "x1", "x2", "cat"], y="yb", training_frame=fr)
    pdp = m.partial_plot(fr, cols=["x0", "cat"], plot=False, nbins=5)
    assert len(pdp) == 2 and pdp[0].col_header[0] == "x0" and len(pdp[0].cell_values) == 5
    assert [r[0] for r in pdp[1].cell_values] == ["a", "b", "c"]
    fi = m.feature_interaction()
    assert fi[0].col_header[:3] == ["Interaction", "Gain", "FScore"]
    assert 0 <= m.h(fr, ["x0", "x1"]) <= 1.5
    from h2o.tree import H2OTree
    t = H2OTree(m, 0)
    assert len(t) > 1 and t.root_node.split_feature in ("x0", "x1", "x2", "cat")
    g = H2OGeneralizedLinearEstimator(family="gaussian", lambda_search=True, nlambdas=5)
    g.train(x=["x0", "x1"], y="yr", training_frame=fr)
    rp = H2OGeneralizedLinearEstimator.getGLMRegularizationPath(g)
    assert len(rp["lambdas"]) == len(rp["coefficients"]) >= 1
    g2 = H2OGeneralizedLinearEstimator.makeGLMModel(g, rp["coefficients"][-1])
    assert abs(g2.coef()["x0"] - rp["coefficients"][-1]["x0"]) < 1e-9
    it = h2o.interaction(fr, ["cat", "yb"], pairwise=False, max_factors=10, min_occurrence=1)
    assert it.names == ["cat_yb"] and it.nrow == fr.nrow
    f2 = fr[["x0", "x1"]]
    f2.insert_missing_values(fraction=0.25, seed=1)
    assert 120 < sum(f2.nacnt()) < 280          # a quarter of the 800 cells
    d = tempfile.mkdtemp()
    assert os.path.getsize(m.download_mojo(d)) > 0
    m3 = h2o.upload_model(h2o.download_model(m, d))
    pred = m.predict(fr)
    assert abs(m3.predict(fr)["yes"].mean()[0] - pred["yes"].mean()[0]) < 1e-9
    mm = h2o.make_metrics(pred["yes"], fr["yb"], domain=["no", "yes"])
    assert abs(mm.auc() - m.model_performance(fr).auc()) < 1e-9
    pid = pred.frame_id
    assert pid in list(h2o.ls()["key"])
    h2o.remove(pred)
    assert pid not in list(h2o.ls()["key"])
    # munging pipelines: POST /99/Assembly and GET /99/Assembly.java (water/api/AssemblyHandler.java)
    from h2o.assembly import H2OAssembly
    from h2o.transforms.preprocessing import H2OBinaryOp, H2OColOp, H2OColSelect
    asm = H2OAssembly(steps=[("col_select", H2OColSelect(["x0", "x1", "cat"])),
                             ("cos_x0", H2OColOp(op=h2o.H2OFrame.cos, col="x0", inplace=True)),
                             ("cnt_cat", H2OColOp(op=h2o.H2OFrame.countmatches, col="cat", inplace=False, pattern="a")),
                             ("plus_x1", H2OBinaryOp(op=H2OAssembly.plus, col="x1", inplace=False, right=1.5))])
    res = asm.fit(fr)
    assert res.names == ["x0", "x1", "cat", "cat0", "x10"], res.names
    import math
    assert abs(res["x0"].max() - math.cos(fr["x0"].min())) < 1e-6 or res["x0"].max() <= 1.0
    assert abs((res["x10"] - res["x1"]).mean()[0] - 1.5) < 1e-9
    assert abs(res["cat0"].sum() - (fr["cat"] == "a").sum()) < 1e-9
    asm.to_pojo("MungePojo", d, get_jar=False)
    java = open(os.path.join(d, "MungePojo.java")).read()
    assert "public class MungePojo extends GenMunger" in java and "GenMunger.countmatches" in java, java[:400]
    print("DONE")
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data(tmp_path):
    rng = np.random.default_rng(3)
    n = 400
    X = rng.normal(size=(n, 3))
    cat = rng.choice(["a", "b", "c"], n)
    yb = np.where(X[:, 0] - X[:, 1] + rng.normal(size=n) * 0.5 > 0, "yes", "no")
    yr = 2.0 * X[:, 0] - 1.0 * X[:, 1] + rng.normal(size=n) * 0.1
    csv = tmp_path / "d.csv"
    with open(csv, "w") as f:
        f.write("x0,x1,x2,cat,yb,yr\n")
        for i in range(n):
            f.write(f"{X[i, 0]:.6f},{X[i, 1]:.6f},{X[i, 2]:.6f},{cat[i]},{yb[i]},{yr[i]:.6f}\n")
    return X, csv


def _run_client(tmp_path, client_src, csv):
    """Serve the REST app on a free localhost port, run ``client_src`` with the reference client,
    return its combined output (asserting a clean exit and the DONE marker)."""
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    log = open(tmp_path / "server.log", "w")
    srv = subprocess.Popen([sys.executable, "-m", "llama_github_io_amd.api.server", "--port", str(port)],
                           cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        t0 = time.time()
        while time.time() - t0 < 120:
            try:
                socket.create_connection(("127.0.0.1", port), timeout=1).close()
                break
            except OSError:
                time.sleep(0.5)
        script = tmp_path / "client.py"
        script.write_text(client_src % dict(ref=REF, port=port, csv=str(csv)))
        cenv = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
        r = subprocess.run([sys.executable, str(script)], cwd=str(tmp_path), env=cenv, capture_output=True,
                           text=True, timeout=600)
        out = r.stdout + r.stderr
        assert r.returncode == 0 and "DONE" in out, out[-4000:] + open(tmp_path / "server.log").read()[-3000:]
        return out
    finally:
        os.killpg(srv.pid, 15)
        srv.wait(timeout=30)
        log.close()


def test_reference_client_end_to_end(tmp_path):
    X, csv = _data(tmp_path)
    out = _run_client(tmp_path, CLIENT, csv)
    vals = {ln.split()[0]: [float(v) for v in ln.split()[1:]] for ln in out.splitlines()
            if ln.split() and ln.split()[0] in ("MEAN", "AUC", "COEF", "DLRMSE")}
    assert abs(vals["MEAN"][0] - X[:, 0].mean()) < 1e-5
    assert vals["AUC"][0] > 0.85 and vals["AUC"][1] > 0.8
    assert abs(vals["COEF"][0] - 2.0) < 0.05 and abs(vals["COEF"][1] + 1.0) < 0.05
    assert vals["DLRMSE"][0] < 0.6          # sd(yr) ~ 2.2: a mis-read enum spelling or a stalled net is far above


def test_reference_client_explain_persist_munging(tmp_path):
    """PartialDependence, FeatureInteraction, Friedman H, Tree, GLM regularization path / makeGLMModel,
    Interaction, MissingInserter, MOJO + binary model download/upload, make_metrics, remove."""
    _, csv = _data(tmp_path)
    _run_client(tmp_path, CLIENT2, csv)


def test_own_facade_connect_url(tmp_path):
    """``h2o.connect(url=...)`` of this repo's facade talks HTTP to a running server: cloud check,
    session, raw ``h2o.api`` import/parse, ``ls``, ``get_frame`` (local copy) and ``remove``."""
    _, csv = _data(tmp_path)
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    srv = subprocess.Popen([sys.executable, "-m", "llama_github_io_amd.api.server", "--port", str(port)],
                           cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)
    import h2o
    from h2o import _conn
    try:
        t0 = time.time()
        while time.time() - t0 < 120:
            try:
                socket.create_connection(("127.0.0.1", port), timeout=1).close()
                break
            except OSError:
                time.sleep(0.5)
        c = h2o.connect(url=f"http://127.0.0.1:{port}", verbose=False)
        assert isinstance(c, _conn.RemoteConnection) and h2o.cluster().cloud_size >= 1
        r = h2o.api("POST /3/ImportFiles", data={"path": str(csv)})
        ps = h2o.api("POST /3/ParseSetup", data={"source_frames": r["destination_frames"]})
        j = h2o.api("POST /3/Parse", data={"source_frames": r["destination_frames"], "destination_frame": "remote.hex",
                                           "column_names": ps["column_names"], "column_types": ps["column_types"],
                                           "separator": ps["separator"], "check_header": ps["check_header"]})
        key = j["job"]["key"]["name"]
        while h2o.api(f"GET /3/Jobs/{key}")["jobs"][0]["status"] not in ("DONE", "FAILED"):
            time.sleep(0.2)
        assert "remote.hex" in list(h2o.ls()["key"])
        fr = h2o.get_frame("remote.hex")
        assert fr.nrows == 400 and fr.ncols == 6
        h2o.remove("remote.hex")
        assert "remote.hex" not in list(h2o.ls()["key"])
    finally:
        _conn.set_current(None)
        os.killpg(srv.pid, 15)
        srv.wait(timeout=30)
