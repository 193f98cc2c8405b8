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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_reference_client_end_to_end(tmp_path):
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
        script.write_text(CLIENT % dict(ref=REF, port=port, csv=str(csv)))
        cenv = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
        r = subprocess.run([sys.executable, str(script)], cwd=str(tmp_path), env=cenv, capture_output=True,
                           text=True, timeout=600)
        out = r.stdout + r.stderr
        assert r.returncode == 0 and "DONE" in out, out[-4000:] + open(tmp_path / "server.log").read()[-3000:]
        vals = {ln.split()[0]: [float(v) for v in ln.split()[1:]] for ln in out.splitlines()
                if ln.split() and ln.split()[0] in ("MEAN", "AUC", "COEF", "DLRMSE")}
        assert abs(vals["MEAN"][0] - X[:, 0].mean()) < 1e-5
        assert vals["AUC"][0] > 0.85 and vals["AUC"][1] > 0.8
        assert abs(vals["COEF"][0] - 2.0) < 0.05 and abs(vals["COEF"][1] + 1.0) < 0.05
        assert vals["DLRMSE"][0] < 0.6          # sd(yr) ~ 2.2: a mis-read enum spelling or a stalled net is far above
    finally:
        os.killpg(srv.pid, 15)
        srv.wait(timeout=30)
        log.close()
