"""The REST API served by a multi-rank SPMD cloud (``api/cloud.py``; reference ``water/api/RequestServer.java``
+ the MRTask fan-out): ``torchrun --nproc-per-node 2 -m llama_github_io_amd.api.server`` under gloo on the CPU,
driven over HTTP by the UNMODIFIED reference h2o-py client (``h2o.connect``): import_file -> GBM -> GLM ->
AutoML(max_models=3) -> predict -> download_mojo. The cloud must report cloud_size == 2, parse the file into
row shards, train row-sharded, and return the models / predictions of the single-process server."""
import json
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

needs_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "h2o")), reason="reference h2o-py not present")

CLIENT = textwrap.dedent("""
    import json, os, sys, tempfile
    sys.path.insert(0, %(ref)r)
    import h2o
    h2o.connect(url="http://127.0.0.1:%(port)d", verbose=False, strict_version_check=False)
    out = {}
    cl = h2o.cluster()
    out["cloud_size"] = cl.cloud_size
    fr = h2o.import_file(%(csv)r)
    out["dim"] = [fr.nrow, fr.ncol]
    out["mean_x0"] = fr["x0"].mean()[0]
    from h2o.estimators import H2OGradientBoostingEstimator, H2OGeneralizedLinearEstimator
    m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1)
    m.train(x=["x0", "x1", "x2", "cat"], y="yb", training_frame=fr)
    out["gbm_auc"] = m.auc()
    out["gbm_logloss"] = m.logloss()
    g = H2OGeneralizedLinearEstimator(family="binomial", lambda_=1e-3)
    g.train(x=["x0", "x1", "x2"], y="yb", training_frame=fr)
    out["glm_coef"] = g.coef()
    from h2o.automl import H2OAutoML
    aml = H2OAutoML(max_models=3, seed=1, nfolds=2, include_algos=["GLM", "GBM", "DRF"])
    aml.train(x=["x0", "x1", "x2", "cat"], y="yb", training_frame=fr)
    lb = aml.leaderboard.as_data_frame(use_pandas=False)
    out["aml_n"] = len(lb) - 1
    out["aml_auc"] = sorted(float(r[1]) for r in lb[1:])
    p = m.predict(fr)
    rows = p.as_data_frame(use_pandas=False)
    out["pred_n"] = len(rows) - 1
    out["pred_yes"] = [float(r[2]) for r in rows[1:]]
    d = tempfile.mkdtemp()
    path = m.download_mojo(d)
    out["mojo_bytes"] = os.path.getsize(path)
    import zipfile
    out["mojo_files"] = sorted(zipfile.ZipFile(path).namelist())[:5]
    print("RESULT " + json.dumps(out))
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(tmp_path, n=600):
    rng = np.random.default_rng(7)
    X = rng.normal(size=(n, 3))
    cat = rng.choice(["a", "b", "c"], n)
    yb = np.where(X[:, 0] - X[:, 1] + 0.6 * (cat == "b") + rng.normal(size=n) * 0.7 > 0, "yes", "no")
    csv = tmp_path / "d.csv"
    with open(csv, "w") as f:
        f.write("x0,x1,x2,cat,yb\n")
        for i in range(n):
            f.write(f"{X[i, 0]:.6f},{X[i, 1]:.6f},{X[i, 2]:.6f},{cat[i]},{yb[i]}\n")
    return csv


def _serve_and_run(tmp_path, csv, world, env_over=None, torchrun=False):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", H2O_AMD_DEVICE="cpu",
               OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    if env_over:
        env.update(env_over)
        if env_over.get("H2O_AMD_DEVICE") == "cuda":
            for k in ("CUDA_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
                if os.environ.get(k) is None:
                    env.pop(k, None)
                else:
                    env[k] = os.environ[k]
    if world == 1 and not torchrun:
        cmd = [sys.executable, "-m", "llama_github_io_amd.api.server", "--port", str(port)]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               "-m", "llama_github_io_amd.api.server", "--port", str(port)]
    tag = f"{world}{'t' if torchrun else ''}{env.get('H2O_AMD_DEVICE')}"
    log = open(tmp_path / f"server{tag}.log", "w")
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        t0 = time.time()
        while time.time() - t0 < 180:
            try:
                socket.create_connection(("127.0.0.1", port), timeout=1).close()
                break
            except OSError:
                assert srv.poll() is None, open(tmp_path / f"server{tag}.log").read()[-3000:]
                time.sleep(0.5)
        script = tmp_path / f"client{tag}.py"
        script.write_text(CLIENT % dict(ref=REF, port=port, csv=str(csv)))
        cenv = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
        r = subprocess.run([sys.executable, str(script)], cwd=str(tmp_path), env=cenv, capture_output=True, text=True,
                           timeout=900)
        out = r.stdout + r.stderr
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
        assert r.returncode == 0 and lines, out[-4000:] + open(tmp_path / f"server{tag}.log").read()[-4000:]
        return json.loads(lines[0][7:])
    finally:
        os.killpg(srv.pid, 15)
        try:
            srv.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(srv.pid, 9)
            srv.wait(timeout=30)
        log.close()


@needs_ref
def test_rest_cloud_two_ranks_matches_single_process(tmp_path):
    csv = _data(tmp_path)
    one = _serve_and_run(tmp_path, csv, 1)
    two = _serve_and_run(tmp_path, csv, 2)
    assert one["cloud_size"] == 1 and two["cloud_size"] == 2
    assert two["dim"] == one["dim"] == [600, 5]
    assert abs(two["mean_x0"] - one["mean_x0"]) < 1e-9
    assert abs(two["gbm_auc"] - one["gbm_auc"]) < 1e-6 and abs(two["gbm_logloss"] - one["gbm_logloss"]) < 1e-6
    for k, v in one["glm_coef"].items():
        assert abs(two["glm_coef"][k] - v) < 1e-5, (k, v, two["glm_coef"][k])
    assert two["aml_n"] == one["aml_n"] >= 3
    # (sharded AUCs merge per-rank score histograms on a fixed 2^18-cell lattice: equal to ~1e-4, not bit-exact)
    assert np.allclose(two["aml_auc"], one["aml_auc"], atol=1e-4), (one["aml_auc"], two["aml_auc"])
    assert two["pred_n"] == one["pred_n"] == 600
    assert np.allclose(two["pred_yes"], one["pred_yes"], atol=1e-6)
    assert two["mojo_bytes"] > 0 and two["mojo_files"] == one["mojo_files"]


CANCEL_CLIENT = textwrap.dedent("""
    import json, sys, time
    sys.path.insert(0, %(ref)r)
    import h2o, requests
    h2o.connect(url="http://127.0.0.1:%(port)d", verbose=False, strict_version_check=False)
    fr = h2o.import_file(%(csv)r)
    base = "http://127.0.0.1:%(port)d"
    r = requests.post(base + "/3/ModelBuilders/gbm", data=dict(training_frame=fr.frame_id, response_column="yb",
                                                               ntrees=5000, max_depth=4, seed=3, score_tree_interval=0))
    key = r.json()["job"]["key"]["name"]
    t0, seen = time.time(), None
    while time.time() - t0 < 120:                       # job polling is answered while the job runs
        j = requests.get(base + "/3/Jobs/" + key, timeout=10).json()["jobs"][0]
        if j["status"] == "RUNNING" and j["progress"] > 0:
            seen = j["progress"]
            break
        time.sleep(0.05)
    c = requests.post(base + "/3/Jobs/" + key + "/cancel", timeout=10)
    status = None
    while time.time() - t0 < 240:
        status = requests.get(base + "/3/Jobs/" + key, timeout=10).json()["jobs"][0]["status"]
        if status in ("CANCELLED", "DONE", "FAILED"):
            break
        time.sleep(0.1)
    # the cloud is still in lock step: a new build on every rank trains and answers
    m = h2o.estimators.H2OGradientBoostingEstimator(ntrees=3, max_depth=2, seed=1)
    m.train(x=["x0", "x1"], y="yb", training_frame=fr)
    print("RESULT " + json.dumps(dict(seen=seen, cancel_status=c.status_code, status=status, auc=m.auc(),
                                      nodes=len(h2o.cluster().nodes))))
""")


@needs_ref
def test_rest_cloud_cancel_and_polling(tmp_path):
    """``GET /3/Jobs`` answers while a cloud job runs (rank 0 alone); ``cancel`` stops the job on EVERY rank at the
    same progress check, and the cloud keeps serving in lock step afterwards."""
    csv = _data(tmp_path)
    global CLIENT
    saved = CLIENT
    CLIENT = CANCEL_CLIENT
    try:
        out = _serve_and_run(tmp_path, csv, 2)
    finally:
        CLIENT = saved
    assert out["seen"] is not None and 0 < out["seen"] < 1
    assert out["cancel_status"] == 200 and out["status"] == "CANCELLED"
    assert out["auc"] > 0.7 and out["nodes"] == 2


RAW_CLIENT = textwrap.dedent('''
    import io, json, sys, time, zipfile
    import requests
    base = "http://127.0.0.1:%(port)d"

    def call(method, route, **data):
        enc = {k: (json.dumps(v) if isinstance(v, (list, dict)) else v) for k, v in data.items()}
        r = requests.request(method, base + route, params=enc if method == "GET" else None,
                             data=None if method == "GET" else enc, timeout=600)
        assert r.status_code == 200, (route, r.status_code, r.text[:500])
        return r

    def wait(job):
        key = job["key"]["name"]
        while True:
            j = call("GET", "/3/Jobs/" + key).json()["jobs"][0]
            if j["status"] in ("DONE", "FAILED", "CANCELLED"):
                assert j["status"] == "DONE", j
                return j
            time.sleep(0.1)

    out = {"cloud_size": call("GET", "/3/Cloud").json()["cloud_size"]}
    src = call("POST", "/3/ImportFiles", path=%(csv)r).json()["destination_frames"]
    ps = call("POST", "/3/ParseSetup", source_frames=src).json()
    wait(call("POST", "/3/Parse", source_frames=src, destination_frame="d.hex", column_names=ps["column_names"],
              column_types=ps["column_types"], separator=ps["separator"], check_header=ps["check_header"]).json()["job"])
    for algo, params in (("gbm", dict(ntrees=5, max_depth=3, seed=1)), ("glm", dict(family="binomial", lambda_=1e-3))):
        j = call("POST", "/3/ModelBuilders/" + algo, training_frame="d.hex", response_column="yb", model_id=algo + "_m",
                 **params).json()["job"]
        wait(j)
        m = call("GET", "/3/Models/" + algo + "_m").json()["models"][0]
        out[algo + "_auc"] = m["output"]["training_metrics"]["AUC"]
    call("POST", "/3/Predictions/models/gbm_m/frames/d.hex", predictions_frame="p.hex")
    csv_txt = call("GET", "/3/DownloadDataset", frame_id="p.hex").text.splitlines()
    out["pred_yes"] = [float(l.split(",")[2]) for l in csv_txt[1:]]
    z = zipfile.ZipFile(io.BytesIO(call("GET", "/3/Models/gbm_m/mojo").content))
    out["mojo_files"] = sorted(z.namelist())[:5]
    print("RESULT " + json.dumps(out))
''')


@pytest.mark.gpu
def test_rest_cloud_gpu_rank_matches_single_process(tmp_path):
    """The cloud executor on a GPU: a 1-rank ``nccl`` cloud (``H2O_FORCE_SHARDED=1``: every trainer takes its
    row-sharded path, collectives through RCCL from the executor thread) serves the same models and predictions as
    the plain single-process GPU server (raw REST client: no reference tree on the GPU box)."""
    global CLIENT
    csv = _data(tmp_path)
    saved = CLIENT
    CLIENT = RAW_CLIENT
    try:
        gpu_env = dict(H2O_AMD_DEVICE="cuda")
        one = _serve_and_run(tmp_path, csv, 1, env_over=gpu_env)
        cl = _serve_and_run(tmp_path, csv, 1, env_over=dict(gpu_env, H2O_FORCE_SHARDED="1"), torchrun=True)
    finally:
        CLIENT = saved
    assert one["cloud_size"] == cl["cloud_size"] == 1
    assert abs(one["gbm_auc"] - cl["gbm_auc"]) < 1e-4 and abs(one["glm_auc"] - cl["glm_auc"]) < 1e-4
    assert np.allclose(one["pred_yes"], cl["pred_yes"], atol=1e-5) and len(cl["pred_yes"]) == 600
    assert one["mojo_files"] == cl["mojo_files"]
