"""Flow web UI (reference: h2o-web / h2o-flow at ``/flow/index.html``): the page is served by the REST
server, and its command layer (``api/flow/flow.js``) drives a whole notebook — import + parse, frame
summary, GBM build, predict, AutoML leaderboard, Rapids, save / load of the notebook — against a live
server, run under node (the same code the browser runs; only ``http`` is injected)."""
import json
import os
import shutil
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLOW = os.path.join(ROOT, "llama_github_io_amd", "api", "flow")
NODE = shutil.which("node")

DRIVER = r"""
const Flow = require(%(flow)s);
const http = require("http");
function call(method, path, body) {
  return new Promise((resolve, reject) => {
    const data = body === undefined || method === "GET" ? null : JSON.stringify(body);
    const req = http.request({ host: "127.0.0.1", port: %(port)d, path, method,
      headers: data ? { "Content-Type": "application/json", "Content-Length": Buffer.byteLength(data) } : {} },
      (res) => { let s = ""; res.on("data", (c) => s += c); res.on("end", () => {
        let j = {}; try { j = JSON.parse(s); } catch (e) {}
        if (res.statusCode >= 400) reject(new Error(method + " " + path + " " + res.statusCode + " " + s.slice(0, 300)));
        else resolve(j); }); });
    req.on("error", reject);
    if (data) req.write(data);
    req.end();
  });
}
const cells = %(cells)s;
(async () => {
  const out = [];
  for (const c of cells) {
    const r = await Flow.runCell(call, c, { cells, pollMs: 100 });
    out.push({ cell: c, kind: r.kind, html: Flow.render(r) });
  }
  console.log(JSON.stringify(out));
})().catch((e) => { console.error("FLOWERR " + e.message); process.exit(1); });
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_flow_cell_parser_under_node():
    if NODE is None:
        pytest.skip("node not available")
    src = "const F = require(%s); console.log(JSON.stringify([F.parseCell('getFrames'), " \
          "F.parseCell('buildModel \"gbm\", {training_frame: \"t\", ntrees: 5, x: [\\'a\\', \"b\"]}'), " \
          "F.parseCell('predict model: \"m\", frame: \"f\"'), F.parseCell('getFrameSummary(\"fr\")')]))" \
          % json.dumps(os.path.join(FLOW, "flow.js"))
    r = subprocess.run([NODE, "-e", src], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    a = json.loads(r.stdout)
    assert a[0] == {"name": "getFrames", "args": []}
    assert a[1] == {"name": "buildModel", "args": ["gbm", {"training_frame": "t", "ntrees": 5, "x": ["a", "b"]}]}
    assert a[2] == {"name": "predict", "args": [{"model": "m", "frame": "f"}]}
    assert a[3] == {"name": "getFrameSummary", "args": ["fr"]}


def test_flow_page_served_and_routes_exist():
    from fastapi.testclient import TestClient
    from llama_github_io_amd.api.server import create_app
    c = TestClient(create_app())
    r = c.get("/flow/index.html")
    assert r.status_code == 200 and "H2O Flow" in r.text and "flow.js" in r.text
    js = c.get("/flow/flow.js")
    assert js.status_code == 200 and "runCell" in js.text
    assert c.get("/", follow_redirects=False).headers["location"] == "/flow/index.html"
    # every REST path the command layer calls is a route of the server
    import re
    paths = set(re.findall(r'"(/(?:3|99)/[A-Za-z0-9_./]+)', js.text))
    assert len(paths) >= 15
    routes = [getattr(rt, "path", "").split("/") for rt in c.app.routes]

    def seg_ok(a, b):                       # literal segment a vs route segment b ({param} matches anything)
        return a == b or (b.startswith("{") and b.endswith("}") and a != "")

    for p in paths:                          # p is a literal prefix; the command appends the parameters
        ps = [x for x in p.rstrip("/").split("/")]
        assert any(len(rt) >= len(ps) and all(seg_ok(a, b) for a, b in zip(ps, rt)) for rt in routes), p


@pytest.mark.skipif(NODE is None, reason="node not available")
def test_flow_notebook_end_to_end(tmp_path):
    rng = np.random.default_rng(5)
    n = 300
    X = rng.normal(size=(n, 3))
    y = np.where(X[:, 0] - X[:, 1] + rng.normal(size=n) * 0.3 > 0, "yes", "no")
    csv = tmp_path / "flow.csv"
    with open(csv, "w") as f:
        f.write("a,b,c,y\n")
        for i in range(n):
            f.write(f"{X[i, 0]:.5f},{X[i, 1]:.5f},{X[i, 2]:.5f},{y[i]}\n")
    cells = [
        "getCloud",
        f'importAndParse "{csv}", "flowfr"',
        'getFrameSummary "flowfr"',
        'getFrameData "flowfr", 5',
        'buildModel "gbm", {training_frame: "flowfr", response_column: "y", ntrees: 5, max_depth: 3, model_id: "flowgbm", seed: 1}',
        'predict model: "flowgbm", frame: "flowfr", predictions_frame: "flowpred"',
        "getModels",
        "getFrames",
        'runRapids "(nrow flowfr)"',
        'runAutoML {training_frame: "flowfr", response_column: "y", max_models: 2, project_name: "flowaml", nfolds: 0, include_algos: ["GLM", "GBM"], seed: 1}',
        'saveFlow "nb1"',
        'loadFlow "nb1"',
        "getJobs",
    ]
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               H2O_NPS_DIR=str(tmp_path / "nps"))
    log = open(tmp_path / "server.log", "w")
    srv = subprocess.Popen([sys.executable, "-m", "llama_github_io_amd.api.server", "--port", str(port)],
                           cwd=str(tmp_path), env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        t0 = time.time()
        while time.time() - t0 < 120:
            try:
                socket.create_connection(("127.0.0.1", port), timeout=1).close()
                break
            except OSError:
                time.sleep(0.5)
        drv = tmp_path / "driver.js"
        drv.write_text(DRIVER % dict(flow=json.dumps(os.path.join(FLOW, "flow.js")), port=port,
                                     cells=json.dumps(cells)))
        r = subprocess.run([NODE, str(drv)], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:] + open(tmp_path / "server.log").read()[-3000:]
        out = json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        os.killpg(srv.pid, 15)
        srv.wait(timeout=30)
    res = {o["cell"].split()[0]: o for o in out}
    assert res["importAndParse"]["kind"] == "frameSummary" and "300 rows" in res["importAndParse"]["html"]
    assert "<td>y</td>" in res["getFrameSummary"]["html"]
    assert res["getFrameData"]["html"].count("<tr>") == 6          # header + 5 rows
    assert res["buildModel"]["kind"] == "model" and "flowgbm" in res["buildModel"]["html"]
    assert "AUC" in res["buildModel"]["html"]
    assert "flowpred" in res["predict"]["html"] and "AUC" in res["predict"]["html"]
    assert "flowgbm" in res["getModels"]["html"] and "flowpred" in res["getFrames"]["html"]
    assert "300" in res["runRapids"]["html"]
    assert res["runAutoML"]["kind"] == "leaderboard" and "Leaderboard" in res["runAutoML"]["html"]
    assert res["loadFlow"]["kind"] == "notebook" and "importAndParse" in res["loadFlow"]["html"]
    assert "DONE" in res["getJobs"]["html"]


def test_h2o_flow_serves_in_process_frames():
    """h2o.flow() in process starts a local REST server over this process's DKV and returns the Flow URL."""
    import urllib.request
    import h2o
    import pandas as pd
    h2o.init()
    fr = h2o.H2OFrame(pd.DataFrame({"a": [1.0, 2.0, 3.0], "b": ["x", "y", "x"]}), destination_frame="flow_inproc")
    url = h2o.flow(open_browser=False)
    assert url.endswith("/flow/index.html")
    page = urllib.request.urlopen(url, timeout=30).read().decode()
    assert "H2O Flow" in page
    base = url.rsplit("/flow/", 1)[0]
    frames = json.loads(urllib.request.urlopen(base + "/3/Frames", timeout=30).read().decode())
    assert any((f["frame_id"]["name"] if isinstance(f["frame_id"], dict) else f["frame_id"]) == "flow_inproc"
               for f in frames["frames"])
    assert fr.nrow == 3
