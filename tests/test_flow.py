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
  const opts = { cells, pollMs: 100, scope: {} };       // one notebook: variables persist across cells
  for (const c of cells) {
    const r = await Flow.runCell(call, c, opts);
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


PACKS = "/root/reference/h2o-docs/src/product/flow/packs"


@pytest.mark.skipif(NODE is None or not os.path.isdir(PACKS), reason="node or the reference's Flow packs not available")
def test_flow_parses_every_reference_pack_cell():
    """Every code cell of every notebook the reference ships (h2o-docs/src/product/flow/packs/**/*.flow, read as
    JSON data) parses, and names a routine this Flow implements — or is a script cell (assignments / if-else)."""
    src = r"""
const F = require(%s);
const fs = require("fs"), path = require("path");
const P = %s;
const names = {}, bad = [];
let n = 0, scripts = 0;
for (const d of fs.readdirSync(P)) {
  const dd = path.join(P, d);
  if (!fs.statSync(dd).isDirectory()) continue;
  for (const f of fs.readdirSync(dd).filter((x) => x.endsWith(".flow"))) {
    for (const c of JSON.parse(fs.readFileSync(path.join(dd, f), "utf8")).cells) {
      if (c.type !== "cs") continue;
      n++;
      try {
        const r = F.parseCell(c.input);
        if (!r) continue;
        if (r.script) { scripts++; continue; }
        names[r.name] = (names[r.name] || 0) + 1;
        if (!F.COMMANDS[r.name]) bad.push(f + ": unknown routine " + r.name);
      } catch (e) { bad.push(f + ": " + e.message); }
    }
  }
}
console.log(JSON.stringify({ n, scripts, names, bad }));
""" % (json.dumps(os.path.join(FLOW, "flow.js")), json.dumps(PACKS))
    r = subprocess.run([NODE, "-e", src], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["bad"] == [], out["bad"][:5]
    assert out["n"] > 3000 and out["scripts"] >= 1
    for routine in ("buildModel", "predict", "parseFiles", "setupParse", "splitFrame", "inspect", "grid", "getGrid",
                    "runAutoML", "getLeaderboard", "bindFrames", "changeColumnType", "imputeColumn", "createFrame",
                    "exportFrame", "assist"):
        assert out["names"].get(routine, 0) >= 1, routine


def test_flow_parser_coffeescript_forms():
    if NODE is None:
        pytest.skip("node not available")
    cells = ['grid inspect \'summary\', getGrid "g1", sort_by:"auc", decreasing:true ',
             'assist buildModel, null, training_frame: "ad.hex"',
             'parseFiles\n  paths: ["a.csv"]\n  destination_frame: "a.hex"\n  separator: 44\n  delete_on_done: true',
             'inspect getPrediction model: "m", frame: "f"',
             'runAutoML {"a": {"b": [1, -2, 0x10]}}, \'exec\'',
             'buildModel \'gbm\', {"hyper_parameters": {"min_rows": ["1";"2"]}}\n\n# steps taken:\n# click',
             'x = 1\nif x\n y = "a" + "b"\nelse\n y = "c"']
    src = "const F = require(%s); console.log(JSON.stringify(%s.map((c) => F.parseCell(c))))" % (
        json.dumps(os.path.join(FLOW, "flow.js")), json.dumps(cells))
    r = subprocess.run([NODE, "-e", src], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    a = json.loads(r.stdout)
    assert a[0] == {"name": "grid", "args": [{"__call": "inspect", "args": ["summary", {"__call": "getGrid", "args": [
        "g1", {"sort_by": "auc", "decreasing": True}]}]}]}
    assert a[1] == {"name": "assist", "args": [{"__ref": "buildModel"}, None, {"training_frame": "ad.hex"}]}
    assert a[2] == {"name": "parseFiles", "args": [{"paths": ["a.csv"], "destination_frame": "a.hex", "separator": 44,
                                                    "delete_on_done": True}]}
    assert a[3] == {"name": "inspect", "args": [{"__call": "getPrediction", "args": [{"model": "m", "frame": "f"}]}]}
    assert a[4] == {"name": "runAutoML", "args": [{"a": {"b": [1, -2, 16]}}, "exec"]}
    assert a[5]["args"][1] == {"hyper_parameters": {"min_rows": ["1", "2"]}}
    assert a[6]["script"][1]["if"] == {"__ref": "x"} and a[6]["script"][1]["then"][0]["set"] == "y"


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


def _serve(tmp_path):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               H2O_NPS_DIR=str(tmp_path / "nps"))
    log = open(tmp_path / "server.log", "w")
    srv = subprocess.Popen([sys.executable, "-m", "llama_github_io_amd.api.server", "--port", str(port)],
                           cwd=str(tmp_path), env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    t0 = time.time()
    while time.time() - t0 < 120:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=1).close()
            break
        except OSError:
            time.sleep(0.5)
    return srv, port


@pytest.mark.skipif(NODE is None, reason="node not available")
def test_flow_reference_syntax_notebook_end_to_end(tmp_path):
    """A notebook written the way the reference's shipped .flow packs write their cells (multi-line parseFiles,
    Flow-form buildModel parameters with string numbers / "" / hex seeds, grid via hyper_parameters, nested
    inspect / grid cells, script variables, the full AutoML spec with 'exec', project@@response leaderboards)
    runs against a live server."""
    rng = np.random.default_rng(7)
    n = 400
    X = rng.normal(size=(n, 2))
    g = rng.choice(["p", "q"], size=n)
    k = rng.integers(0, 3, size=n)
    y = np.where(X[:, 0] - X[:, 1] + (g == "p") * 0.5 + rng.normal(size=n) * 0.3 > 0, "yes", "no")
    with open(tmp_path / "flow.csv", "w") as f:
        f.write("a,b,g,k,y\n")
        for i in range(n):
            b = "" if i % 17 == 0 else f"{X[i, 1]:.5f}"
            f.write(f"{X[i, 0]:.5f},{b},{g[i]},{k[i]},{y[i]}\n")
    gbm = ('buildModel \'gbm\', {"model_id":"flow_gbm","training_frame":"flow_train.hex","validation_frame":'
           '"flow_test.hex","nfolds":0,"response_column":"y","ignored_columns":[],"ignore_const_cols":true,"ntrees":"5",'
           '"max_depth":3,"min_rows":10,"nbins":20,"seed":0xDECAF,"learn_rate":"0.1","distribution":"AUTO",'
           '"checkpoint":"","sample_rate_per_class":[],"histogram_type":"AUTO",'
           '"max_abs_leafnode_pred":1.7976931348623157e+308}\n\n# steps taken:\n# click on `Build Model`')
    grid = ('buildModel \'gbm\', {"model_id":"grid","training_frame":"flow_train.hex","response_column":"y",'
            '"ntrees":"3","seed":"1234","checkpoint":"","grid_id":"depth_grid",'
            '"hyper_parameters":{"max_depth":["1";"2";"3"]},"search_criteria":{"strategy":"Cartesian"}}')
    aml = ('runAutoML {"input_spec":{"training_frame":"flow_train.hex","response_column":"y","leaderboard_frame":'
           '"flow_test.hex","ignored_columns":[],"sort_metric":"AUTO"},"build_control":{"project_name":"flow_aml",'
           '"nfolds":0,"balance_classes":false,"stopping_criteria":{"seed":1,"max_models":2,"max_runtime_secs":360,'
           '"max_runtime_secs_per_model":0,"stopping_rounds":3,"stopping_metric":"AUTO","stopping_tolerance":-1},'
           '"keep_cross_validation_predictions":false,"keep_cross_validation_models":false,'
           '"keep_cross_validation_fold_assignment":false},"build_models":{"include_algos":["GLM","GBM"],'
           '"monotone_constraints":[]}}, \'exec\'')
    cells = [
        {"type": "md", "input": "# Flow pack syntax\n\nThe **reference** notebook forms."},
        f'# Did you download the files?\nhasLocalData = true\nlocation = "{tmp_path}/"\nif hasLocalData\n'
        f' trainFile = location + "flow.csv"\nelse\n trainFile = "https://example.invalid/flow.csv"',
        "importFiles [ trainFile ]",
        "setupParse paths: [ trainFile ]",
        'parseFiles\n  paths: [trainFile]\n  destination_frame: "flow.hex"\n  parse_type: "CSV"\n  separator: 44\n'
        '  number_columns: 5\n  single_quotes: false\n  column_names: ["a","b","g","k","y"]\n'
        '  column_types: ["Numeric","Numeric","Enum","Numeric","Enum"]\n  delete_on_done: true\n  check_header: 1\n'
        '  chunk_size: 4194304',
        'getFrameSummary "flow.hex"',
        'getColumnSummary "flow.hex", "a"',
        "changeColumnType frame: \"flow.hex\", column: \"k\", type: 'enum'",
        'imputeColumn {"frame":"flow.hex","column":"b","method":"MEAN","groupByColumns":["g"]}',
        'splitFrame "flow.hex", [0.75], ["flow_train.hex","flow_test.hex"], 1234',
        gbm,
        'getModel "flow_gbm"',
        'inspect getModel "flow_gbm"',
        'grid inspect "parameters", getModel "flow_gbm"',
        'predict model: "flow_gbm", frame: "flow_test.hex", predictions_frame: "flow_pred"',
        'inspect getPrediction model: "flow_gbm", frame: "flow_test.hex"',
        'predict model: "flow_gbm"',
        grid,
        "getGrids",
        'grid inspect \'summary\', getGrid "depth_grid", sort_by:"auc", decreasing:true ',
        'bindFrames "flow_bound", [ "flow_pred", "flow_test.hex" ]',
        'createFrame {"dest":"flow_rand.hex","rows":"300","cols":5,"seed":7595850248774472000,'
        '"seed_for_column_types":-1,"randomize":true,"value":0,"real_range":100,"categorical_fraction":0.2,'
        '"factors":5,"integer_fraction":0.2,"binary_fraction":0.16,"binary_ones_fraction":0.02,"time_fraction":0,'
        '"string_fraction":0,"integer_range":10000,"missing_fraction":0.01,"response_factors":2,"has_response":true}',
        f'exportFrame "flow_test.hex", "{tmp_path}/exported.csv", overwrite: true',
        'exportFrame "flow_test.hex"',
        aml,
        'getLeaderboard "flow_aml@@y"',
        "getJobs",
        "assist",
        'assist buildModel, null, training_frame: "flow.hex"',
        'getFrame "flow_pred"',
        'getFrameData "flow.hex"',
        'deleteModel "flow_gbm"',
        'saveFlow "nb2"',
        'loadFlow "nb2"',
    ]
    srv, port = _serve(tmp_path)
    try:
        drv = tmp_path / "driver.js"
        drv.write_text(DRIVER % dict(flow=json.dumps(os.path.join(FLOW, "flow.js")), port=port,
                                     cells=json.dumps(cells)))
        r = subprocess.run([NODE, str(drv)], capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-3000:] + open(tmp_path / "server.log").read()[-3000:]
        out = json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        os.killpg(srv.pid, 15)
        srv.wait(timeout=30)
    res = {i: o for i, o in enumerate(out)}
    by = lambda prefix: [o for o in out if isinstance(o["cell"], str) and o["cell"].startswith(prefix)]
    assert res[0]["kind"] == "markdown" and "<h1>Flow pack syntax</h1>" in res[0]["html"] and "<b>reference</b>" in res[0]["html"]
    assert "flow.csv" in by("importFiles")[0]["html"]
    assert by("parseFiles")[0]["kind"] == "frameSummary" and "400 rows" in by("parseFiles")[0]["html"]
    assert "<td>a</td>" in by("getColumnSummary")[0]["html"]
    chg = by("changeColumnType")[0]["html"]
    assert "<td>k</td><td>enum</td>" in chg.replace("Enum", "enum")
    imp = by("imputeColumn")[0]["html"]
    assert "<td>b</td><td>real</td><td>0</td>" in imp.replace("int", "real")          # no NAs left in b
    assert "flow_train.hex" in by("splitFrame")[0]["html"]
    assert by("buildModel 'gbm', {\"model_id\":\"flow_gbm\"")[0]["kind"] == "model"
    insp = by("inspect getModel")[0]
    assert insp["kind"] == "tables" and "parameters" in insp["html"] and "output - training_metrics" in insp["html"]
    assert by('grid inspect "parameters"')[0]["kind"] == "table" and "ntrees" in by('grid inspect "parameters"')[0]["html"]
    assert "AUC" in by("predict model: \"flow_gbm\", frame")[0]["html"]
    assert by('inspect getPrediction')[0]["kind"] == "tables" and "AUC" in by('inspect getPrediction')[0]["html"]
    assert by('predict model: "flow_gbm"')[-1]["kind"] == "form"
    assert by("buildModel 'gbm', {\"model_id\":\"grid\"")[0]["kind"] == "grid"
    assert "depth_grid" in by("getGrids")[0]["html"]
    gsum = by("grid inspect 'summary'")[0]
    assert gsum["kind"] == "table" and gsum["html"].count("<tr>") == 4                # header + 3 depths
    assert "predict" in by("bindFrames")[0]["html"]
    assert "300 rows" in by("createFrame")[0]["html"]
    assert (tmp_path / "exported.csv").exists() and by('exportFrame "flow_test.hex"')[-1]["kind"] == "form"
    assert by("runAutoML")[0]["kind"] == "leaderboard" and "model_id" in by("runAutoML")[0]["html"]
    assert by("getLeaderboard")[0]["kind"] == "leaderboard"
    assert by("assist buildModel")[0]["kind"] == "assist" and "gbm" in by("assist buildModel")[0]["html"]
    assert "getGrid" in by("assist")[0]["html"]
    assert "predict" in by('getFrame "flow_pred"')[0]["html"]
    nb = by('loadFlow "nb2"')[0]
    assert nb["kind"] == "notebook" and "<td>md</td>" in nb["html"] and "trainFile" in nb["html"]
