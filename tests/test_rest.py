"""REST API through FastAPI's TestClient: import/parse, frames, build (async job), predict, metrics,
rapids, grid, MOJO download."""
import time

import numpy as np
import pytest

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    from llama_github_io_amd.api.server import create_app
    d = tmp_path_factory.mktemp("data")
    rng = np.random.default_rng(0)
    with open(d / "train.csv", "w") as f:
        f.write("a,b,c,y\n")
        for i in range(600):
            a, b = rng.normal(), rng.normal()
            c = rng.choice(["u", "v"])
            y = "yes" if a - b + (c == "u") + rng.normal() * 0.3 > 0 else "no"
            f.write(f"{a},{b},{c},{y}\n")
    c = TestClient(create_app())
    c.data_path = str(d / "train.csv")
    return c


def _wait(client, job_key, timeout=120):
    t0 = time.time()
    while time.time() - t0 < timeout:
        j = client.get(f"/3/Jobs/{job_key}").json()["jobs"][0]
        if j["status"] in ("DONE", "FAILED", "CANCELLED"):
            return j
        time.sleep(0.05)
    raise TimeoutError(job_key)


def test_end_to_end(client):
    assert client.get("/3/Cloud").json()["cloud_size"] == 1
    r = client.post("/3/ImportFiles", params=dict(path=client.data_path)).json()
    s = client.post("/3/ParseSetup", data=dict(source_frames=r["destination_frames"][0])).json()
    assert s["column_names"] == ["a", "b", "c", "y"]
    p = client.post("/3/Parse", data=dict(source_frames=r["destination_frames"][0], destination_frame="train.hex")).json()
    assert _wait(client, p["job"]["key"]["name"])["status"] == "DONE"
    fr = client.get("/3/Frames/train.hex").json()["frames"][0]
    assert fr["rows"] == 600 and [c["type"] for c in fr["columns"]] == ["real", "real", "enum", "enum"]
    b = client.post("/3/ModelBuilders/gbm", data=dict(training_frame="train.hex", response_column="y", ntrees=5,
                                                      model_id="gbm1", seed=1)).json()
    assert _wait(client, b["job"]["key"]["name"])["status"] == "DONE"
    m = client.get("/3/Models/gbm1").json()["models"][0]
    assert m["output"]["training_metrics"]["AUC"] > 0.8
    pr = client.post("/3/Predictions/models/gbm1/frames/train.hex", data=dict(predictions_frame="preds")).json()
    assert client.get("/3/Frames/preds").json()["frames"][0]["num_columns"] == 3
    mm = client.post("/3/ModelMetrics/models/gbm1/frames/train.hex").json()["model_metrics"][0]
    assert abs(mm["AUC"] - m["output"]["training_metrics"]["AUC"]) < 1e-9
    rp = client.post("/99/Rapids", data=dict(ast="(nrow train.hex)")).json()
    assert rp["scalar"] == 600
    g = client.post("/99/Grid/gbm", data=dict(training_frame="train.hex", response_column="y", grid_id="g1",
                                             hyper_parameters='{"max_depth": [2, 3]}', ntrees=3)).json()
    assert _wait(client, g["job"]["key"]["name"])["status"] == "DONE"
    assert len(client.get("/99/Grids/g1").json()["model_ids"]) == 2
    z = client.get("/3/Models/gbm1/mojo")
    assert z.status_code == 200 and z.content[:2] == b"PK"
