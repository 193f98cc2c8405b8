"""REST API v4 (water/api/RegisterV4Api.java:13-42): endpoint listing, models info, sessions, the simple
create-frame recipe run as a Job (JobV4) and job fetch."""
import time

import pytest

pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402

from llama_github_io_amd.api.server import create_app  # noqa: E402


@pytest.fixture(scope="module")
def client():
    return TestClient(create_app(), raise_server_exceptions=False)


def test_endpoints_and_modelsinfo(client):
    eps = client.get("/4/endpoints").json()
    assert eps["__meta"]["schema_name"] == "EndpointsListV4"
    urls = {e["url"] for e in eps["endpoints"]}
    for u in ("GET /4/endpoints", "POST /4/sessions", "DELETE /4/sessions/{session_key}", "GET /4/modelsinfo",
              "POST /4/Frames/$simple", "GET /4/jobs/{job_id}"):
        assert u in urls, u
    mi = client.get("/4/modelsinfo").json()["models"]
    by = {m["algo"]: m for m in mi}
    assert by["gbm"]["have_mojo"] and by["gbm"]["have_pojo"] and by["gbm"]["maturity"] == "stable"
    assert by["gbm"]["mojo_version"] == "1.40"
    assert {"glm", "deeplearning", "kmeans", "xgboost"} <= set(by)


def test_simple_frame_job(client):
    r = client.post("/4/Frames/$simple", json=dict(dest="simple4", seed=42, nrows=500, ncols_real=3, ncols_int=2,
                                                   ncols_enum=2, ncols_bool=1, ncols_str=1, ncols_time=1,
                                                   missing_fraction=0.1, response_type="bool"))
    assert r.status_code == 200, r.text
    j = r.json()
    assert j["__meta"]["schema_name"] == "JobV4"
    jid = j["job_id"]
    for _ in range(400):
        j = client.get(f"/4/jobs/{jid}").json()
        if j["status"] in ("DONE", "FAILED"):
            break
        time.sleep(0.02)
    assert j["status"] == "DONE", j
    assert j["target_id"] == "simple4" and j["target_type"] == "Frame"
    fr = client.get("/3/Frames/simple4").json()["frames"][0]
    assert fr["rows"] == 500
    names = [c["label"] for c in fr["columns"]]
    assert names[0] == "response" and len(names) == 11
    assert sorted(n.rstrip("0123456789") for n in names[1:]) == sorted(["R"] * 3 + ["I"] * 2 + ["E"] * 2 + ["B", "S", "T"])
    bad = client.post("/4/Frames/$simple", json=dict(real_lb=5, real_ub=1))
    assert bad.status_code >= 400 or client.get(f"/4/jobs/{bad.json()['job_id']}").json()["status"] in ("FAILED", "RUNNING")


def test_sessions_v4(client):
    sid = client.post("/4/sessions").json()["session_key"]
    assert client.delete(f"/4/sessions/{sid}").json()["session_key"] == sid
