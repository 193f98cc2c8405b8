"""``import_file("http://...")`` (water/persist/PersistManager.java:301,423, PersistEagerHTTP.java) against a local
stdlib HTTP server: CSV and gzip bodies, the REST ImportFiles -> ParseSetup -> Parse flow, a 404, and the refusal of
a store scheme with no backend here (maprfs)."""
import functools
import gzip
import http.server
import threading

import numpy as np
import pandas as pd
import pytest

import h2o


@pytest.fixture(scope="module")
def server(tmp_path_factory):
    root = tmp_path_factory.mktemp("www")
    rng = np.random.default_rng(5)
    df = pd.DataFrame({"a": rng.normal(size=200), "b": rng.integers(0, 5, 200), "c": rng.choice(["x", "y"], 200)})
    df.to_csv(root / "data.csv", index=False)
    with gzip.open(root / "more.csv.gz", "wt") as f:
        df.to_csv(f, index=False)
    handler = functools.partial(http.server.SimpleHTTPRequestHandler, directory=str(root))
    handler.log_message = lambda *a, **k: None
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), handler)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    h2o.init(verbose=False)
    yield f"http://127.0.0.1:{srv.server_address[1]}", df
    srv.shutdown()


def test_import_file_over_http(server):
    base, df = server
    fr = h2o.import_file(base + "/data.csv")
    assert fr.shape == (200, 3)
    assert fr.frame_id == "data.hex"
    got = fr.as_data_frame()
    np.testing.assert_allclose(got["a"].to_numpy(float), df["a"].to_numpy(), rtol=1e-12)
    assert list(got["c"]) == list(df["c"])
    gz = h2o.import_file(base + "/more.csv.gz")
    np.testing.assert_allclose(gz.as_data_frame()["b"].to_numpy(float), df["b"].to_numpy(float))


def test_http_errors_and_object_stores(server):
    base, _ = server
    with pytest.raises(FileNotFoundError, match="Unable to import file from URL"):
        h2o.import_file(base + "/missing.csv")
    with pytest.raises(ValueError, match="persist backend"):
        h2o.import_file("maprfs://cluster/x.csv")     # (s3 / gs / hdfs: tests/test_persist_store.py)


def test_rest_import_parse_over_http(server):
    pytest.importorskip("fastapi")
    from fastapi.testclient import TestClient
    from llama_github_io_amd.api.server import create_app
    base, df = server
    c = TestClient(create_app(), raise_server_exceptions=False)
    r = c.get("/3/ImportFiles", params={"path": base + "/data.csv"}).json()
    assert len(r["files"]) == 1 and r["fails"] == []
    st = c.post("/3/ParseSetup", json=dict(source_frames=r["destination_frames"])).json()
    assert st["column_names"] == ["a", "b", "c"]
