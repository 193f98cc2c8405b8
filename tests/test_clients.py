"""ClientDisconnectCheckThread equivalent: REST clients not heard from within the timeout are dropped
and their sessions end."""
import time

from fastapi.testclient import TestClient

from llama_github_io_amd.api import clients
from llama_github_io_amd.api.server import create_app


def test_client_disconnect_check():
    clients.reset()
    app = create_app()
    tc = TestClient(app)
    sid = tc.post("/4/sessions", headers={"X-H2O-Client": "py-1"}).json()["session_key"]
    tc.get("/3/Cloud", headers={"X-H2O-Client": "py-2"})
    lst = {c["client"]: c for c in tc.get("/3/Clients", headers={"X-H2O-Client": "py-2"}).json()["clients"]}
    assert sid in lst["py-1"]["sessions"] and "py-2" in lst
    seen = []
    clients.on_disconnect(lambda k, s: seen.append((k, s)))
    now = time.time()
    clients.touch("py-2", now=now + 9)
    assert clients.check(10.0, now=now + 11) == ["py-1"]
    assert seen[-1] == ("py-1", [sid]) and "py-1" not in clients.clients()


def test_client_disconnect_thread_runs():
    clients.reset()
    clients.touch("gone", now=time.time() - 100)
    clients.start(0.05)
    try:
        t0 = time.time()
        while "gone" in clients.clients() and time.time() - t0 < 5:
            time.sleep(0.02)
        assert "gone" not in clients.clients()
    finally:
        clients.stop()
