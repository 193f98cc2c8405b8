"""-pam_login: the REST server authenticates through the host's libpam, as h2o-jaas-pam's PamLoginModule (JAAS entry
with a ``service``). The PAM stack here is a private configuration directory (pam_start_confdir) whose service runs
pam_exec with the offered password on stdin, so a real PAM transaction (conversation included) decides."""
import ctypes.util
import os

import pytest

from llama_github_io_amd.api.security import LoginConfig

pytestmark = pytest.mark.skipif(
    not ctypes.util.find_library("pam") or not os.path.exists("/lib/x86_64-linux-gnu/security/pam_exec.so"),
    reason="libpam / pam_exec not installed")


def _stack(tmp_path):
    chk = tmp_path / "check.sh"
    chk.write_text('#!/bin/sh\npw=$(cat | tr -d "\\000")\n[ "$PAM_USER" = "alice" ] && [ "$pw" = "wonder land" ]\n')
    chk.chmod(0o755)
    conf = tmp_path / "pam.d"
    conf.mkdir()
    (conf / "h2otest").write_text(f"auth required pam_exec.so expose_authtok quiet {chk}\n"
                                  "account required pam_permit.so\n")
    jaas = tmp_path / "pam.conf"
    jaas.write_text("pamloginmodule {\n  de.codedo.jaas.PamLoginModule required\n"
                    f'  service = h2otest\n  confdir = "{conf}";\n}};\n')
    return str(jaas)


def test_pam_login_service(tmp_path):
    from llama_github_io_amd.api.pam import PamLoginService
    svc = PamLoginService(_stack(tmp_path))
    assert svc.service == "h2otest"
    assert svc.login("alice", "wonder land")
    assert not svc.login("alice", "wrong")
    assert not svc.login("bob", "wonder land")
    assert not svc.login("alice", "")


def test_pam_config_errors(tmp_path):
    p = tmp_path / "bad.conf"
    p.write_text("pamloginmodule { de.codedo.jaas.PamLoginModule required; };")
    with pytest.raises(ValueError, match="PAM service was not defined"):
        LoginConfig(pam_login=True, login_conf=str(p)).validate()
    p.write_text('x { org.eclipse.jetty.jaas.spi.LdapLoginModule required hostname="h"; };')
    with pytest.raises(ValueError, match="not a PamLoginModule"):
        LoginConfig(pam_login=True, login_conf=str(p)).validate()


def test_rest_server_with_pam_login(tmp_path):
    from fastapi.testclient import TestClient
    from llama_github_io_amd.api.server import create_app
    app = create_app(login=LoginConfig(pam_login=True, login_conf=_stack(tmp_path)).validate())
    c = TestClient(app)
    assert c.get("/3/Cloud").status_code == 401
    assert c.get("/3/Cloud", auth=("alice", "nope")).status_code == 401
    assert c.get("/3/Cloud", auth=("alice", "wonder land")).status_code == 200
