"""-kerberos_login / -spnego_login through the host's MIT Kerberos libraries (api/krb5.py).

No KDC exists in this image, so the Kerberos login is pinned against a stand-in KDC on 127.0.0.1: a UDP socket that
records the AS-REQ libkrb5 sends (the client principal and realm must be in it) and answers with a DER KRB-ERROR
(KDC_ERR_C_PRINCIPAL_UNKNOWN), which libkrb5 must turn into a refused login. A successful ticket exchange needs a
real KDC: parity unpinned. SPNEGO is pinned on its protocol surface: the Negotiate challenge, and GSSAPI refusing a
token that is not a valid Kerberos AP-REQ (no keytab here)."""
import base64
import ctypes.util
import socket
import threading
import time

import pytest

from llama_github_io_amd.api.ldap import ber_int, seq, tlv
from llama_github_io_amd.api.security import LoginConfig

pytestmark = pytest.mark.skipif(not ctypes.util.find_library("krb5") or not ctypes.util.find_library("gssapi_krb5"),
                                reason="MIT Kerberos libraries not installed")

REALM = b"H2O.TEST"


def _krb_error(code: int) -> bytes:
    c = lambda n, v: tlv(0xA0 + n, v)     # noqa: E731  (context tag [n], constructed)
    now = time.strftime("%Y%m%d%H%M%SZ", time.gmtime()).encode()
    return tlv(0x7E, seq(c(0, ber_int(5)), c(1, ber_int(30)), c(4, tlv(0x18, now)), c(5, ber_int(0)),
                         c(6, ber_int(code)), c(9, tlv(0x1B, REALM)),
                         c(10, seq(c(0, ber_int(2)), c(1, seq(tlv(0x1B, b"krbtgt"), tlv(0x1B, REALM)))))))


class FakeKdc:
    def __init__(self):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.settimeout(0.2)
        self.port = self.sock.getsockname()[1]
        self.requests = []
        self._stop = False
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        while not self._stop:
            try:
                data, addr = self.sock.recvfrom(65536)
            except socket.timeout:
                continue
            except OSError:
                return
            self.requests.append(data)
            self.sock.sendto(_krb_error(6), addr)

    def close(self):
        self._stop = True
        self.t.join(2)
        self.sock.close()


@pytest.fixture
def kdc():
    k = FakeKdc()
    yield k
    k.close()


def _jaas(tmp_path, port):
    p = tmp_path / "krb5.jaas"
    p.write_text("krb5loginmodule {\n  com.sun.security.auth.module.Krb5LoginModule required\n"
                 f'  realm="{REALM.decode()}"\n  kdc="127.0.0.1:{port}"\n  useTicketCache=false;\n}};\n')
    return str(p)


def test_kerberos_login_sends_as_req_and_refuses_unknown_client(tmp_path, kdc):
    from llama_github_io_amd.api.krb5 import Krb5LoginService
    svc = Krb5LoginService(_jaas(tmp_path, kdc.port))
    assert svc.principal("alice") == "alice@H2O.TEST" and svc.principal("bob@X.Y") == "bob@X.Y"
    t0 = time.time()
    assert not svc.login("alice", "secret")
    assert time.time() - t0 < 10
    assert "not found" in svc.last_error.lower()
    assert kdc.requests, "libkrb5 sent nothing to the configured KDC"
    req = kdc.requests[0]
    assert req[0] == 0x6A                       # [APPLICATION 10] AS-REQ
    assert b"alice" in req and REALM in req and b"krbtgt" in req
    assert not svc.login("alice", "")           # no KDC round trip for an empty password
    assert len(kdc.requests) == 1


def test_rest_server_with_kerberos_login(tmp_path, kdc):
    from fastapi.testclient import TestClient
    from llama_github_io_amd.api.server import create_app
    app = create_app(login=LoginConfig(kerberos_login=True, login_conf=_jaas(tmp_path, kdc.port)).validate())
    c = TestClient(app)
    r = c.get("/3/Cloud")
    assert r.status_code == 401 and r.headers["www-authenticate"].startswith("Basic")
    assert c.get("/3/Cloud", auth=("alice", "secret")).status_code == 401
    assert kdc.requests and kdc.requests[-1][0] == 0x6A


def test_kerberos_config_errors(tmp_path):
    p = tmp_path / "x.conf"
    p.write_text('x { org.eclipse.jetty.jaas.spi.LdapLoginModule required hostname="h"; };')
    with pytest.raises(ValueError, match="Krb5LoginModule"):
        LoginConfig(kerberos_login=True, login_conf=str(p)).validate()
    with pytest.raises(ValueError, match="File does not exist"):
        LoginConfig(spnego_login=True, login_conf=str(p), spnego_properties=str(tmp_path / "none")).validate()


def test_spnego_challenge_and_invalid_token(tmp_path):
    from fastapi.testclient import TestClient
    from llama_github_io_amd.api.krb5 import SpnegoService, read_properties
    from llama_github_io_amd.api.server import create_app
    props = tmp_path / "spnego.properties"
    props.write_text("# acceptor\ntargetName = HTTP/localhost@H2O.TEST\n")
    assert read_properties(str(props)) == {"targetName": "HTTP/localhost@H2O.TEST"}
    jaas = tmp_path / "spnego.jaas"
    jaas.write_text("com.sun.security.jgss.accept {\n  com.sun.security.auth.module.Krb5LoginModule required\n"
                    f'  storeKey=true\n  keyTab="{tmp_path / "missing.keytab"}"\n  principal="HTTP/localhost";\n}};\n')
    svc = SpnegoService(str(jaas), str(props))
    assert svc.target == "HTTP/localhost@H2O.TEST" and svc.keytab.endswith("missing.keytab")
    user, _ = svc.accept(b"\x60\x03\x06\x01\x00")            # not a SPNEGO / Kerberos token
    assert user is None and svc.last_error
    app = create_app(login=LoginConfig(spnego_login=True, login_conf=str(jaas),
                                       spnego_properties=str(props)).validate())
    c = TestClient(app)
    r = c.get("/3/Cloud")
    assert r.status_code == 401 and r.headers["www-authenticate"] == "Negotiate"
    r = c.get("/3/Cloud", headers={"Authorization": "Negotiate " + base64.b64encode(b"garbage").decode()})
    assert r.status_code == 401 and r.headers["www-authenticate"].startswith("Negotiate")
    assert c.get("/3/Cloud", auth=("alice", "pw")).status_code == 401     # Basic is not accepted under SPNEGO
