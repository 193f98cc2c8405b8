"""-ldap_login: the REST server authenticates against an LDAP directory with Jetty LdapLoginModule's two login paths
(bind as the user / compare the stored userPassword). The directory is an in-process LDAPv3 responder speaking the
same BER subset (RFC 4511 bind + search with AND / equality filters); no LDAP server is in the image."""
import base64
import hashlib
import os
import socketserver
import threading

import pytest

from llama_github_io_amd.api import ldap as L
from llama_github_io_amd.api.security import LoginConfig, _CachedLogin

ADMIN = ("cn=admin,dc=h2o,dc=ai", "adminpw")
USERS = {
    "uid=alice,ou=users,dc=h2o,dc=ai": {"objectclass": [b"inetOrgPerson"], "uid": [b"alice"],
                                        "userpassword": [b"wonderland"]},
    "uid=bob,ou=users,dc=h2o,dc=ai": {"objectclass": [b"inetOrgPerson"], "uid": [b"bob"],
                                      "userpassword": [b"{SHA}" + base64.b64encode(hashlib.sha1(b"builder").digest())]},
    "uid=carol,ou=other,dc=h2o,dc=ai": {"objectclass": [b"inetOrgPerson"], "uid": [b"carol"],
                                        "userpassword": [b"{SSHA}" + base64.b64encode(
                                            hashlib.sha1(b"secret" + b"salt").digest() + b"salt")]},
}


def _password_ok(dn, pw):
    if (dn, pw) == ADMIN:
        return True
    e = USERS.get(dn)
    return e is not None and pw and L.check_stored(e["userpassword"][0], pw.decode() if isinstance(pw, bytes) else pw)


def _match(flt, entry):
    tag, val, _ = L.read_tlv(flt)
    if tag == 0xA0:
        return all(_match(L.tlv(t, v), entry) for t, v in L.read_all(val))
    if tag == 0xA3:
        (_, a), (_, v) = L.read_all(val)
        return v.lower() in [x.lower() for x in entry.get(a.decode().lower(), [])]
    return False


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        bound = None
        self.server.log.append("connect")
        while True:
            try:
                msg = L.recv_msg(self.request)
            except (ConnectionError, OSError):
                return
            _, body, _ = L.read_tlv(msg)
            (_, mid), (tag, op) = L.read_all(body)[:2]
            mid = int.from_bytes(mid, "big")
            if tag == 0x42:                                           # unbind
                return
            if tag == 0x60:                                           # bind
                _, (_, dn), (_, pw) = L.read_all(op)
                dn = dn.decode()
                ok = _password_ok(dn, pw.decode())
                bound = dn if ok else None
                self.server.log.append(("bind", dn, ok))
                rc = 0 if ok else 49                                  # invalidCredentials
                self.request.sendall(L.seq(L.ber_int(mid), L.seq(L.tlv(0x0A, bytes([rc])), L.ber_str(""),
                                                                 L.ber_str(""), tag=0x61)))
            elif tag == 0x63:                                         # search
                parts = L.read_all(op)
                base = parts[0][1].decode()
                flt = L.tlv(*parts[6])
                want = [v.decode().lower() for _, v in L.read_all(parts[7][1])]
                self.server.log.append(("search", bound, base))
                for dn, e in USERS.items():
                    if dn.endswith(base) and _match(flt, e):
                        if bound != ADMIN[0]:                         # only the admin may read passwords
                            e = {k: v for k, v in e.items() if k != "userpassword"}
                        attrs = [L.seq(L.ber_str(k), L.seq(*[L.ber_str(x) for x in v], tag=0x31))
                                 for k, v in e.items() if k in want]
                        self.request.sendall(L.seq(L.ber_int(mid), L.seq(L.ber_str(dn), L.seq(*attrs), tag=0x64)))
                self.request.sendall(L.seq(L.ber_int(mid), L.seq(L.tlv(0x0A, b"\x00"), L.ber_str(""),
                                                                 L.ber_str(""), tag=0x65)))


@pytest.fixture
def directory():
    srv = socketserver.ThreadingTCPServer(("127.0.0.1", 0), _Handler)
    srv.daemon_threads = True
    srv.log = []
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield srv
    srv.shutdown()
    srv.server_close()


def _conf(tmp_path, port, **opts):
    o = dict(hostname="127.0.0.1", port=str(port), bindDn=ADMIN[0], bindPassword=ADMIN[1],
             userBaseDn="ou=users,dc=h2o,dc=ai", userIdAttribute="uid", userObjectClass="inetOrgPerson",
             userPasswordAttribute="userPassword")
    o.update(opts)
    body = "\n".join(f'    {k}="{v}"' for k, v in o.items())
    p = tmp_path / "ldap.conf"
    p.write_text("// H2O LDAP login\nldaploginmodule {\n    org.eclipse.jetty.plus.jaas.spi.LdapLoginModule required\n"
                 f"{body};\n}};\n")
    return str(p)


def test_jaas_parse():
    cfg = L.parse_jaas('/* c */ a { x.y.LdapLoginModule required debug="true"\n hostname="h" port="1"; };\n'
                       'b { com.Other optional; };')
    assert cfg["a"] == dict(module="x.y.LdapLoginModule", flag="required", debug="true", hostname="h", port="1")
    assert cfg["b"]["module"] == "com.Other"


@pytest.mark.parametrize("force", ["true", "false"])
def test_ldap_login_paths(tmp_path, directory, force):
    svc = L.LdapLoginService(_conf(tmp_path, directory.server_address[1], forceBindingLogin=force))
    assert svc.login("alice", "wonderland")
    assert svc.login("bob", "builder")                     # {SHA} digest (compare path) / bind with the digest check
    assert not svc.login("alice", "wrong")
    assert not svc.login("alice", "")                      # no unauthenticated bind
    assert not svc.login("nobody", "x")
    assert not svc.login("carol", "secret")                # outside userBaseDn
    assert not svc.login("*", "wonderland")                # no filter injection: '*' is a literal value
    binds = [e for e in directory.log if isinstance(e, tuple) and e[0] == "bind"]
    if force == "true":
        assert ("bind", "uid=alice,ou=users,dc=h2o,dc=ai", True) in binds
    else:
        assert all(e[1] == ADMIN[0] for e in binds)        # the user's password is compared, never bound


def test_ldap_unreachable_and_bad_admin(tmp_path, directory):
    s = __import__("socket").socket()
    s.bind(("127.0.0.1", 0))
    dead = s.getsockname()[1]
    s.close()
    assert not L.LdapLoginService(_conf(tmp_path, dead)).login("alice", "wonderland")
    assert not L.LdapLoginService(_conf(tmp_path, directory.server_address[1], bindPassword="nope")).login(
        "alice", "wonderland")


def test_stored_password_forms():
    assert L.check_stored(b"{MD5}" + base64.b64encode(hashlib.md5(b"pw").digest()), "pw")
    assert L.check_stored(b"MD5:" + hashlib.md5(b"pw").hexdigest().encode(), "pw")
    assert not L.check_stored(b"{SSHA}AAAA", "pw")
    assert not L.check_stored(b"{SHA}!!notbase64", "pw")


def test_cached_login_counts_round_trips():
    class S:
        n = 0

        def login(self, u, p):
            S.n += 1
            return p == "ok"
    c = _CachedLogin(S(), ttl_s=60)
    assert c.login("u", "ok") and c.login("u", "ok") and S.n == 1
    assert not c.login("u", "bad") and not c.login("u", "bad") and S.n == 3   # failures are never cached


def test_rest_server_with_ldap_login(tmp_path, directory):
    from fastapi.testclient import TestClient
    from llama_github_io_amd.api.server import create_app
    conf = _conf(tmp_path, directory.server_address[1], forceBindingLogin="true")
    app = create_app(login=LoginConfig(ldap_login=True, login_conf=conf).validate())
    c = TestClient(app)
    assert c.get("/3/Cloud").status_code == 401
    assert c.get("/3/Cloud", auth=("alice", "wrong")).status_code == 401
    r = c.get("/3/Cloud", auth=("alice", "wonderland"))
    assert r.status_code == 200 and r.json()["cloud_healthy"]
    n = sum(1 for e in directory.log if e == "connect")
    assert c.get("/3/Cloud", auth=("alice", "wonderland")).status_code == 200
    assert sum(1 for e in directory.log if e == "connect") == n         # cached: no second LDAP round trip


def test_ldap_refuses_bad_config(tmp_path):
    p = tmp_path / "k.conf"
    p.write_text('krb { com.sun.security.auth.module.Krb5LoginModule required; };')
    with pytest.raises(ValueError, match="not an LdapLoginModule"):
        LoginConfig(ldap_login=True, login_conf=str(p)).validate()
    p.write_text('l { org.eclipse.jetty.jaas.spi.LdapLoginModule required authenticationMethod="DIGEST-MD5"; };')
    with pytest.raises(ValueError, match="simple"):
        LoginConfig(ldap_login=True, login_conf=str(p)).validate()
    assert os.path.exists(p)
