"""REST login (api/security.py): Jetty HashLoginService realm files, Basic auth on every route, Form auth for
browsers, the H2O.java option rules. Reference: Jetty9Helper.authWrapper, Jetty9DelegatingAuthenticator,
H2OHttpViewImpl.loginHandler; h2o-assemblies/main/tests/python/pyunit_redirect_relative.py (a browser without
credentials is redirected to a RELATIVE /login) and its realm.properties (plain credential)."""
import base64
import hashlib
import os

import pytest

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402

from llama_github_io_amd.api import security  # noqa: E402
from llama_github_io_amd.api.server import create_app, main  # noqa: E402

REF_REALM = "/root/reference/h2o-assemblies/main/tests/python/realm.properties"


def _realm(tmp_path):
    import crypt
    p = tmp_path / "realm.properties"
    p.write_text("# users\n"
                 "jenkins_user: jenkins_pwd42\n"
                 f"obf_user: {security.obfuscate('s3cret!')}, user\n"
                 f"md5_user: MD5:{hashlib.md5(b'md5pass').hexdigest()}\n"
                 f"crypt_user: CRYPT:{crypt.crypt('cpass', 'cu')}\n")
    return str(p)


def _basic(u, p):
    return {"Authorization": "Basic " + base64.b64encode(f"{u}:{p}".encode()).decode()}


def test_jetty_obfuscation_vector():
    # Jetty's documented Password example (user "me", password "you"): OBF and MD5 forms
    assert security.obfuscate("you") == "OBF:20771x1b206z"
    assert security.deobfuscate("OBF:20771x1b206z") == "you"
    assert security.check_credential("MD5:639bae9ac6b3e1a84cebb7b403297b79", "you")
    for pw in ("", "a", "p@ss word", "ünïcode"):
        assert security.deobfuscate(security.obfuscate(pw)) == pw


def test_basic_auth_every_route(tmp_path):
    app = create_app(login=security.LoginConfig(hash_login=True, login_conf=_realm(tmp_path)))
    c = TestClient(app)
    r = c.get("/3/Cloud")
    assert r.status_code == 401 and r.headers["www-authenticate"] == 'Basic realm="H2O"'
    for u, p in (("jenkins_user", "jenkins_pwd42"), ("obf_user", "s3cret!"), ("md5_user", "md5pass"),
                 ("crypt_user", "cpass")):
        assert c.get("/3/Cloud", headers=_basic(u, p)).status_code == 200, u
        assert c.get("/3/Cloud", headers=_basic(u, p + "x")).status_code == 401, u
    assert c.get("/3/Cloud", headers=_basic("nobody", "x")).status_code == 401
    assert c.request("TRACE", "/3/Cloud", headers=_basic("jenkins_user", "jenkins_pwd42")).status_code == 405
    # non-page requests to the login targets: 401 "Access denied. Please login."
    assert c.get("/login").status_code == 401


@pytest.mark.skipif(not os.path.exists(REF_REALM), reason="reference realm fixture not present")
def test_reference_realm_file():
    svc = security.HashLoginService(REF_REALM)
    assert svc.login("jenkins_user", "jenkins_pwd42") and not svc.login("jenkins_user", "x")


def test_form_auth_browser_flow(tmp_path, monkeypatch):
    app = create_app(login=security.LoginConfig(hash_login=True, login_conf=_realm(tmp_path), form_auth=True,
                                                session_timeout=5))
    c = TestClient(app)
    ua = {"User-Agent": "Mozilla/pyunit"}
    r = c.get("/flow/index.html", headers=ua, follow_redirects=False)
    assert r.status_code in (302, 303) and r.headers["location"].startswith("/login")   # pyunit_redirect_relative
    r = c.get("/login", headers=dict(ua, Accept="text/html"))
    assert r.status_code == 200 and "j_security_check" in r.text
    bad = c.post("/j_security_check", data={"j_username": "jenkins_user", "j_password": "no"}, headers=ua,
                 follow_redirects=False)
    assert bad.status_code == 303 and bad.headers["location"] == "/loginError"
    c.get("/flow/index.html", headers=ua, follow_redirects=False)    # pending session remembers the target
    ok = c.post("/j_security_check", data={"j_username": "jenkins_user", "j_password": "jenkins_pwd42"},
                headers=ua, follow_redirects=False)
    assert ok.status_code == 303 and ok.headers["location"] == "/flow/index.html"
    assert c.get("/3/Cloud", headers=ua).status_code == 200          # session cookie
    # non-browser clients still use Basic
    c2 = TestClient(app)
    assert c2.get("/3/Cloud").status_code == 401
    assert c2.get("/3/Cloud", headers=_basic("md5_user", "md5pass")).status_code == 200
    # idle session timeout
    t = [security.time.time()]
    monkeypatch.setattr(security.time, "time", lambda: t[0])
    assert c.get("/3/Cloud", headers=ua).status_code == 200
    t[0] += 6 * 60
    r = c.get("/3/Cloud", headers=ua, follow_redirects=False)
    assert r.status_code == 302 and r.headers["location"] == "/login"


def test_login_option_rules(tmp_path):
    realm = _realm(tmp_path)
    L = security.LoginConfig
    with pytest.raises(ValueError, match="Must specify -login_conf"):
        L(hash_login=True).validate()
    with pytest.raises(ValueError, match="Can only specify one"):
        L(hash_login=True, pam_login=True, login_conf=realm).validate()
    with pytest.raises(ValueError, match="Form-based authentication can only"):
        L(form_auth=True).validate()
    with pytest.raises(ValueError, match="Session timeout"):
        L(hash_login=True, login_conf=realm, session_timeout=3).validate()
    with pytest.raises(ValueError, match="File does not exist"):
        L(hash_login=True, login_conf=str(tmp_path / "missing")).validate()
    with pytest.raises(ValueError, match="JAAS|KDC"):
        L(kerberos_login=True, login_conf=realm).validate()
    with pytest.raises(ValueError, match="JAAS"):            # a realm file is not a JAAS LDAP config
        L(ldap_login=True, login_conf=realm).validate()
    with pytest.raises(SystemExit):
        main(["-form_auth"])
    assert not L().validate().enabled


def test_form_auth_anonymous_requests_leave_no_server_state(tmp_path):
    """Cookie-less browser requests keep their post-login target in a short-lived cookie: the session table stays
    empty however many arrive, and only a successful login adds (one) entry."""
    app = create_app(login=security.LoginConfig(hash_login=True, login_conf=_realm(tmp_path), form_auth=True))
    ua = {"User-Agent": "Mozilla/flood"}
    for i in range(300):
        r = TestClient(app).get(f"/3/Frames/f{i}", headers=ua, follow_redirects=False)
        assert r.status_code == 302
    assert len(security.install.sessions) == 0
    c = TestClient(app)
    c.get("/3/Cloud", headers=ua, follow_redirects=False)
    ok = c.post("/j_security_check", data={"j_username": "jenkins_user", "j_password": "jenkins_pwd42"}, headers=ua,
                follow_redirects=False)
    assert ok.status_code == 303 and ok.headers["location"] == "/3/Cloud"
    assert len(security.install.sessions) == 1


def test_form_auth_never_redirects_off_host(tmp_path):
    app = create_app(login=security.LoginConfig(hash_login=True, login_conf=_realm(tmp_path), form_auth=True))
    ua = {"User-Agent": "Mozilla/x"}
    for bad in ("//evil.example/x", "/\\evil.example", "https://evil.example/", "/%2F%2Fevil.example"):
        c = TestClient(app)
        c.cookies.set(security.TARGET_COOKIE, bad)
        ok = c.post("/j_security_check", data={"j_username": "jenkins_user", "j_password": "jenkins_pwd42"},
                    headers=ua, follow_redirects=False)
        assert ok.status_code == 303 and ok.headers["location"] == "/", (bad, ok.headers["location"])
    c = TestClient(app)
    c.get("//evil.example/x", headers=ua, follow_redirects=False)
    ok = c.post("/j_security_check", data={"j_username": "jenkins_user", "j_password": "jenkins_pwd42"}, headers=ua,
                follow_redirects=False)
    loc = ok.headers["location"]
    assert loc.startswith("/") and not loc.startswith("//"), loc
    # a bounded table even when sessions never expire (session_timeout 0)
    s = security._Sessions(0.0, cap=8)
    for _ in range(50):
        s.new(user="u")
    assert len(s) == 8


def test_secure_cookie_flag_over_https(tmp_path):
    app = create_app(login=security.LoginConfig(hash_login=True, login_conf=_realm(tmp_path), form_auth=True,
                                                secure_cookies=True))
    c = TestClient(app, base_url="https://testserver")
    ok = c.post("/j_security_check", data={"j_username": "jenkins_user", "j_password": "jenkins_pwd42"},
                headers={"User-Agent": "Mozilla/x"}, follow_redirects=False)
    assert "secure" in ok.headers["set-cookie"].lower()
