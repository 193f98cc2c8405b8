"""REST server login: Jetty HashLoginService + Basic / Form authentication for every route.

Reference behaviour (re-expressed for the FastAPI server, no Jetty):
  * ``-hash_login -login_conf <realm file>`` (``h2o-core/src/main/java/water/H2O.java:244,755,870-910``): one
    login method at most, a login_conf is required, ``-form_auth`` only with a login method, ``-session_timeout``
    only with ``-form_auth``.
  * every path is constrained to any authenticated user, realm "H2O"
    (``h2o-jetty-9/.../Jetty9Helper.java:118-186`` authWrapper: HashLoginService + BasicAuthenticator).
  * with ``-form_auth`` browsers (User-Agent ``Mozilla/`` or ``Opera/``) get Form authentication, every other client
    Basic (``Jetty9DelegatingAuthenticator.java``): an unauthenticated page request is redirected to the relative
    ``/login``; the form posts ``j_username`` / ``j_password`` to ``/j_security_check``; a failure lands on
    ``/loginError``; the session expires after ``session_timeout`` idle minutes.
  * ``/login`` and ``/loginError`` answer the form to page requests (Accept: text/html) and 401 "Access denied.
    Please login." otherwise (``water/webserver/H2OHttpViewImpl.java:112-152``); TRACE is refused with 405 (gateHandler).
The realm file is Jetty's PropertyUserStore format, ``user: credential[, role ...]`` (``#`` comments), with a
credential in plain text or Jetty's ``OBF:`` / ``MD5:`` / ``CRYPT:`` forms (``h2o-assemblies/main/tests/python/
realm.properties`` is a plain one). ``-ldap_login -login_conf <JAAS file>`` authenticates against an LDAP server with
Jetty LdapLoginModule's semantics (:mod:`.ldap`); ``-pam_login`` through the host's libpam as h2o-jaas-pam's
PamLoginModule (:mod:`.pam`). ``-kerberos_login`` checks Basic credentials with a Kerberos AS exchange (JAAS
Krb5LoginModule) and ``-spnego_login`` accepts ``Authorization: Negotiate`` tokens with GSSAPI (Jetty's
SpnegoAuthenticator; ``-spnego_properties`` names the ``targetName``) — both through the host's MIT Kerberos
libraries (:mod:`.krb5`).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import secrets
import threading
import time
from dataclasses import dataclass
from urllib.parse import parse_qs, quote

REALM = "H2O"


# ---- Jetty credential forms (org.eclipse.jetty.util.security.Password / Credential)
def _to36(n: int) -> str:
    d = "0123456789abcdefghijklmnopqrstuvwxyz"
    s = ""
    while n:
        s = d[n % 36] + s
        n //= 36
    return s or "0"


def obfuscate(password: str) -> str:
    """Jetty ``Password.obfuscate``: a reversible ``OBF:`` encoding (not encryption)."""
    b = password.encode("utf-8")
    out = ["OBF:"]
    for i in range(len(b)):
        b1, b2 = b[i], b[len(b) - (i + 1)]
        s1, s2 = (b1 - 256 if b1 > 127 else b1), (b2 - 256 if b2 > 127 else b2)
        if s1 < 0 or s2 < 0:
            x = _to36(b1 * 256 + b2)
            out.append("U0000"[:5 - len(x)] + x)
        else:
            x = _to36((127 + s1 + s2) * 256 + (127 + s1 - s2))
            out.append("000"[:4 - len(x)] + x)
    return "".join(out)


def deobfuscate(s: str) -> str:
    if s.startswith("OBF:"):
        s = s[4:]
    b = bytearray()
    i = 0
    while i < len(s):
        if s[i] == "U":
            i += 1
            b.append((int(s[i:i + 4], 36) >> 8) & 0xFF)
        else:
            i0 = int(s[i:i + 4], 36)
            b.append(((i0 // 256 + i0 % 256 - 254) // 2) & 0xFF)
        i += 4
    return b.decode("utf-8")


def _crypt(password: str, salt: str) -> str:
    try:
        import crypt as _c   # the traditional DES crypt(3) Jetty's UnixCrypt implements
    except ImportError as e:   # pragma: no cover - Python >= 3.13
        raise RuntimeError("CRYPT: credentials need the crypt module") from e
    return _c.crypt(password, salt)


def check_credential(stored: str, password: str) -> bool:
    """Jetty Credential.check for a stored ``plain`` / ``OBF:`` / ``MD5:`` / ``CRYPT:`` credential."""
    if stored.startswith("OBF:"):
        expect = deobfuscate(stored)
        return hmac.compare_digest(expect.encode(), password.encode())
    if stored.startswith("MD5:"):
        return hmac.compare_digest(stored[4:].lower(), hashlib.md5(password.encode("utf-8")).hexdigest())
    if stored.startswith("CRYPT:"):
        c = stored[6:]
        return hmac.compare_digest(c, _crypt(password, c[:2]))
    return hmac.compare_digest(stored.encode(), password.encode())


class HashLoginService:
    """Users of a Jetty PropertyUserStore realm file."""

    def __init__(self, path: str):
        self.path = path
        self.users: dict[str, tuple[str, list[str]]] = {}
        with open(path, encoding="utf-8") as fh:
            for line in fh:
                line = line.strip()
                if not line or line.startswith("#") or ":" not in line:
                    continue
                user, rest = line.split(":", 1)
                parts = [p.strip() for p in rest.split(",")]
                self.users[user.strip()] = (parts[0], [r for r in parts[1:] if r])

    def login(self, user: str, password: str) -> bool:
        u = self.users.get(user)
        return u is not None and check_credential(u[0], password)


@dataclass
class LoginConfig:
    hash_login: bool = False
    ldap_login: bool = False
    kerberos_login: bool = False
    spnego_login: bool = False
    pam_login: bool = False
    login_conf: str | None = None
    form_auth: bool = False
    session_timeout: int = 0          # minutes of inactivity (form_auth); 0 = no timeout
    secure_cookies: bool = False      # the server speaks HTTPS (-jks): session cookies carry the Secure flag
    spnego_properties: str | None = None   # -spnego_properties: Java properties with the acceptor's targetName

    def validate(self) -> "LoginConfig":
        import os
        n = sum(bool(v) for v in (self.hash_login, self.ldap_login, self.kerberos_login, self.spnego_login,
                                  self.pam_login))
        if self.login_conf is not None and not os.path.exists(self.login_conf):
            raise ValueError(f"File does not exist: {self.login_conf}")
        if n > 1:
            raise ValueError("Can only specify one of -hash_login, -ldap_login, -kerberos_login, -spnego_login and "
                             "-pam_login")
        if n and self.login_conf is None:
            raise ValueError("Must specify -login_conf argument")
        if not n and self.form_auth:
            raise ValueError("No login method was specified. Form-based authentication can only be used in conjunction "
                             "with of a LoginService.")
        if self.session_timeout and not self.form_auth:
            raise ValueError("Session timeout can only be enabled for Form based authentication (use -form_auth)")
        if self.spnego_properties is not None and not os.path.exists(self.spnego_properties):
            raise ValueError(f"File does not exist: {self.spnego_properties}")
        if self.ldap_login or self.pam_login or self.kerberos_login or self.spnego_login:
            try:
                self.service()                      # a malformed JAAS config fails at startup, not at first login
            except RuntimeError as e:               # the host lacks the login's native library
                raise ValueError(str(e)) from None
        return self

    @property
    def enabled(self) -> bool:
        return self.hash_login or self.ldap_login or self.pam_login or self.kerberos_login or self.spnego_login

    def service(self):
        if self.spnego_login:
            from .krb5 import SpnegoService
            return SpnegoService(self.login_conf, self.spnego_properties)
        if self.kerberos_login:
            from .krb5 import Krb5LoginService
            return _CachedLogin(Krb5LoginService(self.login_conf))
        if self.ldap_login:
            from .ldap import LdapLoginService
            return _CachedLogin(LdapLoginService(self.login_conf))
        if self.pam_login:
            from .pam import PamLoginService
            return _CachedLogin(PamLoginService(self.login_conf))
        return HashLoginService(self.login_conf)


class _CachedLogin:
    """Remembers successful logins of a remote login service for ``ttl_s`` (Basic auth re-sends the credentials on
    every request; without this each REST call would be an LDAP round trip). Only a salted digest of the credentials
    is kept."""

    def __init__(self, svc, ttl_s: float = 60.0, cap: int = 1024):
        self.svc, self.ttl_s, self.cap = svc, ttl_s, cap
        self._salt = secrets.token_bytes(16)
        self._ok: dict[bytes, float] = {}
        self._lock = threading.Lock()

    def login(self, user: str, password: str) -> bool:
        k = hashlib.sha256(self._salt + user.encode("utf-8") + b"\0" + password.encode("utf-8")).digest()
        now = time.time()
        with self._lock:
            t = self._ok.get(k)
            if t is not None and now - t < self.ttl_s:
                return True
        if not self.svc.login(user, password):
            return False
        with self._lock:
            if len(self._ok) >= self.cap:
                self._ok.clear()
            self._ok[k] = now
        return True


_FORM = """<!DOCTYPE html><html><head><title>H2O Login</title></head><body>
<h1>H2O</h1>{msg}
<form method="POST" action="/j_security_check">
<label>Username <input type="text" name="j_username" autofocus></label>
<label>Password <input type="password" name="j_password"></label>
<input type="submit" value="Login"></form></body></html>"""


class _Sessions:
    """Logged-in sessions only (the pre-login target travels in a short-lived cookie, never here). Bounded: expired
    entries are swept on every new session and at most ``cap`` live ones are kept (the least recently seen go)."""

    def __init__(self, timeout_s: float, cap: int = 4096):
        self.timeout_s = timeout_s
        self.cap = int(cap)
        self._lock = threading.Lock()
        self._s: dict[str, dict] = {}

    def new(self, **kw) -> str:
        sid = secrets.token_urlsafe(24)
        now = time.time()
        with self._lock:
            if self.timeout_s:
                for k in [k for k, v in self._s.items() if now - v["seen"] > self.timeout_s]:
                    del self._s[k]
            while len(self._s) >= self.cap:
                del self._s[min(self._s, key=lambda k: self._s[k]["seen"])]
            self._s[sid] = dict(kw, seen=now)
        return sid

    def __len__(self) -> int:
        with self._lock:
            return len(self._s)

    def get(self, sid: str | None) -> dict | None:
        if not sid:
            return None
        with self._lock:
            s = self._s.get(sid)
            if s is None:
                return None
            now = time.time()
            if self.timeout_s and now - s["seen"] > self.timeout_s:
                del self._s[sid]
                return None
            s["seen"] = now
            return s


TARGET_COOKIE = "H2O_LOGIN_TARGET"


def _safe_target(t: str | None) -> str:
    """A post-login redirect target that stays on this server: a single-slash absolute path, or '/'."""
    from urllib.parse import unquote
    if not t:
        return "/"
    raw = unquote(t)
    if not raw.startswith("/") or raw.startswith("//") or "\\" in raw or ":" in raw.split("?", 1)[0] or \
            any(ord(ch) < 32 for ch in raw):
        return "/"
    return t


def _is_browser(headers) -> bool:
    ua = headers.get("user-agent") or ""
    return ua.startswith("Mozilla/") or ua.startswith("Opera/")


def _basic_user(headers) -> tuple[str, str] | None:
    h = headers.get("authorization") or ""
    if not h.lower().startswith("basic "):
        return None
    try:
        user, _, pw = base64.b64decode(h[6:].strip()).decode("utf-8").partition(":")
    except Exception:
        return None
    return user, pw


def install(app, cfg: LoginConfig) -> None:
    """Constrain every route of ``app`` to authenticated users (no-op when no login method is configured)."""
    if not cfg.enabled:
        return
    from starlette.concurrency import run_in_threadpool
    from starlette.responses import HTMLResponse, JSONResponse, RedirectResponse, Response
    svc = cfg.service()
    sessions = _Sessions(60.0 * cfg.session_timeout)
    install.sessions = sessions                  # (tests: the live session table)
    cookie = "JSESSIONID"
    secure = bool(cfg.secure_cookies)

    def unauthorized(msg="Access denied. Please login."):
        return JSONResponse(status_code=401, content={"http_status": 401, "msg": msg},
                            headers={"WWW-Authenticate": f'Basic realm="{REALM}"'})

    @app.middleware("http")
    async def login_gate(request, call_next):
        if request.method == "TRACE":
            return Response(status_code=405)
        from . import cloud
        if cloud.is_internal(request.headers):     # a cloud rank re-running a request rank 0 already authenticated
            return await call_next(request)
        path = request.url.path
        headers = request.headers
        page = "text/html" in (headers.get("accept") or "")
        if path in ("/login", "/loginError"):
            if page:
                msg = "<p>Invalid username or password.</p>" if path == "/loginError" else ""
                return HTMLResponse(_FORM.format(msg=msg))
            return unauthorized()
        if path == "/j_security_check" and request.method == "POST" and cfg.form_auth:
            form = parse_qs((await request.body()).decode("utf-8", "replace"))
            user = (form.get("j_username") or [""])[0]
            pw = (form.get("j_password") or [""])[0]
            if not await run_in_threadpool(svc.login, user, pw):
                return RedirectResponse("/loginError", status_code=303)
            r = RedirectResponse(_safe_target(request.cookies.get(TARGET_COOKIE)), status_code=303)
            r.set_cookie(cookie, sessions.new(user=user), httponly=True, path="/", secure=secure)
            r.delete_cookie(TARGET_COOKIE, path="/")
            return r
        s = sessions.get(request.cookies.get(cookie))
        if s is not None and s.get("user"):
            return await call_next(request)
        if cfg.spnego_login:
            # SpnegoAuthenticator: a Negotiate token is accepted with GSSAPI, else 401 + "WWW-Authenticate: Negotiate"
            from .krb5 import negotiate_token
            tok = negotiate_token(headers)
            reply = None
            if tok:
                user, reply = await run_in_threadpool(svc.accept, tok)
                if user:
                    r = await call_next(request)
                    if reply:
                        r.headers["WWW-Authenticate"] = "Negotiate " + base64.b64encode(reply).decode("ascii")
                    return r
            return JSONResponse(status_code=401, content={"http_status": 401, "msg": "Access denied. Please login."},
                                headers={"WWW-Authenticate": "Negotiate" + (
                                    " " + base64.b64encode(reply).decode("ascii") if reply else "")})
        cred = _basic_user(headers)
        if cred is not None and await run_in_threadpool(svc.login, *cred):
            return await call_next(request)
        if cfg.form_auth and _is_browser(headers):
            # FormAuthenticator: remember the requested URI (a short-lived cookie: no server state per anonymous
            # request), send the browser to the form
            target = _safe_target(quote(path + (("?" + request.url.query) if request.url.query else ""), safe="/?=&"))
            r = RedirectResponse("/login", status_code=302)
            r.set_cookie(TARGET_COOKIE, target, max_age=600, httponly=True, path="/", secure=secure)
            return r
        return unauthorized()
