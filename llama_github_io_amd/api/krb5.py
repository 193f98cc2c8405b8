"""Kerberos logins for the REST server: ``-kerberos_login`` (Basic credentials checked by a Kerberos AS exchange,
JAAS Krb5LoginModule) and ``-spnego_login`` (``Authorization: Negotiate`` tokens accepted with GSSAPI, Jetty's
SpnegoLoginService + SpnegoAuthenticator).

Reference: ``h2o-jetty-9/src/main/java/water/webserver/jetty9/Jetty9Helper.java:124-143`` (KERBEROS runs through a
JAASLoginService with the ``krb5loginmodule`` realm and Basic authentication; SPNEGO through SpnegoLoginService with
``-spnego_properties`` and a SpnegoAuthenticator), ``h2o-webserver-iface/.../LoginType.java:10-11``, and the Hadoop
driver's ``-kerberos_login`` / ``-spnego_login`` / ``-spnego_properties`` flags (``h2o-mapreduce-generic/.../
h2odriver.java:1210-1218``).

MI355X build, no JVM: the host's MIT Kerberos libraries are called through ctypes — ``libkrb5.so.3``
(``krb5_get_init_creds_password``: the password is proven to the KDC, nothing is stored) and
``libgssapi_krb5.so.2`` (``gss_accept_sec_context`` with the service keytab). KDC / realm come from the system
``krb5.conf``, or from the JAAS entry's ``realm`` + ``kdc`` options (a private krb5.conf is written for them);
the SPNEGO acceptor's keytab is the JAAS entry's ``keyTab`` (``KRB5_KTNAME``) and its principal the
``targetName`` of the spnego properties file (any keytab principal when absent).
"""
from __future__ import annotations

import atexit
import base64
import contextlib
import ctypes
import os
import tempfile
import threading

from .ldap import parse_jaas

_env_lock = threading.Lock()


def _load(names):
    for n in names:
        try:
            return ctypes.CDLL(n)
        except OSError:
            continue
    return None


_krb = None
_gss = None


def libkrb5():
    global _krb
    if _krb is None:
        lib = _load(["libkrb5.so.3", "libkrb5.so"])
        if lib is None:
            raise RuntimeError("libkrb5 (MIT Kerberos) is not installed on this host")
        vp, i32 = ctypes.c_void_p, ctypes.c_int32
        lib.krb5_init_context.argtypes = [ctypes.POINTER(vp)]
        lib.krb5_init_context.restype = i32
        lib.krb5_free_context.argtypes = [vp]
        lib.krb5_parse_name.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(vp)]
        lib.krb5_parse_name.restype = i32
        lib.krb5_free_principal.argtypes = [vp, vp]
        lib.krb5_get_init_creds_password.argtypes = [vp, vp, vp, ctypes.c_char_p, vp, vp, i32, ctypes.c_char_p, vp]
        lib.krb5_get_init_creds_password.restype = i32
        lib.krb5_free_cred_contents.argtypes = [vp, vp]
        lib.krb5_get_error_message.argtypes = [vp, i32]
        lib.krb5_get_error_message.restype = vp
        lib.krb5_free_error_message.argtypes = [vp, vp]
        _krb = lib
    return _krb


def _krb5_conf(realm: str, kdc: str) -> str:
    fd, path = tempfile.mkstemp(prefix="h2o-krb5-", suffix=".conf")
    with os.fdopen(fd, "w") as fh:
        fh.write(f"[libdefaults]\n default_realm = {realm}\n dns_lookup_kdc = false\n dns_lookup_realm = false\n"
                 f" kdc_timeout = 3s\n max_retries = 1\n[realms]\n {realm} = {{\n  kdc = {kdc}\n }}\n")
    atexit.register(_unlink, path)
    return path


def _unlink(path: str) -> None:
    with contextlib.suppress(OSError):
        os.unlink(path)


class _Context:
    """A krb5 context created under a given ``KRB5_CONFIG`` (the library reads the variable at init)."""

    def __init__(self, conf: str | None):
        self.lib = libkrb5()
        self.ctx = ctypes.c_void_p()
        with _env_lock:
            old = os.environ.get("KRB5_CONFIG")
            if conf:
                os.environ["KRB5_CONFIG"] = conf
            try:
                rc = self.lib.krb5_init_context(ctypes.byref(self.ctx))
            finally:
                if conf:
                    if old is None:
                        os.environ.pop("KRB5_CONFIG", None)
                    else:
                        os.environ["KRB5_CONFIG"] = old
        if rc:
            raise RuntimeError(f"krb5_init_context failed ({rc})")

    def error(self, code: int) -> str:
        p = self.lib.krb5_get_error_message(self.ctx, code)
        if not p:
            return f"krb5 error {code}"
        try:
            return ctypes.string_at(p).decode("utf-8", "replace")
        finally:
            self.lib.krb5_free_error_message(self.ctx, p)

    def close(self):
        if self.ctx:
            self.lib.krb5_free_context(self.ctx)
            self.ctx = ctypes.c_void_p()


def _entry(login_conf: str, want: str):
    with open(login_conf, encoding="utf-8") as fh:
        cfg = parse_jaas(fh.read())
    if not cfg:
        raise ValueError(f"{login_conf}: no JAAS login entry")
    for name, o in cfg.items():
        if "Krb5LoginModule" in o["module"] and (name == want or want not in cfg):
            return o
    raise ValueError(f"{login_conf}: no Krb5LoginModule entry")


class Krb5LoginService:
    """``-kerberos_login``: Basic credentials become a Kerberos AS exchange for ``user[@realm]`` (JAAS
    Krb5LoginModule semantics: the login succeeds iff the KDC issues a TGT for that password)."""

    def __init__(self, login_conf: str, entry: str = "krb5loginmodule"):
        o = _entry(login_conf, entry)
        self.realm = o.get("realm")
        self.kdc = o.get("kdc")
        self.conf = o.get("krb5Conf") or (_krb5_conf(self.realm, self.kdc) if self.realm and self.kdc else None)
        self.last_error = ""
        libkrb5()                                 # fail at startup when the library is missing

    def principal(self, user: str) -> str:
        return user if "@" in user or not self.realm else f"{user}@{self.realm}"

    def login(self, user: str, password: str) -> bool:
        if not user or not password:
            return False
        c = _Context(self.conf)
        princ = ctypes.c_void_p()
        creds = ctypes.create_string_buffer(1024)        # krb5_creds (zeroed; ~120 bytes on LP64)
        try:
            rc = c.lib.krb5_parse_name(c.ctx, self.principal(user).encode("utf-8"), ctypes.byref(princ))
            if rc:
                self.last_error = c.error(rc)
                return False
            rc = c.lib.krb5_get_init_creds_password(c.ctx, creds, princ, password.encode("utf-8"), None, None, 0,
                                                     None, None)
            if rc:
                self.last_error = c.error(rc)
                return False
            c.lib.krb5_free_cred_contents(c.ctx, creds)
            return True
        finally:
            if princ:
                c.lib.krb5_free_principal(c.ctx, princ)
            c.close()


# ---- GSSAPI acceptor (SPNEGO)

class _Buf(ctypes.Structure):
    _fields_ = [("length", ctypes.c_size_t), ("value", ctypes.c_void_p)]


GSS_S_COMPLETE = 0
GSS_S_CONTINUE_NEEDED = 1


def libgss():
    global _gss
    if _gss is None:
        lib = _load(["libgssapi_krb5.so.2", "libgssapi_krb5.so"])
        if lib is None:
            raise RuntimeError("libgssapi_krb5 (MIT Kerberos GSSAPI) is not installed on this host")
        vp, u32 = ctypes.c_void_p, ctypes.c_uint32
        pu32 = ctypes.POINTER(u32)
        lib.gss_import_name.argtypes = [pu32, ctypes.POINTER(_Buf), vp, ctypes.POINTER(vp)]
        lib.gss_import_name.restype = u32
        lib.gss_acquire_cred.argtypes = [pu32, vp, u32, vp, ctypes.c_int, ctypes.POINTER(vp), vp, pu32]
        lib.gss_acquire_cred.restype = u32
        lib.gss_accept_sec_context.argtypes = [pu32, ctypes.POINTER(vp), vp, ctypes.POINTER(_Buf), vp,
                                               ctypes.POINTER(vp), vp, ctypes.POINTER(_Buf), pu32, pu32, vp]
        lib.gss_accept_sec_context.restype = u32
        lib.gss_display_name.argtypes = [pu32, vp, ctypes.POINTER(_Buf), vp]
        lib.gss_display_name.restype = u32
        lib.gss_release_buffer.argtypes = [pu32, ctypes.POINTER(_Buf)]
        lib.gss_release_name.argtypes = [pu32, ctypes.POINTER(vp)]
        lib.gss_release_cred.argtypes = [pu32, ctypes.POINTER(vp)]
        lib.gss_delete_sec_context.argtypes = [pu32, ctypes.POINTER(vp), vp]
        _gss = lib
    return _gss


def _oid(lib, name: str):
    return ctypes.c_void_p.in_dll(lib, name)


def read_properties(path: str) -> dict:
    """Java .properties (``key=value`` / ``key: value``, ``#`` / ``!`` comments)."""
    out = {}
    with open(path, encoding="utf-8") as fh:
        for line in fh:
            s = line.strip()
            if not s or s[0] in "#!":
                continue
            cut = min([i for i in (s.find("="), s.find(":")) if i >= 0], default=len(s))
            out[s[:cut].strip()] = s[cut + 1:].strip()
    return out


class SpnegoService:
    """``-spnego_login``: one GSSAPI acceptor step per ``Authorization: Negotiate`` token. ``accept`` returns the
    client principal (or None) and the reply token for ``WWW-Authenticate: Negotiate <token>``."""

    def __init__(self, login_conf: str | None, spnego_properties: str | None):
        props = read_properties(spnego_properties) if spnego_properties else {}
        self.target = props.get("targetName") or None
        o = {}
        if login_conf:
            try:
                o = _entry(login_conf, "com.sun.security.jgss.accept")
            except ValueError:
                o = {}
        self.keytab = o.get("keyTab") or props.get("keyTab") or None
        if self.target is None and o.get("principal"):
            self.target = o["principal"]
        self.last_error = ""
        libgss()

    def accept(self, token: bytes):
        lib = libgss()
        minor = ctypes.c_uint32()
        cred, name, ctx, src = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        out = _Buf(0, None)
        with _env_lock:
            old = os.environ.get("KRB5_KTNAME")
            if self.keytab:
                os.environ["KRB5_KTNAME"] = self.keytab
            try:
                if self.target:
                    b = ctypes.create_string_buffer(self.target.encode("utf-8"))
                    nb = _Buf(len(self.target), ctypes.cast(b, ctypes.c_void_p))
                    nt = _oid(lib, "GSS_KRB5_NT_PRINCIPAL_NAME" if "@" in self.target or "/" in self.target
                              else "GSS_C_NT_HOSTBASED_SERVICE")
                    if lib.gss_import_name(ctypes.byref(minor), ctypes.byref(nb), nt, ctypes.byref(name)):
                        self.last_error = "gss_import_name failed"
                        return None, None
                # GSS_C_ACCEPT = 2, GSS_C_INDEFINITE = 0xffffffff
                major = lib.gss_acquire_cred(ctypes.byref(minor), name if self.target else None, 0xFFFFFFFF, None,
                                             2, ctypes.byref(cred), None, None)
            finally:
                if self.keytab:
                    if old is None:
                        os.environ.pop("KRB5_KTNAME", None)
                    else:
                        os.environ["KRB5_KTNAME"] = old
        try:
            if major:
                self.last_error = f"gss_acquire_cred failed (major {major:#x}, minor {minor.value})"
                return None, None
            tb = ctypes.create_string_buffer(token, len(token))
            inp = _Buf(len(token), ctypes.cast(tb, ctypes.c_void_p))
            major = lib.gss_accept_sec_context(ctypes.byref(minor), ctypes.byref(ctx), cred, ctypes.byref(inp), None,
                                               ctypes.byref(src), None, ctypes.byref(out), None, None, None)
            reply = ctypes.string_at(out.value, out.length) if out.length else None
            if major != GSS_S_COMPLETE:
                # one round trip only (Kerberos SPNEGO completes in one); anything else is a failed login
                self.last_error = f"gss_accept_sec_context failed (major {major:#x}, minor {minor.value})"
                return None, reply
            disp = _Buf(0, None)
            if lib.gss_display_name(ctypes.byref(minor), src, ctypes.byref(disp), None):
                return None, reply
            user = ctypes.string_at(disp.value, disp.length).decode("utf-8", "replace")
            lib.gss_release_buffer(ctypes.byref(minor), ctypes.byref(disp))
            return user, reply
        finally:
            if out.length:
                lib.gss_release_buffer(ctypes.byref(minor), ctypes.byref(out))
            if ctx:
                lib.gss_delete_sec_context(ctypes.byref(minor), ctypes.byref(ctx), None)
            if src:
                lib.gss_release_name(ctypes.byref(minor), ctypes.byref(src))
            if name:
                lib.gss_release_name(ctypes.byref(minor), ctypes.byref(name))
            if cred:
                lib.gss_release_cred(ctypes.byref(minor), ctypes.byref(cred))


def negotiate_token(headers) -> bytes | None:
    h = headers.get("authorization") or ""
    if not h.lower().startswith("negotiate "):
        return None
    try:
        return base64.b64decode(h[10:].strip(), validate=True)
    except ValueError:
        return b""
