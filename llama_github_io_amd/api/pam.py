"""``-pam_login``: PAM authentication of the REST API (reference: ``h2o-jaas-pam/src/main/java/de/codedo/jaas/
PamLoginModule.java``, which ``H2O.java`` -pam_login loads from the JAAS file given by -login_conf).

The JAAS entry names the PAM service, as the reference's module requires (``PamLoginModule.java:62-66``)::

    pamloginmodule {
        de.codedo.jaas.PamLoginModule required
        service = "h2o";
    };

A login is one PAM transaction on the host's libpam (``pam_start`` -> ``pam_authenticate`` -> ``pam_acct_mgmt`` ->
``pam_end``) with a conversation that answers the password prompt (echo off) with the offered password and the
user-name prompt (echo on) with the user — what libpam4j's ``PAM.authenticate`` does for the reference. libpam is
called through ctypes (no PAM binding in the image). The extra option ``confdir`` selects a PAM configuration
directory other than /etc/pam.d (``pam_start_confdir``, Linux-PAM >= 1.4; the tests use it with ``pam_exec``).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import threading

PAM_SUCCESS = 0
PAM_PROMPT_ECHO_OFF, PAM_PROMPT_ECHO_ON, PAM_ERROR_MSG, PAM_TEXT_INFO = 1, 2, 3, 4
PAM_CONV_ERR = 19


class _Msg(ctypes.Structure):
    _fields_ = [("msg_style", ctypes.c_int), ("msg", ctypes.c_char_p)]


class _Resp(ctypes.Structure):
    _fields_ = [("resp", ctypes.c_void_p), ("resp_retcode", ctypes.c_int)]


_CONV = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.POINTER(_Msg)),
                         ctypes.POINTER(ctypes.POINTER(_Resp)), ctypes.c_void_p)


class _Conv(ctypes.Structure):
    _fields_ = [("conv", _CONV), ("appdata_ptr", ctypes.c_void_p)]


_lib = None
_lock = threading.Lock()


def _libs():
    global _lib
    with _lock:
        if _lib is None:
            name = ctypes.util.find_library("pam")
            if not name:
                raise RuntimeError("libpam is not installed on this host")
            pam = ctypes.CDLL(name)
            libc = ctypes.CDLL(ctypes.util.find_library("c"))
            libc.calloc.restype = ctypes.c_void_p
            libc.calloc.argtypes = [ctypes.c_size_t, ctypes.c_size_t]
            libc.strdup.restype = ctypes.c_void_p
            libc.strdup.argtypes = [ctypes.c_char_p]
            libc.free.argtypes = [ctypes.c_void_p]
            pam.pam_start.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(_Conv),
                                      ctypes.POINTER(ctypes.c_void_p)]
            pam.pam_authenticate.argtypes = [ctypes.c_void_p, ctypes.c_int]
            pam.pam_acct_mgmt.argtypes = [ctypes.c_void_p, ctypes.c_int]
            pam.pam_end.argtypes = [ctypes.c_void_p, ctypes.c_int]
            if hasattr(pam, "pam_start_confdir"):
                pam.pam_start_confdir.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(_Conv),
                                                  ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
            _lib = (pam, libc)
        return _lib


def authenticate(service: str, user: str, password: str, confdir: str | None = None) -> bool:
    """One PAM transaction; True when both authentication and account management succeed."""
    if not user or not password or "\0" in user or "\0" in password:
        return False
    pam, libc = _libs()
    u, pw = user.encode("utf-8"), password.encode("utf-8")

    def conv(n, msgs, resp, _data):
        arr = libc.calloc(n, ctypes.sizeof(_Resp))            # libpam frees the array and the strings
        if not arr:
            return PAM_CONV_ERR
        out = ctypes.cast(arr, ctypes.POINTER(_Resp))
        for i in range(n):
            style = msgs[i].contents.msg_style
            if style == PAM_PROMPT_ECHO_OFF:
                out[i].resp = libc.strdup(pw)
            elif style == PAM_PROMPT_ECHO_ON:
                out[i].resp = libc.strdup(u)
            elif style not in (PAM_ERROR_MSG, PAM_TEXT_INFO):
                for j in range(i):
                    if out[j].resp:
                        libc.free(out[j].resp)
                libc.free(arr)
                return PAM_CONV_ERR
        resp[0] = out
        return PAM_SUCCESS

    cb = _CONV(conv)                                         # kept alive for the whole transaction
    cv = _Conv(cb, None)
    h = ctypes.c_void_p()
    if confdir:
        if not hasattr(pam, "pam_start_confdir"):
            raise RuntimeError("this libpam has no pam_start_confdir (Linux-PAM < 1.4): drop the confdir option")
        rc = pam.pam_start_confdir(service.encode(), u, ctypes.byref(cv), confdir.encode(), ctypes.byref(h))
    else:
        rc = pam.pam_start(service.encode(), u, ctypes.byref(cv), ctypes.byref(h))
    if rc != PAM_SUCCESS:
        return False
    try:
        rc = pam.pam_authenticate(h, 0)
        if rc == PAM_SUCCESS:
            rc = pam.pam_acct_mgmt(h, 0)
        return rc == PAM_SUCCESS
    finally:
        pam.pam_end(h, rc)


class PamLoginService:
    """The JAAS ``PamLoginModule`` entry of a login config (``service`` required, as the reference)."""

    def __init__(self, login_conf: str, entry: str | None = None):
        from .ldap import parse_jaas
        with open(login_conf, encoding="utf-8") as fh:
            cfg = parse_jaas(fh.read())
        if not cfg:
            raise ValueError(f"{login_conf}: no JAAS login entry")
        name = entry or ("pamloginmodule" if "pamloginmodule" in cfg else next(iter(cfg)))
        o = cfg[name]
        if "PamLoginModule" not in o["module"]:
            raise ValueError(f"{login_conf}: entry {name} uses {o['module']}, not a PamLoginModule")
        if not o.get("service"):
            raise ValueError("Error: PAM service was not defined")
        self.service = o["service"]
        self.confdir = o.get("confdir") or None
        _libs()                                              # fail at startup when libpam is missing

    def login(self, user: str, password: str) -> bool:
        try:
            return authenticate(self.service, user, password, self.confdir)
        except (OSError, RuntimeError):
            return False
