"""``-ldap_login``: LDAP authentication of the REST API (reference: ``H2O.java`` -ldap_login / -login_conf, which
hands the JAAS config to Jetty's ``LdapLoginModule`` via ``h2o-jetty-9/.../jaas/spi/LdapLoginModule.java``).

The login config is the JAAS file users already have for H2O::

    ldaploginmodule {
        org.eclipse.jetty.plus.jaas.spi.LdapLoginModule required
        hostname="ldap.example.com" port="389" useLdaps="false"
        bindDn="cn=admin,dc=example,dc=com" bindPassword="secret"
        forceBindingLogin="true"
        userBaseDn="ou=users,dc=example,dc=com" userIdAttribute="uid" userObjectClass="inetOrgPerson"
        userPasswordAttribute="userPassword";
    };

and the two login paths of Jetty's LdapLoginModule:

* ``forceBindingLogin="true"``: find the user's entry (``(&(objectClass=<userObjectClass>)(<userIdAttribute>=<user>))``
  under ``userBaseDn``, bound as ``bindDn`` or anonymously), then BIND as that DN with the offered password;
* otherwise: read the entry's ``userPasswordAttribute`` (bound as ``bindDn``) and check the offered password against it
  (``{MD5}`` / ``{SHA}`` / ``{SSHA}`` base64 digests, a Jetty credential ``MD5:`` / ``OBF:``, or plain).

The LDAPv3 client is a small BER codec over a socket (RFC 4511 BindRequest / SearchRequest, simple authentication);
no LDAP library is in the image. ``useLdaps="true"`` wraps the socket in TLS with certificate and host-name
verification against the system trust store, or against the CA bundle named by the extra option ``caFile``.
Kerberos / SPNEGO stay refused (PAM: :mod:`.pam`).
"""
from __future__ import annotations

import base64
import hashlib
import re
import socket
import ssl


# ------------------------------------------------------------------------------------------------ BER codec
def _len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def tlv(tag: int, value: bytes) -> bytes:
    return bytes([tag]) + _len(len(value)) + value


def ber_int(v: int, tag: int = 0x02) -> bytes:
    return tlv(tag, v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big", signed=True))


def ber_str(s, tag: int = 0x04) -> bytes:
    return tlv(tag, s.encode("utf-8") if isinstance(s, str) else bytes(s))


def seq(*parts, tag: int = 0x30) -> bytes:
    return tlv(tag, b"".join(parts))


def read_tlv(buf: bytes, i: int = 0):
    """(tag, value, next index) of the TLV at ``buf[i:]``."""
    if i + 2 > len(buf):
        raise ValueError("truncated BER element")
    tag, n, j = buf[i], buf[i + 1], i + 2
    if n & 0x80:
        k = n & 0x7F
        n = int.from_bytes(buf[j:j + k], "big")
        j += k
    if j + n > len(buf):
        raise ValueError("truncated BER element")
    return tag, buf[j:j + n], j + n


def read_all(buf: bytes):
    out, i = [], 0
    while i < len(buf):
        t, v, i = read_tlv(buf, i)
        out.append((t, v))
    return out


def _recv_exact(sock, n: int) -> bytes:
    out = b""
    while len(out) < n:
        c = sock.recv(n - len(out))
        if not c:
            raise ConnectionError("LDAP peer closed the connection")
        out += c
    return out


def recv_msg(sock, limit: int = 16 << 20) -> bytes:
    """One complete BER element (an LDAPMessage) from the socket."""
    head = _recv_exact(sock, 2)
    n = head[1]
    if n & 0x80:
        lb = _recv_exact(sock, n & 0x7F)
        head += lb
        n = int.from_bytes(lb, "big")
    if n > limit:
        raise ValueError(f"LDAP message of {n} bytes refused")
    return head + _recv_exact(sock, n)


def _int(v: bytes) -> int:
    return int.from_bytes(v, "big", signed=True)


# ------------------------------------------------------------------------------------------------ client
class LdapClient:
    """A synchronous LDAPv3 connection (one outstanding operation at a time)."""

    def __init__(self, host: str, port: int, use_ssl: bool = False, timeout: float = 10.0, ca_file: str | None = None):
        s = socket.create_connection((host, port), timeout=timeout)
        if use_ssl:
            ctx = ssl.create_default_context(cafile=ca_file)
            s = ctx.wrap_socket(s, server_hostname=host)
        self.sock = s
        self.mid = 0

    def close(self):
        try:
            self.sock.sendall(seq(ber_int(self._next()), tlv(0x42, b"")))   # UnbindRequest
        except OSError:
            pass
        self.sock.close()

    def _next(self) -> int:
        self.mid += 1
        return self.mid

    def _response(self):
        _, body, _ = read_tlv(recv_msg(self.sock))
        parts = read_all(body)
        if len(parts) < 2:
            raise ValueError("malformed LDAP response")
        return parts[1]

    def bind(self, dn: str, password: str) -> int:
        """Simple bind; returns the LDAP resultCode (0 = success)."""
        self.sock.sendall(seq(ber_int(self._next()),
                              seq(ber_int(3), ber_str(dn), ber_str(password, 0x80), tag=0x60)))
        tag, op = self._response()
        if tag != 0x61:
            raise ValueError(f"unexpected LDAP response tag {tag:#x}")
        return _int(read_all(op)[0][1])

    def search(self, base: str, flt: bytes, attrs=()) -> list:
        """Whole-subtree search; returns [(dn, {attr (lower case): [values]})]."""
        self.sock.sendall(seq(ber_int(self._next()),
                              seq(ber_str(base), tlv(0x0A, b"\x02"), tlv(0x0A, b"\x00"), ber_int(0), ber_int(0),
                                  tlv(0x01, b"\x00"), flt, seq(*[ber_str(a) for a in attrs]), tag=0x63)))
        out = []
        while True:
            tag, op = self._response()
            if tag == 0x64:                                  # SearchResultEntry
                fields = read_all(op)
                got = {}
                for _, av in read_all(fields[1][1]):
                    name, vals = read_all(av)
                    got[name[1].decode("utf-8").lower()] = [v for _, v in read_all(vals[1])]
                out.append((fields[0][1].decode("utf-8"), got))
            elif tag == 0x65:                                # SearchResultDone
                rc = _int(read_all(op)[0][1])
                if rc not in (0, 32):                        # success / noSuchObject
                    raise ValueError(f"LDAP search failed (resultCode {rc})")
                return out
            # SearchResultReference (0x73) is ignored: referrals are not chased


def eq_filter(attr: str, value: str) -> bytes:
    """equalityMatch filter; the value travels as an OCTET STRING, so no RFC 4515 escaping is involved."""
    return seq(ber_str(attr), ber_str(value), tag=0xA3)


def and_filter(*fs: bytes) -> bytes:
    return tlv(0xA0, b"".join(fs))


# ------------------------------------------------------------------------------------------------ JAAS config
def parse_jaas(text: str) -> dict:
    """{entry name: {"module": class, "flag": flag, **options}} of a JAAS login configuration."""
    text = re.sub(r"//[^\n]*|/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"([\w.-]+)\s*\{(.*?)\}\s*;", text, flags=re.S):
        body = m.group(2).strip().rstrip(";")
        head = re.match(r"\s*([\w.$]+)\s+(required|requisite|sufficient|optional)\b", body)
        if not head:
            continue
        opts = {k: (q if q or not u else u) for k, q, u in
                re.findall(r'(\w+)\s*=\s*(?:"([^"]*)"|([^\s;"]+))', body[head.end():])}
        out[m.group(1)] = dict(opts, module=head.group(1), flag=head.group(2))
    return out


def check_stored(stored: bytes, password: str) -> bool:
    """userPassword attribute vs the offered password: LDAP {MD5} / {SHA} / {SSHA} digests, Jetty credentials, plain."""
    import hmac
    s = stored.decode("utf-8", "replace")
    pw = password.encode("utf-8")
    up = s.upper()
    try:
        if up.startswith("{MD5}"):
            return hmac.compare_digest(base64.b64decode(s[5:]), hashlib.md5(pw).digest())
        if up.startswith("{SHA}"):
            return hmac.compare_digest(base64.b64decode(s[5:]), hashlib.sha1(pw).digest())
        if up.startswith("{SSHA}"):
            raw = base64.b64decode(s[6:])
            return len(raw) > 20 and hmac.compare_digest(hashlib.sha1(pw + raw[20:]).digest(), raw[:20])
    except ValueError:
        return False
    from .security import check_credential
    return check_credential(s, password)


class LdapLoginService:
    """Jetty LdapLoginModule semantics over :class:`LdapClient` (see the module note)."""

    def __init__(self, login_conf: str, entry: str | None = None):
        with open(login_conf, encoding="utf-8") as fh:
            cfg = parse_jaas(fh.read())
        if not cfg:
            raise ValueError(f"{login_conf}: no JAAS login entry")
        name = entry or ("ldaploginmodule" if "ldaploginmodule" in cfg else next(iter(cfg)))
        if name not in cfg:
            raise ValueError(f"{login_conf}: no JAAS entry {name!r}")
        o = cfg[name]
        if "LdapLoginModule" not in o["module"]:
            raise ValueError(f"{login_conf}: entry {name} uses {o['module']}, not an LdapLoginModule")
        if o.get("authenticationMethod", "simple").lower() != "simple":
            raise ValueError('only authenticationMethod="simple" LDAP binds are supported')
        self.host = o.get("hostname", "localhost")
        self.ssl = o.get("useLdaps", "false").lower() == "true"
        self.port = int(o.get("port", "636" if self.ssl else "389"))
        self.ca_file = o.get("caFile") or None
        self.bind_dn, self.bind_pw = o.get("bindDn"), o.get("bindPassword", "")
        self.force_binding = o.get("forceBindingLogin", "false").lower() == "true"
        self.user_base = o.get("userBaseDn", "")
        self.user_id = o.get("userIdAttribute", "cn")
        self.user_pw_attr = o.get("userPasswordAttribute", "userPassword")
        self.user_oc = o.get("userObjectClass", "inetOrgPerson")
        self.timeout = float(o.get("timeout", "10"))

    def _find(self, c: LdapClient, user: str):
        if self.bind_dn and c.bind(self.bind_dn, self.bind_pw) != 0:
            raise PermissionError("LDAP bindDn rejected")
        flt = and_filter(eq_filter("objectClass", self.user_oc), eq_filter(self.user_id, user))
        hits = c.search(self.user_base, flt, [] if self.force_binding else [self.user_pw_attr])
        return hits[0] if len(hits) == 1 else None

    def login(self, user: str, password: str) -> bool:
        # an empty password would make a simple bind "unauthenticated" and succeed (RFC 4513 5.1.2)
        if not user or not password:
            return False
        try:
            c = LdapClient(self.host, self.port, self.ssl, self.timeout, self.ca_file)
        except (OSError, ssl.SSLError):
            return False
        try:
            hit = self._find(c, user)
            if hit is None:
                return False
            dn, attrs = hit
            if self.force_binding:
                return c.bind(dn, password) == 0
            return any(check_stored(v, password) for v in attrs.get(self.user_pw_attr.lower()) or [])
        except (OSError, ValueError, PermissionError, IndexError, UnicodeDecodeError):
            return False
        finally:
            c.close()
