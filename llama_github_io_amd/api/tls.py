"""HTTPS for the REST server from a Java KeyStore (``-jks <keystore> -jks_pass <password> [-jks_alias <alias> |
-hostname_as_jks_alias]``; reference: ``h2o-core/src/main/java/water/H2O.java:130-160`` options, default password
``h2oh2o`` (``H2O.java:45``), ``h2o-jetty-9/.../Jetty9Helper.java`` SslContextFactory over the keystore).

The JKS file (magic 0xFEEDFEED, version 2) is read natively here: a private-key entry's key is unsealed with the
JDK's proprietary KeyProtector (OID 1.3.6.1.4.1.42.2.17.1.1: salt || key XOR SHA-1 keystream of password UTF-16BE
chained from the salt || SHA-1(password || key) check) into its PKCS#8 DER, the certificate chain is taken as
X.509 DER, and both are handed to the TLS stack as PEM. The keystore's integrity digest (SHA-1 over the password,
"Mighty Aphrodite" and the body) verifies the password first."""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import socket
import struct
import tempfile
from dataclasses import dataclass, field

DEFAULT_JKS_PASS = "h2oh2o"
_KEY_PROTECTOR_OID = bytes.fromhex("2b060104012a021101 01".replace(" ", ""))   # 1.3.6.1.4.1.42.2.17.1.1


@dataclass
class KeyEntry:
    alias: str
    key_der: bytes                      # PKCS#8 PrivateKeyInfo
    chain_der: list = field(default_factory=list)


@dataclass
class JavaKeyStore:
    keys: dict
    certs: dict                         # trusted certificate entries: alias -> DER


def _der_read(b: bytes, off: int):
    tag = b[off]
    ln = b[off + 1]
    off += 2
    if ln & 0x80:
        n = ln & 0x7F
        ln = int.from_bytes(b[off:off + n], "big")
        off += n
    return tag, b[off:off + ln], off + ln


def _unseal(protected: bytes, password: str) -> bytes:
    tag, seq, _ = _der_read(protected, 0)            # EncryptedPrivateKeyInfo ::= SEQUENCE { alg, OCTET STRING }
    _, alg, o = _der_read(seq, 0)
    _, oid, _ = _der_read(alg, 0)
    if oid != _KEY_PROTECTOR_OID:
        raise ValueError("unsupported JKS key protection (only the JDK KeyProtector)")
    _, enc, _ = _der_read(seq, o)
    salt, body, check = enc[:20], enc[20:-20], enc[-20:]
    pw = password.encode("utf-16-be")
    out = bytearray(len(body))
    d = salt
    for i in range(0, len(body), 20):
        d = hashlib.sha1(pw + d).digest()
        blk = body[i:i + 20]
        out[i:i + len(blk)] = bytes(x ^ y for x, y in zip(blk, d))
    key = bytes(out)
    if not hmac.compare_digest(hashlib.sha1(pw + key).digest(), check):
        raise ValueError("JKS key password is incorrect")
    return key


def read_jks(data: bytes, password: str) -> JavaKeyStore:
    magic, ver, n = struct.unpack(">IiI", data[:12])
    if magic != 0xFEEDFEED or ver not in (1, 2):
        raise ValueError("not a JKS keystore (JCEKS / PKCS#12 keystores are not served over HTTPS here)")
    body, digest = data[:-20], data[-20:]
    if not hmac.compare_digest(hashlib.sha1(password.encode("utf-16-be") + b"Mighty Aphrodite" + body).digest(),
                               digest):
        raise ValueError("Keystore was tampered with, or password was incorrect")
    off = 12
    keys, certs = {}, {}

    def u16():
        nonlocal off
        v = struct.unpack(">H", data[off:off + 2])[0]
        off += 2
        return v

    def u32():
        nonlocal off
        v = struct.unpack(">I", data[off:off + 4])[0]
        off += 4
        return v

    def utf():
        nonlocal off
        ln = u16()
        s = data[off:off + ln].decode("utf-8")
        off += ln
        return s

    def cert():
        nonlocal off
        if ver == 2:
            utf()                                        # certificate type ("X.509")
        ln = u32()
        c = data[off:off + ln]
        off += ln
        return c

    for _ in range(n):
        tag = u32()
        alias = utf()
        off += 8                                         # creation date
        if tag == 1:
            ln = u32()
            prot = data[off:off + ln]
            off += ln
            chain = [cert() for _ in range(u32())]
            keys[alias] = KeyEntry(alias, _unseal(prot, password), chain)
        elif tag == 2:
            certs[alias] = cert()
        else:
            raise ValueError(f"unknown JKS entry tag {tag}")
    return JavaKeyStore(keys, certs)


def _pem(kind: str, der: bytes) -> str:
    b = base64.b64encode(der).decode()
    return f"-----BEGIN {kind}-----\n" + "\n".join(b[i:i + 64] for i in range(0, len(b), 64)) + f"\n-----END {kind}-----\n"


def pem_files(jks_path: str, password: str | None = None, alias: str | None = None, hostname_as_alias=False,
              directory: str | None = None) -> tuple[str, str]:
    """(certfile, keyfile) PEM paths (mode 0600) of the keystore's private-key entry: ``alias``, the host name
    (``-hostname_as_jks_alias``), or the only key entry."""
    with open(jks_path, "rb") as fh:
        ks = read_jks(fh.read(), DEFAULT_JKS_PASS if password is None else password)
    if hostname_as_alias:
        alias = socket.gethostname()
    if alias is None:
        if len(ks.keys) != 1:
            raise ValueError(f"the keystore holds {len(ks.keys)} private keys: pass -jks_alias")
        alias = next(iter(ks.keys))
    if alias not in ks.keys:
        raise ValueError(f"no private key entry {alias!r} in {jks_path}")
    e = ks.keys[alias]
    d = directory or tempfile.mkdtemp(prefix="h2o_tls_")
    cf, kf = os.path.join(d, "cert.pem"), os.path.join(d, "key.pem")
    for path, text in ((cf, "".join(_pem("CERTIFICATE", c) for c in e.chain_der)),
                       (kf, _pem("PRIVATE KEY", e.key_der))):
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "w") as fh:
            fh.write(text)
    return cf, kf
