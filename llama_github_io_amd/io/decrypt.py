"""Encrypted input files: Decryption Tools (reference: ``water/parser/DecryptionTool.java``,
``GenericDecryptionTool.java``, ``water/api/DecryptionSetupHandler.java``, ``schemas3/DecryptionSetupV3.java``;
R ``h2o.decryptionSetup``).

A :class:`DecryptionSetup` names a Java keystore (a raw file key: the path from ImportFiles, or uploaded bytes in
the DKV), its type, the key alias, the password and the cipher spec. :func:`make_tool` reads the secret key out of
the keystore and installs a :class:`GenericDecryptionTool` in the DKV; ``import_file(..., decrypt_tool=key)`` then
decrypts every file before parse-type detection (so an encrypted gzip / zip container is unpacked after decryption,
as the reference's decrypting input stream feeding the ZipUtil path).

Keystores: ``JCEKS`` (the reference's documented type: JKS cannot hold secret keys). The container is parsed here
(magic 0xCECECECE, entries, SHA-1 integrity digest over the password and "Mighty Aphrodite"); the secret-key entry
is a Java-serialised ``SealedObjectForKeyProtector`` read by a strict stream parser (data only: class
descriptors, strings, arrays, enums — no class is instantiated), its ``encryptedContent`` unsealed with
PBEWithMD5AndTripleDES and the resulting serialised ``SecretKeySpec`` (or ``KeyRep``) parsed the same way. The
ciphers run natively (``csrc/crypto.cpp`` on OpenSSL libcrypto): ``AES/ECB`` and ``DESede/ECB`` with
``PKCS5Padding`` or ``NoPadding`` — the specs ``Cipher.init(DECRYPT_MODE, key)`` accepts without parameters.
"""
from __future__ import annotations

import ctypes
import hashlib
import struct
import uuid
from dataclasses import dataclass

from ..core import dkv


@dataclass
class DecryptionSetup:
    keystore_id: object = None
    keystore_type: str = "JCEKS"
    key_alias: str = ""
    password: str = ""
    cipher_spec: str = ""
    decrypt_tool_id: str | None = None
    decrypt_impl: str = "water.parser.GenericDecryptionTool"


# ------------------------------------------------------------------------------------------------ native ciphers
def _lib():
    from ..ops import _native as nat
    lib = nat.rt()
    if not getattr(lib, "_h2o_crypto_bound", False):
        u8p, ll, llp = ctypes.c_void_p, ctypes.c_longlong, ctypes.POINTER(ctypes.c_longlong)
        lib.h2o_pbe_md5_3des_decrypt.argtypes = [u8p, ctypes.c_int, u8p, ctypes.c_int, u8p, ll, u8p, llp]
        for n in ("h2o_cipher_decrypt", "h2o_cipher_encrypt"):
            getattr(lib, n).argtypes = [ctypes.c_int, u8p, ctypes.c_int, ctypes.c_int, u8p, ll, u8p, llp]
        lib._h2o_crypto_bound = True
    return lib


def _buf(b: bytes):
    return ctypes.create_string_buffer(bytes(b), max(len(b), 1))


def _run(fn, *head, data: bytes, extra: int = 0) -> bytes:
    src = _buf(data)
    out = ctypes.create_string_buffer(len(data) + extra + 32)
    n = ctypes.c_longlong(0)
    rc = fn(*head, ctypes.addressof(src), len(data), ctypes.addressof(out), ctypes.byref(n))
    if rc != 0:
        raise ValueError(f"decryption failed (rc {rc}): wrong key / password or corrupted input")
    return out.raw[: n.value]


def _pbe_unseal(salt: bytes, iters: int, password: str, data: bytes) -> bytes:
    # com.sun.crypto.provider.PBEKey: each password char keeps its low 7 bits
    pw = bytes(ord(ch) & 0x7F for ch in password)
    lib = _lib()
    s, p = _buf(salt), _buf(pw)
    return _run(lib.h2o_pbe_md5_3des_decrypt, ctypes.addressof(s), int(iters), ctypes.addressof(p), len(pw),
                data=data)


_ALGOS = {"AES": 0, "DESEDE": 1, "TRIPLEDES": 1}


def _parse_spec(spec: str):
    parts = [s.strip() for s in str(spec).split("/")]
    algo = parts[0].upper()
    mode = parts[1].upper() if len(parts) > 1 else "ECB"
    pad = parts[2].upper() if len(parts) > 2 else "PKCS5PADDING"
    if algo not in _ALGOS:
        raise ValueError(f"Cipher initialization failed: unsupported cipher algorithm {parts[0]!r} (AES, DESede)")
    if mode != "ECB":
        # Cipher.init(DECRYPT_MODE, key) without parameters: the reference's tool cannot run IV modes either
        raise ValueError(f"Cipher initialization failed: mode {parts[1]} needs parameters (IV) the Decryption Tool "
                         "does not take; use ECB")
    if pad not in ("PKCS5PADDING", "PKCS7PADDING", "NOPADDING"):
        raise ValueError(f"Cipher initialization failed: unsupported padding {parts[2]!r}")
    return _ALGOS[algo], 0 if pad == "NOPADDING" else 1


def cipher_decrypt(spec: str, key: bytes, data: bytes) -> bytes:
    algo, pad = _parse_spec(spec)
    k = _buf(key)
    return _run(_lib().h2o_cipher_decrypt, algo, ctypes.addressof(k), len(key), pad, data=data)


def cipher_encrypt(spec: str, key: bytes, data: bytes) -> bytes:
    algo, pad = _parse_spec(spec)
    k = _buf(key)
    return _run(_lib().h2o_cipher_encrypt, algo, ctypes.addressof(k), len(key), pad, data=data, extra=32)


# ------------------------------------------------------------------------------------------------ Java serialisation
class _JavaStream:
    """Strict reader of a java.io.ObjectOutputStream stream (protocol 2): objects become
    ``{"class": name, "fields": {...}}``, byte arrays ``bytes``, strings ``str``, enums ``("enum", class, name)``.
    Only data is decoded; nothing is looked up or instantiated."""

    TC_NULL, TC_REFERENCE, TC_CLASSDESC, TC_OBJECT, TC_STRING, TC_ARRAY = 0x70, 0x71, 0x72, 0x73, 0x74, 0x75
    TC_BLOCKDATA, TC_ENDBLOCKDATA, TC_LONGSTRING, TC_BLOCKDATALONG, TC_ENUM = 0x77, 0x78, 0x7C, 0x7A, 0x7E
    _PRIM = {"B": (1, ">b"), "C": (2, ">H"), "D": (8, ">d"), "F": (4, ">f"), "I": (4, ">i"), "J": (8, ">q"),
             "S": (2, ">h"), "Z": (1, ">?")}

    def __init__(self, data: bytes, pos: int = 0):
        self.d, self.p = data, pos
        self.handles = []
        if self._take(2) != b"\xac\xed" or self._u16() != 5:
            raise ValueError("not a Java serialization stream")

    def _take(self, n):
        if self.p + n > len(self.d):
            raise ValueError("truncated Java serialization stream")
        b = self.d[self.p:self.p + n]
        self.p += n
        return b

    def _u8(self):
        return self._take(1)[0]

    def _u16(self):
        return struct.unpack(">H", self._take(2))[0]

    def _i32(self):
        return struct.unpack(">i", self._take(4))[0]

    def _utf(self, n=None):
        n = self._u16() if n is None else n
        return self._take(n).decode("utf-8", errors="replace")

    def _new(self, obj):
        self.handles.append(obj)
        return len(self.handles) - 1

    def content(self):
        tc = self._u8()
        if tc == self.TC_NULL:
            return None
        if tc == self.TC_REFERENCE:
            h = self._i32() - 0x7E0000
            if not 0 <= h < len(self.handles):
                raise ValueError("bad handle in Java serialization stream")
            return self.handles[h]
        if tc == self.TC_STRING:
            s = self._utf()
            self._new(s)
            return s
        if tc == self.TC_LONGSTRING:
            n = struct.unpack(">q", self._take(8))[0]
            s = self._take(n).decode("utf-8", errors="replace")
            self._new(s)
            return s
        if tc == self.TC_CLASSDESC:
            self.p -= 1
            return self.classdesc()
        if tc == self.TC_ARRAY:
            cd = self.classdesc()
            h = self._new(None)
            n = self._i32()
            et = cd["name"][1:]
            if et == "B":
                v = self._take(n)
            elif et in self._PRIM:
                sz, f = self._PRIM[et]
                v = [struct.unpack(f, self._take(sz))[0] for _ in range(n)]
            else:
                v = [self.content() for _ in range(n)]
            self.handles[h] = v
            return v
        if tc == self.TC_ENUM:
            cd = self.classdesc()
            h = self._new(None)
            name = self.content()
            self.handles[h] = ("enum", cd["name"], name)
            return self.handles[h]
        if tc == self.TC_OBJECT:
            cd = self.classdesc()
            obj = {"class": cd["name"], "fields": {}}
            self._new(obj)
            chain = []
            c = cd
            while c is not None:
                chain.append(c)
                c = c["super"]
            for c in reversed(chain):            # superclass data first
                for tcode, fname, _ in c["fields"]:
                    if tcode in self._PRIM:
                        sz, f = self._PRIM[tcode]
                        obj["fields"][fname] = struct.unpack(f, self._take(sz))[0]
                    else:
                        obj["fields"][fname] = self.content()
                if c["flags"] & 0x01:              # SC_WRITE_METHOD: custom data up to the end block
                    self._annotation()
            return obj
        raise ValueError(f"unsupported Java serialization type code 0x{tc:02x}")

    def _annotation(self):
        while True:
            tc = self.d[self.p]
            if tc == self.TC_ENDBLOCKDATA:
                self.p += 1
                return
            if tc == self.TC_BLOCKDATA:
                self.p += 1
                self._take(self._u8())
            elif tc == self.TC_BLOCKDATALONG:
                self.p += 1
                self._take(self._i32())
            else:
                self.content()

    def classdesc(self):
        tc = self._u8()
        if tc == self.TC_NULL:
            return None
        if tc == self.TC_REFERENCE:
            self.p -= 1
            return self.content()
        if tc != self.TC_CLASSDESC:
            raise ValueError(f"expected a class descriptor, got 0x{tc:02x}")
        name = self._utf()
        self._take(8)                             # serialVersionUID
        cd = {"name": name, "fields": [], "super": None, "flags": 0}
        self._new(cd)
        cd["flags"] = self._u8()
        for _ in range(self._u16()):
            t = chr(self._u8())
            fname = self._utf()
            cls = self.content() if t in "L[" else None
            cd["fields"].append((t, fname, cls))
        self._annotation()
        cd["super"] = self.classdesc()
        return cd


def _der_pbe_params(b: bytes):
    """PBEParameterSpec DER: SEQUENCE { OCTET STRING salt, INTEGER iterationCount }."""
    def tlv(pos):
        tag = b[pos]
        ln = b[pos + 1]
        pos += 2
        if ln & 0x80:
            k = ln & 0x7F
            ln = int.from_bytes(b[pos:pos + k], "big")
            pos += k
        return tag, b[pos:pos + ln], pos + ln
    tag, body, _ = tlv(0)
    if tag != 0x30:
        raise ValueError("bad PBE parameters")
    t1, salt, nxt = tlv(0 + (len(b) - len(body)))
    t2, it, _ = tlv(nxt)
    if t1 != 0x04 or t2 != 0x02:
        raise ValueError("bad PBE parameters")
    return salt, int.from_bytes(it, "big")


# ------------------------------------------------------------------------------------------------ JCEKS
def read_jceks_secret_key(data: bytes, alias: str, password: str):
    """(algorithm, key bytes) of the secret-key entry ``alias`` of a JCEKS keystore (KeyStore.load + getKey)."""
    if len(data) < 32 or data[:4] != b"\xce\xce\xce\xce":
        raise ValueError("Failed to read keystore: not a JCEKS keystore")
    version, count = struct.unpack(">ii", data[4:12])
    if version not in (1, 2):
        raise ValueError(f"Failed to read keystore: unsupported JCEKS version {version}")
    # integrity: SHA-1(password UTF-16BE || "Mighty Aphrodite" || keystore bytes) == trailing digest
    body, digest = data[:-20], data[-20:]
    h = hashlib.sha1(password.encode("utf-16-be") + b"Mighty Aphrodite" + body).digest()
    if h != digest:
        raise ValueError("Keystore was tampered with, or password was incorrect")
    p = 12
    entries = {}

    def utf(pos):
        n = struct.unpack(">H", data[pos:pos + 2])[0]
        return data[pos + 2:pos + 2 + n].decode("utf-8"), pos + 2 + n
    for _ in range(count):
        tag = struct.unpack(">i", data[p:p + 4])[0]
        p += 4
        name, p = utf(p)
        p += 8                                   # creation date
        if tag == 1:                             # private key + certificate chain
            n = struct.unpack(">i", data[p:p + 4])[0]
            p += 4 + n
            nc = struct.unpack(">i", data[p:p + 4])[0]
            p += 4
            for _ in range(nc):
                if version == 2:
                    _, p = utf(p)
                n = struct.unpack(">i", data[p:p + 4])[0]
                p += 4 + n
            entries[name] = ("private", None)
        elif tag == 2:                           # trusted certificate
            if version == 2:
                _, p = utf(p)
            n = struct.unpack(">i", data[p:p + 4])[0]
            p += 4 + n
            entries[name] = ("cert", None)
        elif tag == 3:                           # secret key: serialized SealedObjectForKeyProtector
            js = _JavaStream(data, p)
            obj = js.content()
            p = js.p
            entries[name] = ("secret", obj)
        else:
            raise ValueError(f"Failed to read keystore: unknown entry tag {tag}")
    key = alias.lower()                          # JCEKS aliases are case-insensitive (stored lower-case)
    if key not in entries:
        raise ValueError("Alias for key not found")
    kind, sealed = entries[key]
    if kind != "secret":
        raise ValueError(f"entry {alias!r} is not a secret key")
    f = sealed["fields"]
    if str(f.get("sealAlg", "")).upper() != "PBEWITHMD5ANDTRIPLEDES":
        raise ValueError(f"unsupported key protection {f.get('sealAlg')!r}")
    salt, iters = _der_pbe_params(f["encodedParams"])
    plain = _pbe_unseal(salt, iters, password, f["encryptedContent"])
    keyobj = _JavaStream(plain).content()
    kf = keyobj["fields"]
    if "key" in kf:                              # javax.crypto.spec.SecretKeySpec
        return str(kf["algorithm"]), bytes(kf["key"])
    if "encoded" in kf:                          # java.security.KeyRep (provider key classes)
        return str(kf["algorithm"]), bytes(kf["encoded"])
    raise ValueError(f"unsupported sealed key class {keyobj['class']}")


# ------------------------------------------------------------------------------------------------ tools
class GenericDecryptionTool:
    """Decrypts whole files with the keystore's secret key and the setup's cipher spec."""

    def __init__(self, setup: DecryptionSetup, algorithm: str, key: bytes):
        self.key_id = setup.decrypt_tool_id
        self.algorithm, self._key = algorithm, key
        self.cipher_spec = setup.cipher_spec
        _parse_spec(self.cipher_spec)             # fail at setup time, as Cipher.getInstance would

    def decrypt(self, data: bytes) -> bytes:
        return cipher_decrypt(self.cipher_spec, self._key, data)


def _keystore_bytes(ks) -> bytes:
    if isinstance(ks, (bytes, bytearray)):
        return bytes(ks)
    if isinstance(ks, dict) and "name" in ks:    # a KeyV3 dict
        ks = ks["name"]
    obj = dkv.get(str(ks)) if dkv.contains(str(ks)) else None
    if isinstance(obj, (bytes, bytearray)):
        return bytes(obj)
    path = str(ks)
    for pre in ("nfs://", "file://"):
        if path.startswith(pre):
            path = path[len(pre):]
    with open(path, "rb") as f:
        return f.read()


def make_tool(setup: DecryptionSetup) -> GenericDecryptionTool:
    """DecryptionTool.make: read the key, build the tool, install it in the DKV under decrypt_tool_id."""
    if setup.decrypt_impl not in ("water.parser.GenericDecryptionTool", "GenericDecryptionTool", "", None):
        raise ValueError(f"Unknown decrypt tool: {setup.decrypt_impl}")
    if str(setup.keystore_type).upper() != "JCEKS":
        raise ValueError(f"keystore type {setup.keystore_type!r} is not supported (JCEKS; JKS cannot hold secret keys)")
    if not setup.decrypt_tool_id:
        setup.decrypt_tool_id = f"decrypt_tool_{uuid.uuid4().hex[:12]}"
    algo, key = read_jceks_secret_key(_keystore_bytes(setup.keystore_id), setup.key_alias, setup.password)
    tool = GenericDecryptionTool(setup, algo, key)
    dkv.put(setup.decrypt_tool_id, tool)
    return tool


def get_tool(key):
    """DecryptionTool.get: the installed tool for a key (None: no decryption)."""
    if key is None or key == "":
        return None
    if isinstance(key, GenericDecryptionTool):
        return key
    if isinstance(key, dict) and "name" in key:
        key = key["name"]
    tool = dkv.get(str(key)) if dkv.contains(str(key)) else None
    if not isinstance(tool, GenericDecryptionTool):
        raise ValueError(f"Decryption tool {key!r} not found")
    return tool
