"""Encrypted input files (reference: water/parser/DecryptionTool.java, ParseTestEncrypted.java; R h2o.decryptionSetup).

Fixtures from the reference (read in place): ``h2o-r/h2o-package/inst/extdata/keystore.jks`` — a JCEKS keystore whose
entry ``secretKeyAlias`` (password ``Password123``) holds an AES key — and ``prostate.csv.aes``, ``prostate.csv``
encrypted with it under AES/ECB/PKCS5Padding (the R documentation example)."""
import gzip
import io
import os
import zipfile

import numpy as np
import pytest

EXT = "/root/reference/h2o-r/h2o-package/inst/extdata"
KS, AES, PLAIN = (os.path.join(EXT, n) for n in ("keystore.jks", "prostate.csv.aes", "prostate.csv"))
pytestmark = pytest.mark.skipif(not os.path.exists(KS), reason="reference fixtures not present")
SPEC = "AES/ECB/PKCS5Padding"


def test_jceks_key_decrypts_reference_file_bit_exactly():
    from llama_github_io_amd.io import decrypt as D
    algo, key = D.read_jceks_secret_key(open(KS, "rb").read(), "secretKeyAlias", "Password123")
    assert algo == "AES" and len(key) == 16
    assert D.cipher_decrypt(SPEC, key, open(AES, "rb").read()) == open(PLAIN, "rb").read()
    with pytest.raises(ValueError, match="password was incorrect"):
        D.read_jceks_secret_key(open(KS, "rb").read(), "secretKeyAlias", "Password124")
    with pytest.raises(ValueError, match="Alias for key not found"):
        D.read_jceks_secret_key(open(KS, "rb").read(), "otherAlias", "Password123")
    with pytest.raises(ValueError, match="IV"):
        D.cipher_decrypt("AES/CBC/PKCS5Padding", key, b"0" * 16)


def test_import_encrypted_csv_gz_zip(tmp_path):
    """ParseTestEncrypted: encrypted CSV, encrypted gzip and encrypted zip containers parse like the plain file."""
    import h2o
    from llama_github_io_amd.io import decrypt as D
    dt = h2o.decryption_setup(KS, key_alias="secretKeyAlias", password="Password123", cipher_spec=SPEC)
    plain = h2o.import_file(PLAIN)
    got = h2o.import_file(AES, decrypt_tool=dt)
    assert got.names == plain.names and got.nrows == plain.nrows == 380
    np.testing.assert_allclose(got.as_data_frame().to_numpy(float), plain.as_data_frame().to_numpy(float))
    _, key = D.read_jceks_secret_key(open(KS, "rb").read(), "secretKeyAlias", "Password123")
    raw = open(PLAIN, "rb").read()
    zb = io.BytesIO()
    with zipfile.ZipFile(zb, "w") as z:
        z.writestr("prostate.csv", raw)
    for name, payload in (("e.gz.aes", gzip.compress(raw)), ("e.zip.aes", zb.getvalue())):
        p = tmp_path / name
        p.write_bytes(D.cipher_encrypt(SPEC, key, payload))
        fr = h2o.import_file(str(p), decrypt_tool=dt)
        assert fr.nrows == 380 and fr.names == plain.names
        np.testing.assert_allclose(fr.as_data_frame().to_numpy(float), plain.as_data_frame().to_numpy(float))
    with pytest.raises(ValueError):
        h2o.decryption_setup(KS, key_alias="secretKeyAlias", password="nope", cipher_spec=SPEC)


def test_rest_decryption_setup_and_parse():
    pytest.importorskip("fastapi")
    from fastapi.testclient import TestClient
    from llama_github_io_amd.api.server import create_app
    c = TestClient(create_app(), raise_server_exceptions=False)
    r = c.post("/3/DecryptionSetup", json=dict(keystore_id=KS, keystore_type="JCEKS", key_alias="secretKeyAlias",
                                               password="Password123", cipher_spec=SPEC))
    assert r.status_code == 200, r.text
    tool = r.json()["decrypt_tool_id"]["name"]
    st = c.post("/3/ParseSetup", json=dict(source_frames=[AES], decrypt_tool=tool)).json()
    assert st["column_names"][:3] == ["ID", "CAPSULE", "AGE"]
    j = c.post("/3/Parse", json=dict(source_frames=[AES], destination_frame="prostate_dec", decrypt_tool=tool,
                                     check_header=1)).json()
    import time
    for _ in range(400):
        s = c.get(f"/3/Jobs/{j['job']['key']['name']}").json()["jobs"][0]["status"]
        if s in ("DONE", "FAILED"):
            break
        time.sleep(0.05)
    assert s == "DONE"
    fr = c.get("/3/Frames/prostate_dec").json()["frames"][0]
    assert fr["rows"] == 380
    bad = c.post("/3/DecryptionSetup", json=dict(keystore_id=KS, key_alias="secretKeyAlias", password="x",
                                                 cipher_spec=SPEC))
    assert bad.status_code >= 400


def _jdk_pbe_md5_3des_seal(salt: bytes, iters: int, password: str, plain: bytes) -> bytes:
    """PBEWithMD5AndTripleDES encryption as com.sun.crypto.provider.PBES1Core does it, modelled in Python:
    MD5 chains over each salt half, DESede/CBC with the derived IV, PKCS5 padding. Salts with identical halves go
    through the JDK's swap loop that stores at index 3 - 1 ([a, b, c, d] -> [d, a, b, d])."""
    import hashlib
    from llama_github_io_amd.io.decrypt import cipher_encrypt
    s = bytearray(salt)
    if s[:4] == s[4:]:
        for i in range(2):
            t = s[i]
            s[i] = s[3 - i]
            s[3 - 1] = t
    pw = bytes(ord(ch) & 0x7F for ch in password)
    derived = b""
    for h in range(2):
        buf = bytes(s[4 * h:4 * h + 4])
        for _ in range(iters):
            buf = hashlib.md5(buf + pw).digest()
        derived += buf
    key, iv = derived[:24], derived[24:32]
    n = 8 - len(plain) % 8
    data = plain + bytes([n]) * n
    out, prev = b"", iv
    for i in range(0, len(data), 8):
        blk = bytes(a ^ b for a, b in zip(data[i:i + 8], prev))
        prev = cipher_encrypt("DESede/ECB/NoPadding", key, blk)
        out += prev
    return out


@pytest.mark.parametrize("salt", [bytes([1, 2, 3, 4, 9, 8, 7, 6]), bytes([0x11, 0x22, 0x33, 0x44] * 2)])
def test_pbe_unseal_matches_jdk_salt_handling(salt):
    """JCEKS key sealing: random salts and the equal-halves case, where the JDK's PBES1Core turns the first half
    [a, b, c, d] into [d, a, b, d] (not a reversal); keys it sealed must unseal bit-exactly."""
    from llama_github_io_amd.io.decrypt import _pbe_unseal
    plain = b"secret key material \x00\x01\x02 of 37 bytes!!"
    sealed = _jdk_pbe_md5_3des_seal(salt, 20, "Password123", plain)
    assert _pbe_unseal(salt, 20, "Password123", sealed) == plain
