"""HTTPS from a Java KeyStore (api/tls.py, server -jks / -jks_pass): the reference's own keystore fixtures
(h2o-core/src/test/resources/keystore.jks with a private-key entry, cacerts.jks with a trusted certificate; password
"password" per SSLSocketChannelFactoryTest.java:34-37) are read natively, the unsealed key pairs with its certificate
in the TLS stack, and a live uvicorn server answers /3/Cloud over HTTPS (with Basic login on top)."""
import base64
import os
import socket
import ssl
import threading
import time

import pytest

from llama_github_io_amd.api import tls

KS = "/root/reference/h2o-core/src/test/resources/keystore.jks"
TS = "/root/reference/h2o-core/src/test/resources/cacerts.jks"
pytestmark = pytest.mark.skipif(not os.path.exists(KS), reason="reference keystore fixtures not present")


def test_read_reference_keystores(tmp_path):
    ks = tls.read_jks(open(KS, "rb").read(), "password")
    assert list(ks.keys) == ["mydomain"] and len(ks.keys["mydomain"].chain_der) == 1
    assert ks.keys["mydomain"].key_der[:2] == b"\x30\x82"            # PKCS#8 PrivateKeyInfo SEQUENCE
    ts = tls.read_jks(open(TS, "rb").read(), "password")
    assert list(ts.certs) == ["mydomain"] and ts.certs["mydomain"] == ks.keys["mydomain"].chain_der[0]
    with pytest.raises(ValueError, match="password was incorrect"):
        tls.read_jks(open(KS, "rb").read(), "h2oh2o")
    cf, kf = tls.pem_files(KS, "password", directory=str(tmp_path))
    assert oct(os.stat(kf).st_mode & 0o777) == "0o600"
    ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER).load_cert_chain(cf, kf)   # the key matches the certificate
    with pytest.raises(ValueError, match="no private key entry"):
        tls.pem_files(KS, "password", alias="other", directory=str(tmp_path))


def test_https_server_with_login(tmp_path):
    uvicorn = pytest.importorskip("uvicorn")
    requests = pytest.importorskip("requests")
    from llama_github_io_amd.api.security import LoginConfig
    from llama_github_io_amd.api.server import create_app
    realm = tmp_path / "realm.properties"
    realm.write_text("jenkins_user: jenkins_pwd42\n")
    cf, kf = tls.pem_files(KS, "password", directory=str(tmp_path))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    app = create_app(login=LoginConfig(hash_login=True, login_conf=str(realm)))
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning", ssl_certfile=cf,
                                           ssl_keyfile=kf))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    try:
        url = f"https://127.0.0.1:{port}/3/Cloud"
        for _ in range(100):
            if server.started:
                break
            time.sleep(0.05)
        assert requests.get(url, verify=False, timeout=10).status_code == 401
        r = requests.get(url, verify=False, timeout=10, auth=("jenkins_user", "jenkins_pwd42"))
        assert r.status_code == 200 and "cloud_name" in r.json()
        with pytest.raises(requests.exceptions.SSLError):
            requests.get(url, verify=True, timeout=10)                # self-signed: verification must fail
    finally:
        server.should_exit = True
        th.join(10)


def test_jks_private_key_pem_deleted_after_startup(tmp_path):
    """The PEM files unsealed from the keystore live only until uvicorn has built its SSL context."""
    pytest.importorskip("uvicorn")
    from llama_github_io_amd.api.server import create_app, uvicorn_config
    cf, kf = tls.pem_files(KS, "password")
    assert os.path.exists(kf)
    cfg = uvicorn_config(create_app(), "127.0.0.1", 0, dict(ssl_certfile=cf, ssl_keyfile=kf))
    assert cfg.loaded and cfg.ssl is not None
    assert not os.path.exists(kf) and not os.path.exists(cf) and not os.path.exists(os.path.dirname(kf))
