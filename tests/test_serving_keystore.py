"""HTTPS from a Java keystore (SecureAPIConfigIT, ``T[lserving]/SecureAPIConfigIT.java:48-97``):
``oryx.serving.api.keystore-file`` + ``keystore-password`` name a JKS or PKCS#12 keystore, as
the reference's Tomcat connector takes them (``[lserving]/ServingLayer.java:214-217``), and the
serving layer answers over HTTPS on both front ends -- the native one (OpenSSL,
``csrc/runtime/oryx_http.cpp``) and the Python fallback -- from the keystore's first key entry
(native parser: ``csrc/runtime/oryx_keystore.cpp``).

Keystores: a PKCS#12 file made with ``openssl pkcs12 -export``; a JKS file written by the small
writer below (the JDK key protector and the file digest, the inverse of the native reader);
and, where the reference tree is present, its own fixture ``oryxtest.jks`` (password
``oryxpass``), read as data only.
"""

import hashlib
import os
import ssl
import struct
import subprocess
import urllib.request

import pytest

from oryx_amd.serving.layer import keystore_pem

from .test_serving_layer import _get, _layer, _self_signed

HAVE_OPENSSL = any(os.path.exists(os.path.join(d, "openssl"))
                   for d in os.environ.get("PATH", "").split(":"))
REF_JKS = "/root/reference/framework/oryx-lambda-serving/src/test/resources/oryxtest.jks"

pytestmark = pytest.mark.skipif(not HAVE_OPENSSL,
                                reason="no openssl binary to make test certificates")


def _der_len(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _tlv(tag, body):
    return bytes([tag]) + _der_len(len(body)) + body


def _write_jks(path, password, alias, pkcs8_der, cert_ders, salt=b"\x5a" * 20):
    """A JKS v2 keystore with one private-key entry (what ``keytool -genkeypair`` writes)."""
    pw = password.encode("utf-16-be")
    # JDK KeyProtector: key stream SHA1(pw || salt), SHA1(pw || previous); check SHA1(pw || key)
    stream, block = b"", salt
    while len(stream) < len(pkcs8_der):
        block = hashlib.sha1(pw + block).digest()
        stream += block
    enc = bytes(a ^ b for a, b in zip(pkcs8_der, stream))
    protected = salt + enc + hashlib.sha1(pw + pkcs8_der).digest()
    oid = bytes([0x06, 0x0A, 0x2B, 0x06, 0x01, 0x04, 0x01, 0x2A, 0x02, 0x11, 0x01, 0x01])
    epki = _tlv(0x30, _tlv(0x30, oid + b"\x05\x00") + _tlv(0x04, protected))
    body = b"\xfe\xed\xfe\xed" + struct.pack(">II", 2, 1)
    a = alias.encode()
    body += struct.pack(">IH", 1, len(a)) + a + struct.pack(">Q", 1415890723927)
    body += struct.pack(">I", len(epki)) + epki + struct.pack(">I", len(cert_ders))
    for c in cert_ders:
        body += struct.pack(">H", 5) + b"X.509" + struct.pack(">I", len(c)) + c
    body += hashlib.sha1(pw + b"Mighty Aphrodite" + body).digest()
    with open(path, "wb") as fh:
        fh.write(body)


def _openssl(*args):
    subprocess.run(["openssl"] + list(args), check=True, capture_output=True, timeout=60)


@pytest.fixture
def stores(tmp_path):
    cert, key = _self_signed(tmp_path)
    p12 = str(tmp_path / "server.p12")
    _openssl("pkcs12", "-export", "-in", cert, "-inkey", key, "-name", "oryxtest", "-out", p12,
             "-passout", "pass:oryxpass")
    der_key, der_cert = str(tmp_path / "key.der"), str(tmp_path / "cert.der")
    _openssl("pkcs8", "-topk8", "-nocrypt", "-in", key, "-outform", "DER", "-out", der_key)
    _openssl("x509", "-in", cert, "-outform", "DER", "-out", der_cert)
    jks = str(tmp_path / "server.jks")
    _write_jks(jks, "oryxpass", "oryxtest", open(der_key, "rb").read(),
               [open(der_cert, "rb").read()])
    return {"cert": cert, "key": key, "p12": p12, "jks": jks}


def test_keystore_pem_decodes_jks_and_pkcs12(stores):
    want = open(stores["cert"], "rb").read().strip()
    for kind in ("jks", "p12"):
        cert, key = keystore_pem(stores[kind], "oryxpass")
        assert cert.strip() == want, kind
        assert key.startswith(b"-----BEGIN PRIVATE KEY-----"), kind
        with pytest.raises(ValueError, match="password"):
            keystore_pem(stores[kind], "wrong")
    # a PEM file is not a keystore: used as is
    assert keystore_pem(stores["cert"], None) is None
    # a damaged JKS body fails the file digest
    raw = bytearray(open(stores["jks"], "rb").read())
    raw[40] ^= 1
    bad = stores["jks"] + ".bad"
    with open(bad, "wb") as fh:
        fh.write(bytes(raw))
    with pytest.raises(ValueError, match="integrity"):
        keystore_pem(bad, "oryxpass")


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("kind", ["jks", "p12"])
def test_https_from_keystore(stores, kind, native):
    """SecureAPIConfigIT.testHTTPS: HTTPS with the keystore's certificate; plain HTTP on the
    TLS port fails (testBadHTTPS's connection error)."""
    lay = _layer({"oryx.serving.api.secure-port": 0,
                  "oryx.serving.api.keystore-file": '"%s"' % stores[kind],
                  "oryx.serving.api.keystore-password": "oryxpass",
                  "oryx.serving.api.native-http": "true" if native else "false"})
    try:
        from oryx_amd.serving.http import NativeHTTPServer
        assert isinstance(lay._server, NativeHTTPServer) == native
        ctx = ssl.create_default_context(cafile=stores["cert"])
        ctx.check_hostname = False
        st, _, body = _get("https://127.0.0.1:%d/recommend/U0" % lay.actual_port,
                           {"Accept": "application/json"}, context=ctx)
        assert st == 200 and b"I1" in body
        with pytest.raises(Exception):
            urllib.request.urlopen("http://127.0.0.1:%d/ready" % lay.actual_port, timeout=5)
    finally:
        lay.close()


@pytest.mark.parametrize("native", [True, False])
def test_keystore_wrong_password_does_not_start(stores, native):
    with pytest.raises(Exception, match="(?i)password|integrity"):
        _layer({"oryx.serving.api.secure-port": 0,
                "oryx.serving.api.keystore-file": '"%s"' % stores["jks"],
                "oryx.serving.api.keystore-password": "not-it",
                "oryx.serving.api.native-http": "true" if native else "false"})


@pytest.mark.skipif(not os.path.exists(REF_JKS), reason="reference tree not present")
def test_reference_fixture_keystore():
    """The reference IT's own keystore (``oryxtest.jks``, password ``oryxpass``) serves HTTPS on
    the native front end with the keystore's certificate."""
    cert, key = keystore_pem(REF_JKS, "oryxpass")
    assert cert.startswith(b"-----BEGIN CERTIFICATE-----") and b"PRIVATE KEY" in key
    lay = _layer({"oryx.serving.api.secure-port": 0,
                  "oryx.serving.api.keystore-file": '"%s"' % REF_JKS,
                  "oryx.serving.api.keystore-password": "oryxpass"})
    try:
        # (the fixture's certificate has expired since 2014: compare it, do not verify it)
        served = ssl.get_server_certificate(("127.0.0.1", lay.actual_port))
        assert ssl.PEM_cert_to_DER_cert(served) == \
            ssl.PEM_cert_to_DER_cert(cert.decode().split("-----END CERTIFICATE-----")[0] +
                                     "-----END CERTIFICATE-----\n")
        st, _, _ = _get("https://127.0.0.1:%d/ready" % lay.actual_port,
                        context=ssl._create_unverified_context())
        assert st == 200
    finally:
        lay.close()
