"""The serving container over real HTTP(S): ports of the reference's ServingLayerTest,
SecureAPIConfigIT (TLS + DIGEST auth), CompressedResponseTest, IngestTest (text / gzip /
deflate / multipart with gzip and zip parts), ErrorResourceTest and ReadOnlyTest
(``framework/oryx-lambda-serving/src/test/java/com/cloudera/oryx/lambda/serving/*``,
``app/oryx-app-serving/src/test/java/com/cloudera/oryx/app/serving/als/*``)."""

import gzip
import io
import json
import os
import ssl
import subprocess
import urllib.error
import urllib.request
import uuid
import zipfile
import zlib

import pytest

from oryx_amd.serving.layer import ServingLayer
from oryx_amd.transport.producer import MockTopicProducer
from oryx_amd.utils import config as cfg

from .serving_harness import MockManager
from .test_als_serving import build_test_model


def _layer(overlay=None, read_only=False):
    o = {
        "oryx.serving.api.port": 0,
        "oryx.serving.no-init-topics": "true",
        "oryx.serving.api.read-only": "true" if read_only else "false",
        "oryx.serving.application-resources":
            '"com.cloudera.oryx.app.serving,com.cloudera.oryx.app.serving.als"',
    }
    o.update(overlay or {})
    config = cfg.overlay_on(o, cfg.get_default())
    MockTopicProducer.clear()
    layer = ServingLayer(config, manager=MockManager(config, build_test_model()),
                         input_producer=MockTopicProducer(), host="127.0.0.1")
    return layer.start()


def _get(url, headers=None, context=None, method="GET", data=None):
    req = urllib.request.Request(url, headers=headers or {}, method=method, data=data)
    try:
        with urllib.request.urlopen(req, context=context, timeout=20) as r:
            return r.status, dict(r.headers), r.read()
    except urllib.error.HTTPError as e:
        return e.code, dict(e.headers), e.read()


@pytest.fixture
def layer():
    lay = _layer()
    yield lay
    lay.close()


def test_ready_recommend_and_error_pages(layer):
    base = "http://127.0.0.1:%d" % layer.actual_port
    assert _get(base + "/ready")[0] == 200
    st, _, body = _get(base + "/recommend/U0", {"Accept": "application/json"})
    assert st == 200
    recs = json.loads(body)
    assert recs[0]["id"] == "I1" and abs(recs[0]["value"] - 0.4653969) < 1e-5
    st, _, body = _get(base + "/recommend/U0", {"Accept": "text/csv"})
    assert st == 200 and body.decode().splitlines()[0].startswith("I1,0.465")
    # unknown user -> 404 with an error page; unknown path -> 404
    st, hdr, body = _get(base + "/recommend/nobody", {"Accept": "text/html,*/*;q=0.8"})
    assert st == 404 and b"nobody" in body
    # an Accept the resource cannot produce -> 406 (JAX-RS content negotiation)
    assert _get(base + "/recommend/U0", {"Accept": "image/png"})[0] == 406
    assert _get(base + "/no/such/endpoint")[0] == 404
    st, _, body = _get(base + "/error?code=503&message=down", {"Accept": "text/plain"})
    assert st == 503 and b"down" in body
    # bad argument -> 400
    assert _get(base + "/recommend/U0?howMany=-1")[0] == 400


def test_context_path():
    lay = _layer({"oryx.serving.api.context-path": '"/oryx"'})
    try:
        base = "http://127.0.0.1:%d" % lay.actual_port
        assert _get(base + "/oryx/ready")[0] == 200
        assert _get(base + "/ready")[0] == 404
    finally:
        lay.close()


def test_compressed_responses(layer):
    base = "http://127.0.0.1:%d" % layer.actual_port
    for enc, dec in (("gzip", gzip.decompress), ("deflate", zlib.decompress)):
        st, hdr, body = _get(base + "/recommend/U0", {"Accept": "application/json",
                                                        "Accept-Encoding": enc})
        assert st == 200 and hdr.get("Content-Encoding") == enc
        assert json.loads(dec(body))[0]["id"] == "I1"
    st, hdr, body = _get(base + "/recommend/U0", {"Accept": "application/json"})
    assert "Content-Encoding" not in hdr and json.loads(body)[0]["id"] == "I1"


def _multipart(parts):
    boundary = uuid.uuid4().hex
    out = io.BytesIO()
    for name, ctype, data in parts:
        out.write(("--%s\r\nContent-Disposition: form-data; name=\"%s\"; filename=\"%s\"\r\n"
                   "Content-Type: %s\r\n\r\n" % (boundary, name, name, ctype)).encode())
        out.write(data)
        out.write(b"\r\n")
    out.write(("--%s--\r\n" % boundary).encode())
    return "multipart/form-data; boundary=" + boundary, out.getvalue()


def test_ingest_formats(layer):
    url = "http://127.0.0.1:%d/ingest" % layer.actual_port
    lines = b"a,B,1\nc,B\nc,D,5.,123456\n"
    assert _get(url, {"Content-Type": "text/plain"}, method="POST", data=lines)[0] == 204
    assert _get(url, {"Content-Type": "text/plain", "Content-Encoding": "gzip"},
                method="POST", data=gzip.compress(lines))[0] == 204
    assert _get(url, {"Content-Type": "text/plain", "Content-Encoding": "deflate"},
                method="POST", data=zlib.compress(lines))[0] == 204
    zbuf = io.BytesIO()
    with zipfile.ZipFile(zbuf, "w") as zf:
        zf.writestr("data.csv", lines)
    ctype, body = _multipart([("plain", "text/plain", lines),
                              ("gz", "application/gzip", gzip.compress(lines)),
                              ("zip", "application/zip", zbuf.getvalue())])
    assert _get(url, {"Content-Type": ctype}, method="POST", data=body)[0] == 204
    msgs = [m for _, m in MockTopicProducer.get_key_messages()]
    # 3 lines per upload: text, gzip, deflate, then 3 multipart parts
    assert len(msgs) == 3 * 6
    assert all(m.startswith("a,B,1.0,") for m in msgs[0::3])
    assert all(m == "c,D,5.0,123456" for m in msgs[2::3])


def test_read_only_layer():
    lay = _layer(read_only=True)
    try:
        base = "http://127.0.0.1:%d" % lay.actual_port
        assert _get(base + "/ingest", {"Content-Type": "text/plain"}, method="POST",
                    data=b"a,b,1\n")[0] == 403
        assert _get(base + "/pref/U1/I2", method="POST", data=b"1")[0] == 403
        assert _get(base + "/recommend/U0")[0] == 200
    finally:
        lay.close()


def _self_signed(tmp_path):
    cert, key = str(tmp_path / "cert.pem"), str(tmp_path / "key.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                    "-out", cert, "-days", "2", "-subj", "/CN=127.0.0.1"], check=True,
                   capture_output=True, timeout=60)
    return cert, key


@pytest.mark.skipif(not any(os.path.exists(os.path.join(d, "openssl"))
                            for d in os.environ.get("PATH", "").split(":")),
                    reason="no openssl binary to make a test certificate")
def test_https_and_digest_auth(tmp_path):
    cert, key = _self_signed(tmp_path)
    lay = _layer({"oryx.serving.api.secure-port": 0,
                  "oryx.serving.api.keystore-file": '"%s"' % cert,
                  "oryx.serving.api.key-file": '"%s"' % key,
                  "oryx.serving.api.user-name": "oryx",
                  "oryx.serving.api.password": "pass"})
    try:
        from oryx_amd.serving.http import NativeHTTPServer
        # HTTPS stays on the native front end (OpenSSL in oryx_http.cpp)
        assert isinstance(lay._server, NativeHTTPServer) and lay._server.tls
        url = "https://127.0.0.1:%d/recommend/U0" % lay.actual_port
        ctx = ssl.create_default_context(cafile=cert)
        ctx.check_hostname = False
        # no credentials -> 401 with a DIGEST challenge
        st, hdr, _ = _get(url, context=ctx)
        assert st == 401 and hdr.get("WWW-Authenticate", "").startswith("Digest")
        # right credentials (urllib answers the challenge)
        for user, pw, want in (("oryx", "pass", 200), ("oryx", "wrong", 401)):
            mgr = urllib.request.HTTPPasswordMgrWithDefaultRealm()
            mgr.add_password(None, url, user, pw)
            opener = urllib.request.build_opener(urllib.request.HTTPSHandler(context=ctx),
                                                 urllib.request.HTTPDigestAuthHandler(mgr))
            try:
                with opener.open(urllib.request.Request(
                        url, headers={"Accept": "application/json"}), timeout=20) as r:
                    status, body = r.status, r.read()
            except urllib.error.HTTPError as e:
                status, body = e.code, b""
            assert status == want
            if want == 200:
                assert json.loads(body)[0]["id"] == "I1"
        # plain HTTP against the TLS port fails
        with pytest.raises(Exception):
            urllib.request.urlopen("http://127.0.0.1:%d/ready" % lay.actual_port, timeout=5)
    finally:
        lay.close()


def _digest_header(auth, method, uri, nonce, nc, password="pass", user="oryx"):
    import hashlib
    ha1 = hashlib.md5(("%s:%s:%s" % (user, auth.realm, password)).encode()).hexdigest()
    ha2 = hashlib.md5(("%s:%s" % (method, uri)).encode()).hexdigest()
    ncs = "%08x" % nc
    resp = hashlib.md5(("%s:%s:%s:%s:%s:%s" % (ha1, nonce, ncs, "abc", "auth", ha2)).encode()
                       ).hexdigest()
    return ('Digest username="%s", realm="%s", nonce="%s", uri="%s", qop=auth, nc=%s, '
            'cnonce="abc", response="%s"' % (user, auth.realm, nonce, uri, ncs, resp))


def test_digest_auth_replay_uri_and_expiry():
    import re as _re
    from oryx_amd.serving.http import DigestAuth
    auth = DigestAuth("oryx", "pass", nonce_ttl_s=60)
    nonce = _re.search(r'nonce="([0-9a-f]+)"', auth.challenge()).group(1)
    h1 = _digest_header(auth, "GET", "/recommend/U0", nonce, 1)
    assert auth.verify("GET", "/recommend/U0", h1) == "ok"
    # the same header again (captured and replayed): nc did not increase
    assert auth.verify("GET", "/recommend/U0", h1) == "denied"
    # a valid header pointed at another endpoint
    h2 = _digest_header(auth, "POST", "/ingest", nonce, 2)
    assert auth.verify("POST", "/pref/U0/I0", h2) == "denied"
    assert auth.verify("POST", "/ingest", h2) == "ok"
    # wrong password
    assert auth.verify("GET", "/x", _digest_header(auth, "GET", "/x", nonce, 9, "bad")) == "denied"
    # expired nonce: stale (client re-authenticates with a fresh nonce)
    auth._nonces[nonce][0] -= 3600
    h3 = _digest_header(auth, "GET", "/recommend/U0", nonce, 3)
    assert auth.verify("GET", "/recommend/U0", h3) == "stale"
    assert "stale=true" in auth.challenge(stale=True)
