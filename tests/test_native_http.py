"""The native HTTP front end (csrc/runtime/oryx_http.cpp + serving/http.NativeHTTPServer):
HTTP/1.1 semantics the serving layer relies on -- keep-alive, pipelined requests answered in
order, Content-Length and chunked bodies, Expect: 100-continue, Connection: close, HEAD,
malformed requests, many concurrent connections -- against a small router."""

import http.client
import socket
import threading
import time

import pytest

from oryx_amd.serving import http as ohttp


def _server():
    def echo(req):
        return ohttp.Response(200, req.raw_body, ohttp.TEXT)

    def slow(req, ms):
        time.sleep(int(ms) / 1000.0)
        return "slept %s" % ms

    def hello(req):
        return "hello %s" % ",".join(req.query.get("x", []))

    routes = [ohttp.Route("POST", "/echo", echo, produces=(ohttp.TEXT,)),
              ohttp.Route("GET", "/slow/{ms}", slow, produces=(ohttp.TEXT,)),
              ohttp.Route("GET", "/hello", hello, produces=(ohttp.TEXT,))]
    srv = ohttp.NativeHTTPServer("127.0.0.1", 0, ohttp.Router(routes, "/"), {}, threads=4)
    srv.start_background()
    return srv


def _recv_responses(sock, n, timeout=10.0):
    """n HTTP responses from a raw socket: [(status, headers dict, body)]."""
    sock.settimeout(timeout)
    buf = b""
    out = []
    while len(out) < n:
        while b"\r\n\r\n" not in buf:
            chunk = sock.recv(65536)
            if not chunk:
                return out
            buf += chunk
        head, buf = buf.split(b"\r\n\r\n", 1)
        lines = head.decode("latin-1").split("\r\n")
        status = int(lines[0].split()[1])
        hdrs = {k.strip().lower(): v.strip() for k, _, v in (l.partition(":") for l in lines[1:])}
        clen = int(hdrs.get("content-length", "0"))
        while len(buf) < clen:
            buf += sock.recv(65536)
        out.append((status, hdrs, buf[:clen]))
        buf = buf[clen:]
    return out


def test_keepalive_query_and_bodies():
    srv = _server()
    try:
        c = http.client.HTTPConnection("127.0.0.1", srv.port, timeout=10)
        for j in range(50):
            c.request("GET", "/hello?x=%d&x=b" % j)
            r = c.getresponse()
            assert r.status == 200 and r.read() == b"hello %d,b" % j
        big = bytes(range(256)) * 4000            # ~1 MB body
        c.request("POST", "/echo", body=big, headers={"Content-Type": "text/plain"})
        r = c.getresponse()
        assert r.status == 200 and r.read() == big
        c.request("GET", "/nope")
        r = c.getresponse()
        assert r.status == 404
        r.read()
        c.request("HEAD", "/hello")
        r = c.getresponse()
        assert r.status == 200 and r.read() == b"" and int(r.getheader("Content-Length")) > 0
        c.close()
    finally:
        srv.shutdown()
        srv.server_close()


def test_pipelined_responses_in_request_order_and_chunked():
    srv = _server()
    try:
        s = socket.create_connection(("127.0.0.1", srv.port))
        # the first request finishes last on the handler threads; responses keep the order
        reqs = (b"GET /slow/300 HTTP/1.1\r\nHost: x\r\n\r\n"
                b"GET /slow/1 HTTP/1.1\r\nHost: x\r\n\r\n"
                b"POST /echo HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n"
                b"Content-Type: text/plain\r\n\r\n"
                b"5\r\nhello\r\n7;ext=1\r\n, world\r\n0\r\nX-Trailer: 1\r\n\r\n"
                b"GET /hello?x=z HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
        # sent in small pieces: the parser resumes across reads
        for k in range(0, len(reqs), 7):
            s.sendall(reqs[k:k + 7])
        res = _recv_responses(s, 4)
        assert [r[2] for r in res] == [b"slept 300", b"slept 1", b"hello, world", b"hello z"]
        assert s.recv(10) == b""                   # closed after Connection: close
        s.close()
    finally:
        srv.shutdown()
        srv.server_close()


def test_expect_continue_malformed_and_concurrency():
    srv = _server()
    try:
        s = socket.create_connection(("127.0.0.1", srv.port))
        s.sendall(b"POST /echo HTTP/1.1\r\nHost: x\r\nContent-Length: 4\r\n"
                  b"Content-Type: text/plain\r\nExpect: 100-continue\r\n\r\n")
        s.settimeout(5)
        interim = s.recv(100)
        assert interim.startswith(b"HTTP/1.1 100 Continue\r\n\r\n")
        rest = interim[len(b"HTTP/1.1 100 Continue\r\n\r\n"):]
        s.sendall(b"abcd")
        if rest:
            pytest.fail("unexpected bytes after the interim response: %r" % rest)
        (st, _, body), = _recv_responses(s, 1)
        assert st == 200 and body == b"abcd"
        s.close()
        bad = socket.create_connection(("127.0.0.1", srv.port))
        bad.sendall(b"NONSENSE\r\n\r\n")
        (st, hdrs, _), = _recv_responses(bad, 1)
        assert st == 400 and hdrs.get("connection") == "close"
        bad.close()
        errors = []

        def client(j):
            try:
                c = http.client.HTTPConnection("127.0.0.1", srv.port, timeout=20)
                for i in range(20):
                    c.request("GET", "/hello?x=%d-%d" % (j, i))
                    r = c.getresponse()
                    if r.read() != b"hello %d-%d" % (j, i):
                        errors.append((j, i))
                c.close()
            except Exception as e:                 # surfaced below
                errors.append(repr(e))

        ts = [threading.Thread(target=client, args=(j,)) for j in range(32)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors
    finally:
        srv.shutdown()
        srv.server_close()


def _raw(srv, data, n=1, timeout=10.0):
    s = socket.create_connection(("127.0.0.1", srv.port), timeout=timeout)
    try:
        s.sendall(data)
        return _recv_responses(s, n, timeout)
    finally:
        s.close()


def test_chunked_limits_and_incremental_parse():
    """Chunk sizes are validated before anything is buffered: a size past max_body, a size that
    would wrap a signed sum (1-byte chunk then 7fff...f), a non-hex size -- all answered with an
    error and the connection closed; a body of many tiny chunks is parsed incrementally."""
    def echo(req):
        return ohttp.Response(200, req.raw_body, ohttp.TEXT)

    srv = ohttp.NativeHTTPServer("127.0.0.1", 0,
                                 ohttp.Router([ohttp.Route("POST", "/echo", echo,
                                                           produces=(ohttp.TEXT,))], "/"),
                                 {}, threads=2, max_body=1 << 20)
    srv.start_background()
    head = b"POST /echo HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
    try:
        # larger than max_body
        (st, _, _), = _raw(srv, head + b"200000\r\n")
        assert st == 413
        # overflow attempt: the second size alone exceeds what is left
        (st, _, _), = _raw(srv, head + b"1\r\na\r\n7fffffffffffffff\r\n")
        assert st in (400, 413)           # 16 hex digits: rejected as malformed
        (st, _, _), = _raw(srv, head + b"1\r\na\r\nfffffffffffffff\r\n")
        assert st == 413
        # 16+ hex digits / junk sizes
        (st, _, _), = _raw(srv, head + b"10000000000000000\r\n")
        assert st == 400
        (st, _, _), = _raw(srv, head + b"zz\r\n")
        assert st == 400
        # 20k one-byte chunks sent in small pieces, then a normal request on the same socket
        body = b"".join(b"1\r\n%c\r\n" % (65 + j % 26) for j in range(20000)) + b"0\r\n\r\n"
        s = socket.create_connection(("127.0.0.1", srv.port), timeout=30)
        try:
            s.sendall(head)
            t0 = time.perf_counter()
            for o in range(0, len(body), 97):
                s.sendall(body[o:o + 97])
            s.sendall(b"POST /echo HTTP/1.1\r\nHost: x\r\nContent-Length: 2\r\n\r\nok")
            out = _recv_responses(s, 2, 30)
            dt = time.perf_counter() - t0
        finally:
            s.close()
        want = bytes(65 + j % 26 for j in range(20000))
        assert [o[0] for o in out] == [200, 200] and out[0][2] == want and out[1][2] == b"ok"
        assert dt < 10.0
        # Content-Length above max_body
        (st, _, _), = _raw(srv, b"POST /echo HTTP/1.1\r\nContent-Length: 2000000\r\n\r\n")
        assert st == 413
    finally:
        srv.shutdown()
        srv.server_close()


def test_native_https(tmp_path):
    """HTTPS on the native loop (OpenSSL, non-blocking handshake): keep-alive requests,
    a chunked body, pipelining, and a plain-HTTP client refused."""
    import shutil
    import ssl
    import subprocess
    if not shutil.which("openssl"):
        pytest.skip("no openssl binary to make a test certificate")
    cert, key = str(tmp_path / "c.pem"), str(tmp_path / "k.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                    "-out", cert, "-days", "2", "-subj", "/CN=127.0.0.1"], check=True,
                   capture_output=True, timeout=60)

    def echo(req):
        return ohttp.Response(200, req.raw_body, ohttp.TEXT)

    def hello(req):
        return "hello %s" % ",".join(req.query.get("x", []))

    routes = [ohttp.Route("POST", "/echo", echo, produces=(ohttp.TEXT,)),
              ohttp.Route("GET", "/hello", hello, produces=(ohttp.TEXT,))]
    srv = ohttp.NativeHTTPServer("127.0.0.1", 0, ohttp.Router(routes, "/"), {}, threads=4,
                                 tls=(cert, key, None))
    srv.start_background()
    try:
        ctx = ssl.create_default_context(cafile=cert)
        ctx.check_hostname = False
        c = http.client.HTTPSConnection("127.0.0.1", srv.port, timeout=10, context=ctx)
        for j in range(20):
            c.request("GET", "/hello?x=%d" % j)
            r = c.getresponse()
            assert r.status == 200 and r.read() == b"hello %d" % j
        big = bytes(range(256)) * 2000
        c.request("POST", "/echo", body=iter([big[:1000], big[1000:]]),
                  headers={"Transfer-Encoding": "chunked"}, encode_chunked=True)
        r = c.getresponse()
        assert r.status == 200 and r.read() == big
        c.close()
        # pipelined over one TLS connection
        raw = socket.create_connection(("127.0.0.1", srv.port), timeout=10)
        s = ctx.wrap_socket(raw, server_hostname="127.0.0.1")
        s.sendall(b"".join(b"GET /hello?x=%d HTTP/1.1\r\nHost: x\r\n\r\n" % j
                           for j in range(10)))
        out = _recv_responses(s, 10)
        s.close()
        assert [o[2] for o in out] == [b"hello %d" % j for j in range(10)]
        # concurrent TLS clients
        errs = []

        def client(cid):
            try:
                cc = http.client.HTTPSConnection("127.0.0.1", srv.port, timeout=20, context=ctx)
                for j in range(10):
                    cc.request("GET", "/hello?x=%d-%d" % (cid, j))
                    rr = cc.getresponse()
                    assert rr.read() == b"hello %d-%d" % (cid, j)
                cc.close()
            except Exception as e:   # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=client, args=(i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(30)
        assert not errs, errs[:2]
        # plain HTTP against the TLS port gets no HTTP answer
        with pytest.raises(Exception):
            pc = http.client.HTTPConnection("127.0.0.1", srv.port, timeout=5)
            pc.request("GET", "/hello")
            pc.getresponse().read()
    finally:
        srv.shutdown()
        srv.server_close()
