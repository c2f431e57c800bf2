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
