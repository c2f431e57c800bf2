"""Minimal JAX-RS-style REST framework for the serving layer.

Replaces the reference's embedded Tomcat + Jersey stack (``[lserving]/ServingLayer.java:55-339``,
``OryxApplication.java:54-96``, ``CSVMessageBodyWriter.java:60-85``,
``OryxExceptionMapper.java:27-38``, ``ErrorResource.java:35-128``, ``InMemoryRealm.java:47-85``):

* resources are plain functions registered with :func:`route` using JAX-RS path templates
  (``/recommend/{userID}``, ``/recommendToMany/{userID : .+}`` -> list of path segments);
* responses are negotiated from ``Accept``: ``application/json`` (Jackson-like rendering of
  ``IDValue`` etc. via ``to_json()``), ``text/csv`` / ``text/plain`` (one ``to_csv()`` line
  per element, like ``CSVMessageBodyWriter``);
* ``OryxServingException(status, msg)`` -> that status with an HTML / plain-text error body;
* request bodies: ``Content-Encoding`` gzip/deflate, ``multipart/form-data`` parts (with
  ``application/gzip`` / ``application/zip`` part decompression done by resources);
* response compression (gzip / deflate) for text, CSV and JSON when the client accepts it;
* optional HTTPS (PEM cert + key) and HTTP DIGEST authentication (RFC 2617, MD5, qop=auth);
* context path prefix; HTTP/1.1 keep-alive; one thread per connection.
"""

from __future__ import annotations

import email.parser
import email.utils
import gzip
import hashlib
import http.server
import io
import json
import logging
import math
import os
import re
import secrets
import socketserver
import ssl
import struct
import threading
import time
import urllib.parse
import zlib
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

from ..api import OryxServingException

__all__ = ["route", "Route", "Request", "Response", "Router", "OryxHTTPServer", "Part",
           "collect_routes", "render_body", "HTTP_STATUS"]

log = logging.getLogger(__name__)

HTTP_STATUS = {200: "OK", 204: "No Content", 400: "Bad Request", 401: "Unauthorized",
               403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed",
               406: "Not Acceptable", 415: "Unsupported Media Type",
               500: "Internal Server Error", 503: "Service Unavailable"}

TEXT = "text/plain"
CSV = "text/csv"
JSON = "application/json"
HTML = "text/html"
DEFAULT_PRODUCES = (TEXT, CSV, JSON)


class Part:
    """One multipart/form-data part."""

    def __init__(self, name: Optional[str], filename: Optional[str], content_type: Optional[str],
                 data: bytes):
        self.name = name
        self.filename = filename
        self.content_type = content_type
        self.data = data

    def get_input_stream(self) -> io.BytesIO:
        return io.BytesIO(self.data)


class Request:
    def __init__(self, method: str, path: str, query: Dict[str, List[str]],
                 headers: Dict[str, str], body: bytes, context: dict):
        self.method = method
        self.path = path
        self.query = query
        self.headers = headers
        self.raw_body = body
        self.context = context
        self.path_params: Dict[str, Any] = {}

    def header(self, name: str, default: Optional[str] = None) -> Optional[str]:
        return self.headers.get(name.lower(), default)

    @property
    def content_type(self) -> str:
        return (self.header("content-type") or "").split(";")[0].strip().lower()

    def body(self) -> bytes:
        enc = (self.header("content-encoding") or "").lower()
        data = self.raw_body
        if enc == "gzip":
            data = gzip.decompress(data)
        elif enc == "deflate":
            try:
                data = zlib.decompress(data)
            except zlib.error:
                data = zlib.decompress(data, -zlib.MAX_WBITS)
        return data

    def text(self) -> str:
        return self.body().decode("utf-8")

    def q(self, name: str, default=None):
        v = self.query.get(name)
        return v[0] if v else default

    def q_int(self, name: str, default: int) -> int:
        v = self.q(name)
        if v is None:
            return default
        try:
            return int(v)
        except ValueError:
            raise OryxServingException(404, "Bad parameter %s" % name)

    def q_bool(self, name: str, default: bool) -> bool:
        v = self.q(name)
        if v is None:
            return default
        return v.lower() == "true"

    def q_list(self, name: str) -> List[str]:
        return list(self.query.get(name, []))

    def is_multipart(self) -> bool:
        return self.content_type.startswith("multipart/")

    def multipart_parts(self) -> List[Part]:
        ctype = self.header("content-type") or ""
        msg = email.parser.BytesParser().parsebytes(
            b"Content-Type: " + ctype.encode("latin-1") + b"\r\n\r\n" + self.body())
        if not msg.is_multipart():
            raise OryxServingException(400, "Not multipart")
        parts = []
        for p in msg.get_payload():
            disp = p.get("Content-Disposition", "")
            name = p.get_param("name", header="content-disposition")
            filename = p.get_filename()
            payload = p.get_payload(decode=True) or b""
            parts.append(Part(name, filename, p.get_content_type() if p.get("Content-Type")
                              else None, payload))
        if not parts:
            raise OryxServingException(400, "No parts")
        return parts


class Response:
    def __init__(self, status: int = 200, body: bytes = b"", content_type: Optional[str] = None,
                 headers: Optional[Dict[str, str]] = None):
        self.status = status
        self.body = body
        self.content_type = content_type
        self.headers = headers or {}


class Route:
    def __init__(self, method: str, template: str, fn: Callable, produces=DEFAULT_PRODUCES,
                 consumes: Optional[Tuple[str, ...]] = None):
        self.method = method.upper()
        self.template = template
        self.fn = fn
        self.produces = tuple(produces)
        self.consumes = consumes
        self.regex, self.params = self._compile(template)
        # literal prefix length: more specific routes win (JAX-RS ordering approximation)
        self.literal_len = len(re.sub(r"\{[^}]*\}", "", template))

    @staticmethod
    def _compile(template: str):
        params = []
        out = []
        pos = 0
        for m in re.finditer(r"\{\s*(\w+)\s*(?::\s*([^}]+?))?\s*\}", template):
            lit = template[pos:m.start()]
            name, rx = m.group(1), m.group(2)
            multi = rx is not None and ("+" in rx or "*" in rx)
            params.append((name, multi))
            if rx is not None and rx.strip() == ".*" and lit.endswith("/"):
                # '/x/{p : .*}' also matches '/x' (empty list of segments)
                out.append(re.escape(lit[:-1]))
                out.append("(?:/(?P<%s>.*))?" % name)
            else:
                out.append(re.escape(lit))
                out.append("(?P<%s>%s)" % (name, rx if rx else "[^/]+"))
            pos = m.end()
        out.append(re.escape(template[pos:]))
        return re.compile("^" + "".join(out) + "/?$"), params

    def match(self, path: str) -> Optional[Dict[str, Any]]:
        m = self.regex.match(path)
        if not m:
            return None
        res = {}
        for name, multi in self.params:
            raw = m.group(name) or ""
            if multi:
                res[name] = [urllib.parse.unquote(s) for s in raw.split("/") if s != ""]
            else:
                res[name] = urllib.parse.unquote(raw)
        return res


_ROUTES: Dict[str, List[Route]] = {}


def route(method: str, template: str, produces=DEFAULT_PRODUCES, consumes=None):
    """Decorator registering ``fn(request, **path_params)`` in the calling module's routes."""
    def deco(fn):
        mod = fn.__module__
        _ROUTES.setdefault(mod, []).append(Route(method, template, fn, produces, consumes))
        return fn
    return deco


def collect_routes(module_names: Iterable[str]) -> List[Route]:
    import importlib
    routes: List[Route] = []
    seen = set()
    pending = list(module_names)
    while pending:
        name = pending.pop(0)
        if name in seen:
            continue
        seen.add(name)
        mod = importlib.import_module(name)
        routes.extend(_ROUTES.get(mod.__name__, []))
        # an app package may pull in a generic one (e.g. kmeans -> clustering endpoints)
        pending.extend(getattr(mod, "INCLUDE_RESOURCES", ()))
    return routes


# ---------------------------------------------------------------- rendering

def _json_default(o):
    if hasattr(o, "to_json"):
        return o.to_json()
    if isinstance(o, (set, frozenset)):
        return list(o)
    try:
        import numpy as np
        if isinstance(o, np.generic):
            return o.item()
        if isinstance(o, np.ndarray):
            return o.tolist()
    except ImportError:
        pass
    raise TypeError("not JSON serializable: %r" % type(o))


def _fmt_scalar(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        from ..utils.text import java_double_str
        return java_double_str(v)
    return str(v)


def _csv_line(v) -> str:
    if hasattr(v, "to_csv"):
        return v.to_csv()
    return _fmt_scalar(v)


def render_body(value, media: str) -> Tuple[bytes, str]:
    if value is None:
        return b"", media
    if media == JSON:
        return json.dumps(value, default=_json_default, separators=(",", ":"),
                          allow_nan=True).encode("utf-8"), JSON
    if isinstance(value, (bytes, bytearray)):
        return bytes(value), media
    if isinstance(value, str):
        return value.encode("utf-8"), media
    if isinstance(value, (list, tuple, set, frozenset)) or hasattr(value, "__iter__") and \
            not isinstance(value, dict):
        lines = [_csv_line(v) for v in value]
        return ("".join(l + "\n" for l in lines)).encode("utf-8"), media
    return (_csv_line(value) + "\n").encode("utf-8"), media


def _negotiate(accept: Optional[str], produces: Tuple[str, ...]) -> Optional[str]:
    if not accept:
        return produces[0]
    best, best_q = None, -1.0
    for item in accept.split(","):
        parts = item.strip().split(";")
        mt = parts[0].strip().lower()
        qv = 1.0
        for p in parts[1:]:
            p = p.strip()
            if p.startswith("q="):
                try:
                    qv = float(p[2:])
                except ValueError:
                    qv = 0.0
        for cand in produces:
            if mt == cand or mt == "*/*" or (mt.endswith("/*") and cand.startswith(mt[:-1])):
                # exact matches beat wildcards at equal q
                score = qv + (0.001 if mt == cand else 0.0)
                if score > best_q:
                    best, best_q = cand, score
                break
    return best


def error_body(status: int, message: Optional[str], media: str) -> Tuple[bytes, str]:
    reason = HTTP_STATUS.get(status, "")
    msg = message or ""
    if media == HTML:
        esc = (msg.replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;"))
        body = ("<!DOCTYPE html><html><head><title>Error %d</title></head><body>"
                "<h1>Error %d %s</h1><p>%s</p></body></html>" % (status, status, reason, esc))
        return body.encode("utf-8"), HTML
    return ("%d %s\n%s\n" % (status, reason, msg)).encode("utf-8"), TEXT


class Router:
    def __init__(self, routes: List[Route], context_path: str = "/"):
        self.routes = sorted(routes, key=lambda r: -r.literal_len)
        cp = context_path or "/"
        self.context_path = "" if cp == "/" else "/" + cp.strip("/")

    def dispatch(self, req: Request) -> Response:
        path = req.path
        if self.context_path:
            if not (path == self.context_path or path.startswith(self.context_path + "/")):
                return self._error(req, 404, path)
            path = path[len(self.context_path):] or "/"
        candidates = []
        for r in self.routes:
            params = r.match(path)
            if params is not None:
                candidates.append((r, params))
        if not candidates:
            return self._error(req, 404, path)
        method = "GET" if req.method == "HEAD" else req.method
        matching = [(r, p) for r, p in candidates if r.method == method]
        if not matching:
            return self._error(req, 405, req.method)
        if len(matching) > 1 and req.method in ("POST", "PUT"):
            ct = req.content_type
            pref = [(r, p) for r, p in matching if r.consumes and ct and any(
                ct.startswith(c) for c in r.consumes)]
            if pref:
                matching = pref
        r, params = matching[0]
        media = _negotiate(req.header("accept"), r.produces)
        if media is None:
            return self._error(req, 406, "Not acceptable")
        req.path_params = params
        try:
            value = r.fn(req, **params)
        except OryxServingException as e:
            return self._error(req, e.status, e.message)
        except (ValueError, TypeError, KeyError) as e:
            log.debug("Bad request %s: %s", path, e, exc_info=True)
            return self._error(req, 400, str(e))
        except Exception as e:  # 500 with log, like the reference's exception mapper
            log.exception("Unexpected error serving %s", path)
            return self._error(req, 500, str(e))
        if isinstance(value, Response):
            return value
        if value is None:
            return Response(204 if req.method in ("POST", "PUT", "DELETE") else 200, b"", None)
        body, ctype = render_body(value, media)
        return Response(200, body, ctype)

    def _error(self, req: Request, status: int, message: Optional[str]) -> Response:
        accept = req.header("accept") or ""
        media = HTML if "text/html" in accept else TEXT
        body, ctype = error_body(status, message, media)
        return Response(status, b"" if req.method == "HEAD" else body, ctype)


# ---------------------------------------------------------------- auth

class DigestAuth:
    """HTTP DIGEST authentication (RFC 2617, MD5, qop=auth) against one user/password.

    The response is bound to the request target (the ``uri`` parameter must equal it), nonces
    expire after ``nonce_ttl_s`` (answered with ``stale=true`` so clients retry without
    prompting) and each nonce's ``nc`` must strictly increase, so a captured Authorization
    header can neither be replayed nor pointed at another endpoint.
    """

    def __init__(self, user: str, password: str, realm: str = "Oryx",
                 nonce_ttl_s: float = 300.0):
        self.user = user
        self.password = password
        self.realm = realm
        self.nonce_ttl_s = float(nonce_ttl_s)
        self._nonces: Dict[str, list] = {}      # nonce -> [issued_at, last nc]
        self._lock = threading.Lock()

    def challenge(self, stale: bool = False) -> str:
        nonce = secrets.token_hex(16)
        now = time.time()
        with self._lock:
            self._nonces[nonce] = [now, 0]
            if len(self._nonces) > 1024:
                cutoff = now - self.nonce_ttl_s
                self._nonces = {n: v for n, v in self._nonces.items() if v[0] > cutoff}
        return 'Digest realm="%s", qop="auth", nonce="%s", opaque="%s"%s' % (
            self.realm, nonce, hashlib.md5(self.realm.encode()).hexdigest(),
            ", stale=true" if stale else "")

    @staticmethod
    def _parse(header: str) -> Dict[str, str]:
        out = {}
        for m in re.finditer(r'(\w+)\s*=\s*(?:"([^"]*)"|([^,\s]*))', header):
            out[m.group(1).lower()] = m.group(2) if m.group(2) is not None else m.group(3)
        return out

    def verify(self, method: str, target: str, header: Optional[str]) -> str:
        """``"ok"``, ``"stale"`` (right credentials, expired nonce) or ``"denied"``."""
        if not header or not header.lower().startswith("digest "):
            return "denied"
        p = self._parse(header[7:])
        if p.get("username") != self.user or p.get("realm") != self.realm:
            return "denied"
        if p.get("uri", "") != target:
            return "denied"
        ha1 = hashlib.md5(("%s:%s:%s" % (self.user, self.realm, self.password)).encode()).hexdigest()
        ha2 = hashlib.md5(("%s:%s" % (method, p.get("uri", ""))).encode()).hexdigest()
        if p.get("qop") != "auth":
            return "denied"
        expected = hashlib.md5(("%s:%s:%s:%s:%s:%s" % (
            ha1, p.get("nonce"), p.get("nc"), p.get("cnonce"), p.get("qop"), ha2)).encode()
        ).hexdigest()
        if not secrets.compare_digest(expected, p.get("response", "")):
            return "denied"
        try:
            nc = int(p.get("nc", ""), 16)
        except ValueError:
            return "denied"
        with self._lock:
            entry = self._nonces.get(p.get("nonce"))
            if entry is None:
                return "stale"
            if time.time() - entry[0] > self.nonce_ttl_s:
                del self._nonces[p.get("nonce")]
                return "stale"
            if nc <= entry[1]:
                return "denied"                  # replayed (or reordered) request
            entry[1] = nc
        return "ok"

    def check(self, method: str, header: Optional[str], target: str = "") -> bool:
        return self.verify(method, target, header) == "ok"


# ---------------------------------------------------------------- server

_COMPRESSIBLE = (TEXT, CSV, JSON, HTML)


class _Handler(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "Oryx"
    sys_version = ""
    # TCP_NODELAY: with keep-alive, Nagle + the client's delayed ACK would add ~40 ms to
    # every response
    disable_nagle_algorithm = True

    def log_message(self, fmt, *args):
        log.debug("%s - %s", self.address_string(), fmt % args)

    def _handle(self):
        srv = self.server
        t0 = time.perf_counter()
        length = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(length) if length > 0 else b""
        if self.headers.get("Transfer-Encoding", "").lower() == "chunked":
            body = self._read_chunked()
        parsed = urllib.parse.urlsplit(self.path)
        query = urllib.parse.parse_qs(parsed.query, keep_blank_values=True)
        headers = {k.lower(): v for k, v in self.headers.items()}
        req = Request(self.command, parsed.path, query, headers, body, srv.app_context)
        verdict = "ok" if srv.auth is None else srv.auth.verify(
            self.command, self.path, headers.get("authorization"))
        if verdict != "ok":
            resp = Response(401, b"401 Unauthorized\n", TEXT,
                            {"WWW-Authenticate": srv.auth.challenge(stale=verdict == "stale")})
        else:
            resp = srv.router.dispatch(req)
        payload = resp.body
        headers_out = dict(resp.headers)
        if payload and resp.content_type in _COMPRESSIBLE and len(payload) > 64:
            ae = (headers.get("accept-encoding") or "").lower()
            if "gzip" in ae:
                payload = gzip.compress(payload, 5)
                headers_out["Content-Encoding"] = "gzip"
            elif "deflate" in ae:
                payload = zlib.compress(payload, 5)
                headers_out["Content-Encoding"] = "deflate"
        self.send_response(resp.status, HTTP_STATUS.get(resp.status))
        if resp.content_type:
            self.send_header("Content-Type", resp.content_type + "; charset=UTF-8")
        for k, v in headers_out.items():
            self.send_header(k, v)
        self.send_header("Content-Length", str(len(payload)))
        # status line, headers and body leave in ONE write
        self._headers_buffer.append(b"\r\n")
        if self.command != "HEAD" and payload:
            self._headers_buffer.append(payload)
        self.flush_headers()
        if srv.metrics is not None:
            srv.metrics.observe_request(parsed.path, resp.status, time.perf_counter() - t0)

    def _read_chunked(self) -> bytes:
        out = bytearray()
        while True:
            line = self.rfile.readline().strip()
            size = int(line.split(b";")[0], 16)
            if size == 0:
                self.rfile.readline()
                return bytes(out)
            out += self.rfile.read(size)
            self.rfile.readline()

    do_GET = _handle
    do_POST = _handle
    do_PUT = _handle
    do_DELETE = _handle
    do_HEAD = _handle


def _respond_bytes(srv, req_headers: Dict[str, str], method: str, target: str, path: str,
                   resp: "Response", t0: float) -> bytes:
    """A response's bytes as one buffer (compression as negotiated), shared by the servers."""
    payload = resp.body
    headers_out = dict(resp.headers)
    if payload and resp.content_type in _COMPRESSIBLE and len(payload) > 64:
        ae = (req_headers.get("accept-encoding") or "").lower()
        if "gzip" in ae:
            payload = gzip.compress(payload, 5)
            headers_out["Content-Encoding"] = "gzip"
        elif "deflate" in ae:
            payload = zlib.compress(payload, 5)
            headers_out["Content-Encoding"] = "deflate"
    lines = ["HTTP/1.1 %d %s" % (resp.status, HTTP_STATUS.get(resp.status, "")),
             "Server: Oryx", "Date: " + email.utils.formatdate(usegmt=True)]
    if resp.content_type:
        lines.append("Content-Type: " + resp.content_type + "; charset=UTF-8")
    for k, v in headers_out.items():
        lines.append("%s: %s" % (k, v))
    lines.append("Content-Length: %d" % len(payload))
    head = ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")
    if srv.metrics is not None:
        srv.metrics.observe_request(path, resp.status, time.perf_counter() - t0)
    return head + payload if method != "HEAD" and payload else head


class NativeHTTPServer:
    """The serving front end on the native HTTP loop (``csrc/runtime/oryx_http.cpp``: epoll
    accept / parse / keep-alive / pipelining on a native thread): ``threads`` Python handler
    threads take complete requests from its queue (blocking without the GIL) and hand back
    response bytes, so Python runs only routing and the endpoint per request.  Same routes,
    auth, compression and metrics as :class:`OryxHTTPServer` (which keeps the TLS path)."""

    def __init__(self, host: str, port: int, router: "Router", app_context: dict,
                 auth: Optional[DigestAuth] = None, metrics=None, threads: int = 16,
                 max_body: int = 64 << 20, tls: Optional[Tuple[str, Optional[str],
                                                               Optional[str]]] = None):
        from .. import native
        self.router = router
        self.app_context = app_context
        self.auth = auth
        self.metrics = metrics
        self._lib = native.runtime()
        self._h = self._lib.oryx_http_start(host.encode() if host else b"", int(port), 1024,
                                            int(max_body))
        if not self._h:
            raise OSError("cannot listen on %s:%d" % (host, port))
        if tls is not None:
            # HTTPS on the same loop: PEM certificate chain, key (None: in the certificate
            # file), key password (ServingLayer.java:194-245 keystore)
            cert, key, password = tls
            enc = (lambda v: v.encode() if v else None)
            if self._lib.oryx_http_tls(self._h, enc(cert), enc(key), enc(password)) != 0:
                err = (self._lib.oryx_http_tls_error() or b"").decode(errors="replace")
                self._lib.oryx_http_stop(self._h)
                self._lib.oryx_http_free(self._h)
                self._h = None
                raise ssl.SSLError("TLS setup failed: %s" % err)
        self.tls = tls is not None
        self.server_address = (host, int(self._lib.oryx_http_port(self._h)))
        self._threads: List[threading.Thread] = []
        self._n_threads = max(1, int(threads))
        self._stopping = False

    @property
    def port(self) -> int:
        return self.server_address[1]

    def start_background(self) -> threading.Thread:
        for j in range(self._n_threads):
            t = threading.Thread(target=self._work, name="oryx-http-%d" % j, daemon=True)
            t.start()
            self._threads.append(t)
        return self._threads[0]

    def _work(self) -> None:
        import ctypes
        lib, h = self._lib, self._h
        cap = 1 << 16
        buf = ctypes.create_string_buffer(cap)
        while not self._stopping:
            n = lib.oryx_http_next(h, buf, cap, 200)
            if n == 0:
                continue
            if n == -1:
                return
            if n < 0:
                cap = -n
                buf = ctypes.create_string_buffer(cap)
                continue
            raw = ctypes.string_at(buf, n)
            if cap > (1 << 20):             # one large body: do not keep a huge buffer
                cap = 1 << 16
                buf = ctypes.create_string_buffer(cap)
            rid, ml, tl, hl, bl = struct.unpack_from("<QIIIQ", raw, 0)
            o = 28
            method = raw[o:o + ml].decode("latin-1")
            o += ml
            target = raw[o:o + tl].decode("latin-1")
            o += tl
            hraw = raw[o:o + hl].decode("latin-1")
            o += hl
            body = raw[o:o + bl]
            try:
                out, close = self._handle(method, target, hraw, body)
            except Exception:                       # never leave a request unanswered
                log.exception("request failed")
                out = (b"HTTP/1.1 500 Internal Server Error\r\nContent-Length: 0\r\n"
                       b"Connection: close\r\n\r\n")
                close = True
            lib.oryx_http_respond(h, rid, out, len(out), int(close))

    def _handle(self, method: str, target: str, hraw: str, body: bytes):
        t0 = time.perf_counter()
        headers: Dict[str, str] = {}
        for line in hraw.split("\r\n"):
            k, sep, v = line.partition(":")
            if sep:
                key = k.strip().lower()
                v = v.strip()
                headers[key] = headers[key] + ", " + v if key in headers else v
        parsed = urllib.parse.urlsplit(target)
        query = urllib.parse.parse_qs(parsed.query, keep_blank_values=True)
        req = Request(method, parsed.path, query, headers, body, self.app_context)
        verdict = "ok" if self.auth is None else self.auth.verify(
            method, target, headers.get("authorization"))
        if verdict != "ok":
            resp = Response(401, b"401 Unauthorized\n", TEXT,
                            {"WWW-Authenticate": self.auth.challenge(stale=verdict == "stale")})
        else:
            resp = self.router.dispatch(req)
        close = "close" in (headers.get("connection") or "").lower()
        return _respond_bytes(self, headers, method, target, parsed.path, resp, t0), close

    def shutdown(self) -> None:
        self._stopping = True
        self._lib.oryx_http_stop(self._h)
        for t in self._threads:
            t.join(timeout=5)

    def server_close(self) -> None:
        if self._h:
            if not self._stopping:
                self.shutdown()
            if not any(t.is_alive() for t in self._threads):
                self._lib.oryx_http_free(self._h)
            self._h = None


def make_server(host: str, port: int, router: "Router", app_context: dict,
                ssl_context: Optional[ssl.SSLContext] = None,
                auth: Optional[DigestAuth] = None, metrics=None, native: bool = True,
                threads: int = 16,
                tls_files: Optional[Tuple[str, Optional[str], Optional[str]]] = None):
    """The native front end (:class:`NativeHTTPServer`, HTTP or -- with ``tls_files`` =
    (certificate chain, key, password) -- HTTPS); the Python :class:`OryxHTTPServer` when
    ``native`` is off or TLS comes only as an ``ssl_context``."""
    if native and (ssl_context is None or tls_files is not None):
        return NativeHTTPServer(host, port, router, app_context, auth, metrics, threads,
                                tls=tls_files)
    return OryxHTTPServer(host, port, router, app_context, ssl_context, auth, metrics)


class OryxHTTPServer(socketserver.ThreadingMixIn, http.server.HTTPServer):
    daemon_threads = True
    allow_reuse_address = True
    request_queue_size = 1024

    def __init__(self, host: str, port: int, router: Router, app_context: dict,
                 ssl_context: Optional[ssl.SSLContext] = None,
                 auth: Optional[DigestAuth] = None, metrics=None):
        self.router = router
        self.app_context = app_context
        self.auth = auth
        self.metrics = metrics
        super().__init__((host, port), _Handler)
        if ssl_context is not None:
            self.socket = ssl_context.wrap_socket(self.socket, server_side=True)

    @property
    def port(self) -> int:
        return self.server_address[1]

    def start_background(self) -> threading.Thread:
        t = threading.Thread(target=self.serve_forever, name="oryx-http", daemon=True)
        t.start()
        return t
