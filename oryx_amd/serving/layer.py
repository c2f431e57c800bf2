"""The serving layer: HTTP API over an in-memory (GPU-resident) model fed by the update topic.

Equivalent of ``ServingLayer`` + ``ModelManagerListener`` (``[lserving]/ServingLayer.java:88-339``,
``[lserving]/ModelManagerListener.java:103-224``):

* loads ``oryx.serving.model-manager-class`` by name (reference Java names are aliased);
* unless ``oryx.serving.api.read-only``, opens an async producer on the input topic
  (``/ingest``, ``/pref``, ``/add``, ``/train`` write there);
* starts a consumer thread that replays the update topic **from the beginning** into
  ``manager.consume`` and keeps tailing it;
* serves the resources of ``oryx.serving.application-resources`` (plus ``/ready``,
  ``/error``, ``/metrics``) on ``oryx.serving.api.port`` -- or HTTPS on ``secure-port`` when a
  key/cert is configured -- with optional DIGEST auth and a context path.
"""

from __future__ import annotations

import ctypes
import gc
import logging
import os
import ssl
import tempfile
import threading
import time
from typing import Iterator, List, Optional, Tuple

from .. import native
from ..api import KeyMessage, ServingModelManager
from ..metrics import Registry
from ..transport import log as tlog
from ..transport.producer import LogTopicProducer, topic_root
from ..utils import config as cfg
from ..utils import ioutils, lang
from . import http
from .resources import INPUT_PRODUCER_KEY, MODEL_MANAGER_KEY

__all__ = ["ServingLayer", "UpdateIterator", "resource_modules"]

log = logging.getLogger(__name__)


class UpdateIterator:
    """Blocking iterator of :class:`KeyMessage` over a topic, until closed."""

    # records decoded into Python objects per poll: small, because a manager that can parse a
    # run of UP rows natively (take_up_block) takes the rest of the run from the log itself
    # (8192 decoded 2.7 KB rows cost ~0.4 s at the start of every model load)
    POLL_RECORDS = 256

    def __init__(self, consumer: tlog.TopicConsumer, poll_ms: int = 100):
        self.consumer = consumer
        self.poll_ms = poll_ms
        self.closed = False
        self._pending: List = []
        self._rr = 0

    def __iter__(self):
        return self

    def __next__(self) -> KeyMessage:
        while not self._pending:
            if self.closed:
                raise StopIteration
            recs = self.consumer.poll(self.POLL_RECORDS, self.poll_ms)
            self._pending = [KeyMessage(k, v) for _, _, _, k, v in recs]
            self._pending.reverse()
        return self._pending.pop()

    def has_buffered(self) -> bool:
        return bool(self._pending)

    def take_buffered(self, pred, max_n: int = 1 << 16, poll: bool = True
                      ) -> List[KeyMessage]:
        """Already-fetched messages from the front while ``pred`` holds (no blocking) -- lets
        a manager apply a run of ``UP`` rows as one batch; ``poll`` also fetches (without
        waiting) what the log already holds while the run continues."""
        out: List[KeyMessage] = []
        if not poll:
            while self._pending and len(out) < max_n and pred(self._pending[-1]):
                out.append(self._pending.pop())
            return out
        if not self._pending and not self.closed:
            recs = self.consumer.poll(self.POLL_RECORDS, 0)
            self._pending = [KeyMessage(k, v) for _, _, _, k, v in recs]
            self._pending.reverse()
        while self._pending and len(out) < max_n and pred(self._pending[-1]):
            out.append(self._pending.pop())
            if not self._pending and len(out) < max_n and not self.closed:
                recs = self.consumer.poll(self.POLL_RECORDS, 0)
                self._pending = [KeyMessage(k, v) for _, _, _, k, v in recs]
                self._pending.reverse()
        return out

    def take_up_block(self, k: int, max_n: int = 1 << 15, known_dict=None):
        """The next run of ``UP`` records parsed natively straight from the log's raw poll
        buffer -- no per-message Python objects -- as (kinds, ids, vectors [n, k], known
        lists); None when nothing is buffered-free to read or the next record is not a
        parseable ``UP`` (the records after the run are queued as ordinary messages).  Only
        used when no already-decoded messages are pending, so the order is kept."""
        if self._pending or self.closed:
            return None
        from .. import ingest
        readers = self.consumer.readers
        for step in range(len(readers)):
            r = readers[(self._rr + step) % len(readers)]
            t0 = time.perf_counter()
            n = r.poll_frames(max_n)
            if not n:
                continue
            t1 = time.perf_counter()
            self._rr = (self._rr + step + 1) % len(readers)
            addr, used = r.frame_buffer()
            got, consumed, kinds, ids, vecs, known = ingest.parse_up_records(
                addr, used, n, k, n, known_dict=known_dict, frames=True)
            t2 = time.perf_counter()
            rest = r.decode_frames(consumed, n - got)
            TAKE_STATS["poll_s"] += t1 - t0
            TAKE_STATS["parse_s"] += t2 - t1
            TAKE_STATS["rest_s"] += time.perf_counter() - t2
            self._pending = [KeyMessage(key, v) for _, _, key, v in rest]
            self._pending.reverse()
            return (kinds, ids, vecs, known) if got else None
        return None

    def close(self) -> None:
        self.closed = True


# where the bulk UP reads of take_up_block spend their time (bench records read these)
TAKE_STATS = {"poll_s": 0.0, "parse_s": 0.0, "rest_s": 0.0}


def resource_modules(config) -> List[str]:
    mods = ["oryx_amd.serving.resources"]
    names = cfg.get_optional_string(config, "oryx.serving.application-resources")
    if names:
        for n in names.split(","):
            n = n.strip()
            if n:
                mods.append(lang.JAVA_CLASS_ALIASES.get(n, n))
    else:
        mgr = cfg.get_optional_string(config, "oryx.serving.model-manager-class")
        if mgr:
            mgr = lang.JAVA_CLASS_ALIASES.get(mgr, mgr)
            pkg = mgr.rsplit(".", 2)[0]
            mods.append(pkg + ".resources")
    out = []
    for m in mods:
        if m not in out:
            out.append(m)
    return out


def keystore_pem(path: str, password: Optional[str], alias: Optional[str] = None
                 ) -> Optional[Tuple[bytes, bytes]]:
    """(certificate chain PEM, private key PEM) of a JKS or PKCS#12 keystore, or None when
    ``path`` is not a keystore (PEM).  Raises ``ValueError`` for a wrong password or a file it
    cannot read (native parser: ``csrc/runtime/oryx_keystore.cpp``)."""
    lib = native.runtime()
    cert_p, key_p = ctypes.c_void_p(), ctypes.c_void_p()
    cert_n, key_n = ctypes.c_longlong(), ctypes.c_longlong()
    enc = (lambda v: v.encode() if v is not None else None)
    rc = lib.oryx_keystore_to_pem(enc(path), enc(password), enc(alias), ctypes.byref(cert_p),
                                  ctypes.byref(cert_n), ctypes.byref(key_p),
                                  ctypes.byref(key_n))
    if rc == 1:
        return None
    if rc != 0:
        raise ValueError("keystore %s: %s" % (path, (lib.oryx_keystore_error() or b"")
                                              .decode(errors="replace")))
    try:
        return (ctypes.string_at(cert_p.value, cert_n.value),
                ctypes.string_at(key_p.value, key_n.value))
    finally:
        lib.oryx_keystore_free(cert_p)
        lib.oryx_keystore_free(key_p)


class ServingLayer:
    def __init__(self, config, manager: Optional[ServingModelManager] = None,
                 input_producer=None, host: str = "0.0.0.0"):
        self.config = config
        self.host = host
        self.read_only = config.get_bool("oryx.serving.api.read-only")
        self.port = config.get_int("oryx.serving.api.port")
        self.secure_port = config.get_int("oryx.serving.api.secure-port")
        self.user_name = cfg.get_optional_string(config, "oryx.serving.api.user-name")
        self.password = cfg.get_optional_string(config, "oryx.serving.api.password")
        self.keystore_file = cfg.get_optional_string(config, "oryx.serving.api.keystore-file")
        self.key_file = cfg.get_optional_string(config, "oryx.serving.api.key-file")
        self.keystore_password = cfg.get_optional_string(config,
                                                         "oryx.serving.api.keystore-password")
        self.context_path = config.get_string("oryx.serving.api.context-path")
        self.native_http = config.get_bool("oryx.serving.api.native-http")
        self.handler_threads = config.get_int("oryx.serving.api.handler-threads")
        self.update_topic = config.get_string("oryx.update-topic.message.topic")
        self.update_broker = config.get_string("oryx.update-topic.broker")
        self.input_topic = config.get_string("oryx.input-topic.message.topic")
        self.input_broker = config.get_string("oryx.input-topic.broker")
        self.max_message = config.get_int("oryx.update-topic.message.max-size")
        self._manager = manager
        self._input_producer = input_producer
        self._server = None       # http.NativeHTTPServer or http.OryxHTTPServer
        self._consumer_thread: Optional[threading.Thread] = None
        self._updates: Optional[UpdateIterator] = None
        self._consumer: Optional[tlog.TopicConsumer] = None
        self._closed = threading.Event()
        self.metrics = Registry()
        self.context: dict = {"config": config, "metrics": self.metrics}

    # ---------------------------------------------------------------- lifecycle
    def _load_manager(self) -> ServingModelManager:
        name = self.config.get_string("oryx.serving.model-manager-class")
        return lang.load_instance_of(name, None, self.config)

    def start(self) -> "ServingLayer":
        log.info("Starting serving layer")
        if self._manager is None:
            self._manager = self._load_manager()
        self.context[MODEL_MANAGER_KEY] = self._manager
        no_init = self.config.get_bool("oryx.serving.no-init-topics")
        if not self.read_only:
            if self._input_producer is None:
                partitions = self.config.get_int("oryx.input-topic.partitions")
                self._input_producer = LogTopicProducer(self.input_broker, self.input_topic,
                                                        self.config, async_=True,
                                                        create_partitions=partitions)
            self.context[INPUT_PRODUCER_KEY] = self._input_producer
        if not no_init:
            self._start_update_consumer()
        router = http.Router(http.collect_routes(resource_modules(self.config)),
                             self.context_path)
        ssl_ctx = self._ssl_context()
        auth = None
        if self.user_name and self.password:
            auth = http.DigestAuth(self.user_name, self.password)
        port = self.secure_port if ssl_ctx is not None else self.port
        tls_files = None
        if ssl_ctx is not None:
            tls_files = (ioutils.to_local_path(self.keystore_file),
                         ioutils.to_local_path(self.key_file) if self.key_file else None,
                         self.keystore_password)
        # the native front end (csrc/runtime/oryx_http.cpp: HTTP, or HTTPS through OpenSSL)
        # unless oryx.serving.api.native-http is false
        self._server = http.make_server(self.host, port, router, self.context, ssl_ctx, auth,
                                        self.metrics, native=self.native_http,
                                        threads=self.handler_threads, tls_files=tls_files)
        # everything built so far (modules, torch, the router) lives as long as the process:
        # out of the cyclic GC's generations, so a gen-2 pass under traffic walks only what
        # requests and updates allocate (handlers stop for the whole pass)
        gc.freeze()
        self._server.start_background()
        log.info("Serving layer listening on %s:%d%s", self.host, self._server.port,
                 " (HTTPS)" if ssl_ctx else "")
        lang.close_at_shutdown(self)
        return self

    def _ssl_context(self) -> Optional[ssl.SSLContext]:
        """HTTPS when ``keystore-file`` is set: a Java keystore (JKS or PKCS#12, unlocked by
        ``keystore-password``, as the reference's Tomcat connector takes it:
        ``ServingLayer.java:214-217``) or a PEM certificate chain (+ ``key-file``)."""
        cert = self.keystore_file
        if not cert:
            return None
        cert = ioutils.to_local_path(cert)
        key = ioutils.to_local_path(self.key_file) if self.key_file else None
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        pem = keystore_pem(cert, self.keystore_password)
        if pem is None:
            ctx.load_cert_chain(cert, key, password=self.keystore_password)
            return ctx
        # ssl loads only files: the keystore's PEM form goes through a private temporary
        # directory that exists only while it is loaded (the native front end reads the
        # keystore itself, oryx_keystore.cpp)
        with tempfile.TemporaryDirectory(prefix="oryx-tls-") as d:
            cp, kp = os.path.join(d, "cert.pem"), os.path.join(d, "key.pem")
            for path, text in ((cp, pem[0]), (kp, pem[1])):
                fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
                with os.fdopen(fd, "wb") as fh:
                    fh.write(text)
            ctx.load_cert_chain(cp, kp)
        return ctx

    def _start_update_consumer(self) -> None:
        root = topic_root(self.update_broker, self.config)
        tlog.maybe_create_topic(root, self.update_topic, 1, self.max_message)
        topic = tlog.Topic(root, self.update_topic)
        self._consumer = tlog.TopicConsumer(topic, start="earliest")
        self._updates = UpdateIterator(self._consumer)

        def run():
            try:
                self._manager.consume(self._updates, None)
            except Exception:
                log.exception("Error while consuming updates")
                self.close()

        self._consumer_thread = threading.Thread(target=run,
                                                 name="OryxServingLayerUpdateConsumerThread",
                                                 daemon=True)
        self._consumer_thread.start()

    @property
    def actual_port(self) -> int:
        return self._server.port if self._server else -1

    @property
    def manager(self) -> Optional[ServingModelManager]:
        return self._manager

    def await_termination(self, timeout: Optional[float] = None) -> None:
        self._closed.wait(timeout)

    def close(self) -> None:
        if self._closed.is_set():
            return
        self._closed.set()
        log.info("Shutting down serving layer")
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
        if self._updates is not None:
            self._updates.close()
        if self._consumer_thread is not None:
            self._consumer_thread.join(timeout=10)
        if self._consumer is not None:
            self._consumer.close()
        if self._manager is not None:
            self._manager.close()
        if self._input_producer is not None:
            self._input_producer.close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.close()
        return False
