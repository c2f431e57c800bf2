"""Topic producers over the native log.

Equivalents of the reference's Kafka producer wrappers (``[lambda]/TopicProducerImpl.java:32-84``
and ``[lserving]/TopicProducerImpl.java:32-81``): lazily opened, synchronous (the batch
layer's ``MODEL`` publish) or asynchronous with batching (``UP`` streams, serving ingest).
Async producers buffer records and append them with one native call per batch
(batch 100 / 10 ms linger by default), so millions of ``UP`` rows cost few syscalls.
"""

from __future__ import annotations

import logging
import threading
import time
from typing import List, Optional, Tuple

from ..api import TopicProducer
from . import log as tlog

__all__ = ["LogTopicProducer", "MockTopicProducer", "open_topic", "topic_root"]

_log = logging.getLogger(__name__)


def topic_root(broker: Optional[str], config=None) -> str:
    return tlog.log_root_for(broker, config)


def open_topic(broker: Optional[str], topic: str, config=None, create_partitions: int = 0,
               max_message: int = 16777216) -> tlog.Topic:
    root = topic_root(broker, config)
    if create_partitions and not tlog.topic_exists(root, topic):
        tlog.maybe_create_topic(root, topic, create_partitions, max_message)
    return tlog.Topic(root, topic)


class LogTopicProducer(TopicProducer):
    def __init__(self, broker: str, topic: str, config=None, async_: bool = True,
                 batch_size: int = 100, linger_ms: float = 10.0, create_partitions: int = 1,
                 max_message: int = 16777216):
        self._broker = broker
        self._topic_name = topic
        self._config = config
        self._async = async_
        self._batch_size = int(batch_size)
        self._linger = linger_ms / 1000.0
        self._create_partitions = create_partitions
        self._max_message = max_message
        self._topic: Optional[tlog.Topic] = None
        self._buf: List[Tuple[Optional[str], str]] = []
        self._lock = threading.Condition(threading.Lock())
        self._closed = False
        self._flusher: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None

    # lazily opened, as the reference does
    def _get_topic(self) -> tlog.Topic:
        if self._topic is None:
            self._topic = open_topic(self._broker, self._topic_name, self._config,
                                     create_partitions=self._create_partitions,
                                     max_message=self._max_message)
        return self._topic

    def get_update_broker(self) -> str:
        return self._broker

    def get_topic(self) -> str:
        return self._topic_name

    def send(self, key: Optional[str], message: str) -> None:
        if not self._async:
            self._get_topic().append(key, message)
            return
        with self._lock:
            if self._error is not None:
                raise self._error
            self._buf.append((key, message))
            if self._flusher is None:
                self._flusher = threading.Thread(target=self._run, name="oryx-producer",
                                                 daemon=True)
                self._flusher.start()
            if len(self._buf) >= self._batch_size:
                self._lock.notify()

    def send_many(self, pairs) -> None:
        pairs = list(pairs)
        if not self._async:
            if pairs:
                self._get_topic().append_batch(pairs)
            return
        with self._lock:
            self._buf.extend(pairs)
            if self._flusher is None:
                self._flusher = threading.Thread(target=self._run, name="oryx-producer",
                                                 daemon=True)
                self._flusher.start()
            self._lock.notify()

    def send_block(self, key: Optional[str], block) -> None:
        """Messages queued before are appended first, then the block in one native call."""
        if len(block) == 0:
            return
        self._drain()
        try:
            self._get_topic().append_block(block, key=key)
        except tlog.MessageTooLargeError:
            # per-message size errors: the per-record path drops just the oversized ones
            self.send_many((key, m) for m in block)
            self._drain()

    def _drain(self) -> None:
        with self._lock:
            batch, self._buf = self._buf, []
        if batch:
            try:
                # per-record max-size errors surface here; keep going with the rest
                self._get_topic().append_batch(batch)
            except tlog.MessageTooLargeError as e:
                for rec in batch:
                    try:
                        self._get_topic().append(*rec)
                    except tlog.MessageTooLargeError:
                        _log.error("Dropping message larger than max size: %s", e)

    def _run(self) -> None:
        while True:
            with self._lock:
                if not self._buf and not self._closed:
                    self._lock.wait(self._linger)
                if self._closed and not self._buf:
                    return
            try:
                self._drain()
            except BaseException as e:  # surfaced on next send
                _log.exception("Async producer failed")
                with self._lock:
                    self._error = e
                return
            time.sleep(0)

    def flush(self) -> None:
        self._drain()

    def close(self) -> None:
        with self._lock:
            self._closed = True
            self._lock.notify_all()
        if self._flusher is not None:
            self._flusher.join(timeout=30)
        self._drain()
        if self._topic is not None:
            self._topic.close()
            self._topic = None


class MockTopicProducer(TopicProducer):
    """Records sent (key, message) pairs (``T[lserving]/MockTopicProducer.java:24-47``)."""

    KEY_MESSAGES: List[Tuple[Optional[str], str]] = []

    def __init__(self, *args, **kwargs):
        pass

    def get_update_broker(self) -> str:
        return "mock"

    def get_topic(self) -> str:
        return "mock"

    def send(self, key, message) -> None:
        MockTopicProducer.KEY_MESSAGES.append((key, message))

    @classmethod
    def get_key_messages(cls):
        return cls.KEY_MESSAGES

    @classmethod
    def clear(cls):
        cls.KEY_MESSAGES.clear()
