"""The speed layer: incremental model updates within seconds of new input.

Equivalent of ``SpeedLayer`` + ``SpeedLayerUpdate`` (``[lambda]/speed/SpeedLayer.java:94-200``,
``[lambda]/speed/SpeedLayerUpdate.java:51-64``):

* thread A replays the update topic from the beginning into ``manager.consume`` (so the
  speed model follows every batch ``MODEL`` and every ``UP``, including its own);
* every ``generation-interval-sec`` the interval's new input is handed to
  ``manager.build_updates``; each returned update is published as ``UP`` with an async
  producer, then input offsets are committed.

GPU managers (ALS/k-means/RDF) run their fold-in on a dedicated HIP stream so the interval's
device work overlaps the update-consumer thread's host work.
"""

from __future__ import annotations

import logging
import threading
import time
from typing import Optional

from ..api import Dataset, MessageBlock, SpeedModelManager
from ..serving.layer import UpdateIterator
from ..transport import log as tlog
from ..transport.producer import LogTopicProducer
from ..utils import config as cfg
from ..utils import lang
from .common import AbstractLayer, IntervalTimer, drain_dataset

__all__ = ["SpeedLayer", "measure_intervals", "publish_blocks"]

log = logging.getLogger(__name__)



class _BlockWriter:
    """One persistent writer thread for :func:`publish_blocks` (per process): handing a block
    to a waiting thread costs ~0.03 ms where starting and joining a thread per interval cost
    0.1-0.27 ms of the interval's latency.  Jobs run in submission order."""

    _inst: "Optional[_BlockWriter]" = None
    _inst_pid = 0
    _lock = threading.Lock()

    @classmethod
    def get(cls) -> "_BlockWriter":
        import os
        with cls._lock:
            if cls._inst is None or cls._inst_pid != os.getpid():   # a forked child
                cls._inst = cls()
                cls._inst_pid = os.getpid()
            return cls._inst

    def __init__(self):
        import queue
        self.q: "queue.Queue" = queue.Queue()
        threading.Thread(target=self._run, name="oryx-up-writer", daemon=True).start()

    def _run(self):
        while True:
            producer, b, st = self.q.get()
            if b is None:
                st["done"].set()
                continue
            try:
                if st["errors"]:
                    continue
                t0 = time.perf_counter()
                try:
                    if isinstance(b, MessageBlock):
                        producer.send_block("UP", b)
                    else:
                        producer.send_many(("UP", m) for m in b)
                except BaseException as e:     # surfaced on the caller's thread
                    st["errors"].append(e)
                st["write_s"] += time.perf_counter() - t0
            finally:
                st["slots"].release()


def publish_blocks(producer, blocks, stats: Optional[dict] = None) -> int:
    """Append a stream of UP blocks (``MessageBlock`` or lists of messages) in order, each on
    the writer thread while the next is produced (the native append and the native assembly
    both run without the GIL, so the log write overlaps the rest of the interval's output); at
    most two blocks wait.  Returns the number of messages sent; ``stats`` (a dict) receives
    ``write_ms`` (the appends) and ``tail_ms`` (waiting for them after the last block was
    produced)."""
    w = _BlockWriter.get()
    st = {"errors": [], "write_s": 0.0, "done": threading.Event(),
          "slots": threading.BoundedSemaphore(2)}
    sent = 0
    try:
        for b in blocks:
            if st["errors"]:
                break
            if len(b):
                st["slots"].acquire()
                w.q.put((producer, b, st))
                sent += len(b)
    finally:
        t_end = time.perf_counter()
        w.q.put((producer, None, st))
        st["done"].wait()
    if stats is not None:
        stats["write_ms"] = st["write_s"] * 1e3
        stats["tail_ms"] = (time.perf_counter() - t_end) * 1e3
    if st["errors"]:
        raise st["errors"][0]
    return sent


def measure_intervals(manager, dataset: Dataset, producer, reps: int = 12, warmup: int = 2,
                      gap_s: float = 0.05) -> dict:
    """The speed layer's per-interval latency for one micro-batch, as :meth:`SpeedLayer.
    run_interval` spends it: the manager's update build plus the append of every update to
    ``producer`` (the update log), timed end to end over ``reps`` repetitions after
    ``warmup`` (``gap_s`` idle between, as between intervals).  Returns median / p90 ms, the
    per-rep times and the messages per interval (the benchmarks' speed-layer records)."""
    import numpy as np
    times = []
    phases = []
    sent = 0
    dev = getattr(manager, "device", None)
    for rep in range(warmup + reps):
        time.sleep(gap_s)
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        except ImportError:     # pragma: no cover
            pass
        t0 = time.perf_counter()
        blocks = getattr(manager, "build_update_blocks", None)
        if blocks is not None:
            sent = publish_blocks(producer, blocks(dataset))
            t1 = time.perf_counter()
        else:
            updates = manager.build_updates(dataset)
            t1 = time.perf_counter()
            if isinstance(updates, MessageBlock):
                producer.send_block("UP", updates)
            elif updates:
                producer.send_many(("UP", u) for u in updates)
            sent = len(updates) if updates is not None else 0
        producer.flush()
        if rep >= warmup:
            times.append((time.perf_counter() - t0) * 1e3)
            ph = dict(getattr(manager, "last_phase_ms", None) or {})
            ph["append"] = (time.perf_counter() - t1) * 1e3
            phases.append(ph)
    del dev
    keys = sorted({k for p in phases for k in p})
    return {"median_ms": float(np.median(times)), "p90_ms": float(np.percentile(times, 90)),
            "reps": reps, "times_ms": times, "messages": int(sent),
            "phase_ms": {k: float(np.median([p.get(k, 0.0) for p in phases])) for k in keys}}


class SpeedLayer(AbstractLayer):
    layer_name = "SpeedLayer"
    config_group = "speed"

    def __init__(self, config, manager: Optional[SpeedModelManager] = None):
        super().__init__(config)
        self.manager_class = cfg.get_optional_string(config, "oryx.speed.model-manager-class")
        self._manager = manager
        self._timer: Optional[IntervalTimer] = None
        self._consumer_thread: Optional[threading.Thread] = None
        self._updates: Optional[UpdateIterator] = None
        self._update_consumer: Optional[tlog.TopicConsumer] = None
        self._producer: Optional[LogTopicProducer] = None
        self.intervals_run = 0
        self.updates_sent = 0

    def load_manager_instance(self) -> SpeedModelManager:
        if self._manager is not None:
            return self._manager
        if not self.manager_class:
            raise ValueError("oryx.speed.model-manager-class is not set")
        return lang.load_instance_of(self.manager_class, None, self.config)

    @property
    def manager(self) -> Optional[SpeedModelManager]:
        return self._manager

    def start(self, start_timer: bool = True) -> "SpeedLayer":
        self._manager = self.load_manager_instance()
        self._context = self.layer_context()
        tlog.maybe_create_topic(self.update_root, self.update_topic, 1, self.max_message)
        topic = tlog.Topic(self.update_root, self.update_topic)
        self._update_consumer = tlog.TopicConsumer(topic, start="earliest")
        self._updates = UpdateIterator(self._update_consumer)

        def consume():
            try:
                self._manager.consume(self._updates, self._context)
            except Exception:
                log.exception("Error while consuming updates")
                self.close()

        self._consumer_thread = threading.Thread(target=consume,
                                                 name="OryxSpeedLayerUpdateConsumerThread",
                                                 daemon=True)
        self._consumer_thread.start()
        self.build_input_consumer()
        self._producer = LogTopicProducer(self.update_broker, self.update_topic, self.config,
                                          async_=True, max_message=self.max_message)
        if start_timer:
            self._timer = IntervalTimer(self.generation_interval_sec, self.run_interval,
                                        "OryxSpeedLayer")
            self._timer.start()
        lang.close_at_shutdown(self)
        return self

    def run_interval(self, timestamp: Optional[int] = None) -> int:
        records = drain_dataset(self._input_consumer)
        sent = 0
        if len(records):
            blocks = getattr(self._manager, "build_update_blocks", None)
            if blocks is not None:
                sent = publish_blocks(self._producer, blocks(records))
            else:
                updates = self._manager.build_updates(records)
                if isinstance(updates, MessageBlock):
                    self._producer.send_block("UP", updates)
                    sent = len(updates)
                elif updates:
                    self._producer.send_many(("UP", u) for u in updates)
                    sent = len(updates) if hasattr(updates, "__len__") else 0
            self._producer.flush()
        self.commit_input_offsets()
        self.intervals_run += 1
        self.updates_sent += sent
        return sent

    def await_termination(self, timeout: Optional[float] = None) -> None:
        t0 = time.time()
        while self._timer is not None and self._timer.is_alive():
            if timeout is not None and time.time() - t0 > timeout:
                return
            time.sleep(0.5)

    def close(self) -> None:
        if self._timer is not None:
            self._timer.stop()
            self._timer = None
        if self._updates is not None:
            self._updates.close()
        if self._consumer_thread is not None and \
                self._consumer_thread is not threading.current_thread():
            self._consumer_thread.join(timeout=10)
        if self._update_consumer is not None:
            self._update_consumer.close()
            self._update_consumer = None
        if self._producer is not None:
            self._producer.close()
            self._producer = None
        if self._manager is not None:
            self._manager.close()
        self.close_input()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.close()
        return False
