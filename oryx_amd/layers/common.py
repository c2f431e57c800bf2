"""Shared batch/speed layer plumbing (the reference's ``AbstractSparkLayer``).

``[lambda]/AbstractSparkLayer.java:77-252``: instance id (random when ``oryx.id`` is unset),
consumer group ``OryxGroup-<Layer>-<id>``, the input-topic consumer that resumes from the
committed group offsets when an id is configured (missing partitions fall back to the
latest offset; without an id reading starts at the latest offset -- at-most-once), and the
generation interval.  Spark Streaming's micro-batch scheduler becomes :class:`IntervalTimer`.
"""

from __future__ import annotations

import logging
import os
import threading
import time
import uuid
from dataclasses import dataclass
from typing import Any, List, Optional, Tuple

from ..api import Dataset
from ..parallel import dist, watchdog
from ..transport import log as tlog
from ..transport.producer import topic_root
from ..utils import config as cfg
from ..utils import lang

__all__ = ["AbstractLayer", "LayerContext", "IntervalTimer", "drain", "drain_dataset"]

log = logging.getLogger(__name__)


@dataclass
class LayerContext:
    """What a layer hands to app code (in place of a JavaSparkContext)."""

    config: Any
    dist: dist.DistContext
    layer: str = ""

    @property
    def device(self):
        return self.dist.device


def read_text_parallel(jobs):
    """``PartitionReader.read_text_lines(end)`` of every (reader, end) job, partitions read
    concurrently (the native read runs without the GIL); one result per job, in order."""
    if len(jobs) <= 1:
        return [r.read_text_lines(end)[0] for r, end in jobs]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
        return list(ex.map(lambda job: job[0].read_text_lines(job[1])[0], jobs))


def read_text_segments(jobs, threads: int = 16):
    """As :func:`read_text_parallel`, with every partition's range cut at its segment files'
    first offsets (64 MB segments: a 2.8 GB partition is ~44 pieces) and the pieces read by
    ``threads`` workers, each with a reader of its own: one list of pieces (in order) per job,
    or None for a job with a keyed / multi-line record (its reader is left where it was, for
    the per-record path); a job read in full has its reader moved to its end."""
    from concurrent.futures import ThreadPoolExecutor
    tasks = []
    for k, (r, end) in enumerate(jobs):
        start = r.position
        if start >= end:
            continue
        cuts = [b for b in r.topic.segment_bases(r.partition) if start < b < end]
        edges = [start] + cuts + [end]
        tasks += [(k, lo, hi) for lo, hi in zip(edges[:-1], edges[1:])]

    def run(task):
        k, lo, hi = task
        rr = jobs[k][0].topic.reader(jobs[k][0].partition, lo)
        try:
            return rr.read_text_lines(hi)[0]
        finally:
            rr.close()

    with ThreadPoolExecutor(max_workers=max(1, min(len(tasks), threads))) as ex:
        got = list(ex.map(run, tasks))
    out = [[] for _ in jobs]
    for (k, _, _), lines in zip(tasks, got):
        if out[k] is not None:
            out[k] = None if lines is None else out[k] + [lines]
    for k, (r, end) in enumerate(jobs):
        if out[k] is not None and r.position < end:
            r.seek(end)
    return out


def _read_text_one_buffer(jobs):
    """Every (reader, end) job's text read concurrently into ONE buffer (each partition into
    its slice, sized by the reader's bound), gaps closed afterwards: the drain's text without
    per-partition buffers and a concatenating copy.  None when a partition needs the
    per-record path (keys, multi-line values) or grew past its bound.

    Opt-in (``ORYX_DRAIN_ONE_BUFFER=1``): on the MI355X box the 22.5 GB k-means drain took
    1.88 s this way against 1.19 s with per-partition buffers and the threaded concatenation
    (2.91 s with the buffer prefaulted first, ``ORYX_DRAIN_PREFAULT=1``;
    profiles/r5_drain_ab_v1.txt)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    from .. import hostbuf
    from ..textlines import TextLines
    bounds = [r.text_bound(end) for r, end in jobs]
    total = sum(bounds)
    if total == 0:
        return TextLines(b"", 0)
    buf = hostbuf.empty(total)
    if os.environ.get("ORYX_DRAIN_PREFAULT", "0") == "1":
        hostbuf.prefault(buf)
    offs = np.concatenate([[0], np.cumsum(bounds)]).astype(np.int64)
    base = buf.ctypes.data
    with ThreadPoolExecutor(max_workers=min(len(jobs), 16)) as ex:
        got = list(ex.map(lambda k: jobs[k][0].read_text_into(
            jobs[k][1], base + int(offs[k]), bounds[k]), range(len(jobs))))
    if any(g is None for g in got):
        # (readers that did read keep their new position: rewind them for the fallback)
        return None
    at = 0
    n = 0
    for k, (used, recs) in enumerate(got):
        if used and at != offs[k]:
            ctypes.memmove(base + at, base + int(offs[k]), used)
        at += used
        n += recs
    return TextLines(buf[:at], n)


def drain_dataset(consumer: tlog.TopicConsumer,
                  end_offsets: Optional[List[int]] = None) -> Dataset:
    """Everything currently available as a :class:`Dataset`: partitions are read in bulk
    natively (messages only, into one buffer) unless a record has a key or a multi-line
    value."""
    from ..textlines import concat_lines
    topic = consumer.topic
    ends = end_offsets or topic.end_offsets()
    texts = []
    pairs: List[Tuple[Optional[str], str]] = []
    readers = list(consumer.readers)
    jobs = [(r, ends[r.partition]) for r in readers]
    starts = [r.position for r in readers]
    one = _read_text_one_buffer(jobs) \
        if len(jobs) > 1 and os.environ.get("ORYX_DRAIN_ONE_BUFFER", "0") == "1" else None
    if one is not None:
        return Dataset.from_values(one)
    for r, p in zip(readers, starts):
        if r.position != p:
            r.seek(p)
    if os.environ.get("ORYX_DRAIN_SEGMENTS", "1") != "0":
        bulk = read_text_segments(jobs)
    else:
        bulk = [[t] if t is not None else None for t in read_text_parallel(jobs)]
    for r, pieces in zip(readers, bulk):
        target = ends[r.partition]
        if pieces is not None:
            texts.extend(pieces)
            continue
        while r.position < target:
            recs = r.poll(min(65536, target - r.position), 50)
            if not recs:
                break
            for off, _, k, v in recs:
                if off >= target:
                    r.seek(off)
                    break
                pairs.append((k, v))
    # keyless single-line messages stay one buffer (TextLines): no Python string per record
    values = concat_lines(texts)
    if not pairs:
        return Dataset.from_values(values)
    return Dataset([(None, v) for v in values] + pairs)


def drain(consumer: tlog.TopicConsumer, max_records: int = 1 << 24,
          end_offsets: Optional[List[int]] = None) -> List[Tuple[Optional[str], str]]:
    """Everything currently available (up to the end offsets at call time)."""
    topic = consumer.topic
    ends = end_offsets or topic.end_offsets()
    out: List[Tuple[Optional[str], str]] = []
    for r in consumer.readers:
        target = ends[r.partition]
        while r.position < target and len(out) < max_records:
            recs = r.poll(min(65536, target - r.position), 50)
            if not recs:
                break
            for off, _, k, v in recs:
                if off >= target:
                    r.seek(off)
                    break
                out.append((k, v))
    return out


class IntervalTimer:
    """Calls ``fn(timestamp_ms)`` every ``interval_s`` on a daemon thread until stopped."""

    def __init__(self, interval_s: float, fn, name: str):
        self.interval_s = float(interval_s)
        self.fn = fn
        self.name = name
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.error: Optional[BaseException] = None

    def start(self) -> None:
        self._thread = threading.Thread(target=self._run, name=self.name, daemon=True)
        self._thread.start()

    def _run(self) -> None:
        next_t = time.time() + self.interval_s
        while not self._stop.is_set():
            if self._stop.wait(max(0.0, next_t - time.time())):
                break
            ts = int(time.time() * 1000)
            try:
                self.fn(ts)
            except BaseException as e:
                log.exception("Error in %s interval", self.name)
                self.error = e
            next_t += self.interval_s
            if next_t < time.time():
                next_t = time.time() + self.interval_s

    def stop(self, timeout: float = 60.0) -> None:
        self._stop.set()
        if self._thread is not None and self._thread is not threading.current_thread():
            self._thread.join(timeout)

    def is_alive(self) -> bool:
        return self._thread is not None and self._thread.is_alive()


class AbstractLayer:
    layer_name = "Layer"
    config_group = "batch"

    def __init__(self, config):
        self.config = config
        log.info("Configuration:\n%s", cfg.pretty_print(config))
        oid = cfg.get_optional_string(config, "oryx.id")
        self.id = oid if oid else self.generate_random_id()
        self.has_id = oid is not None
        self.input_topic = config.get_string("oryx.input-topic.message.topic")
        self.input_broker = config.get_string("oryx.input-topic.broker")
        self.update_topic = cfg.get_optional_string(config, "oryx.update-topic.message.topic")
        self.update_broker = cfg.get_optional_string(config, "oryx.update-topic.broker")
        self.max_message = config.get_int("oryx.update-topic.message.max-size")
        self.input_partitions = config.get_int("oryx.input-topic.partitions")
        self.generation_interval_sec = config.get_int(
            "oryx.%s.streaming.generation-interval-sec" % self.config_group)
        if self.generation_interval_sec <= 0:
            raise ValueError("generation-interval-sec must be > 0")
        self.group_id = "OryxGroup-%s-%s" % (self.layer_name, self.id)
        self.input_root = topic_root(self.input_broker, config)
        self.update_root = topic_root(self.update_broker, config) if self.update_broker else None
        self._input_consumer: Optional[tlog.TopicConsumer] = None
        self._input_topic: Optional[tlog.Topic] = None
        wd = cfg.get_optional_int(config, "oryx.gpu.collective-timeout-sec") or 0
        if wd > 0:
            watchdog.configure(wd)

    @staticmethod
    def generate_random_id() -> str:
        return uuid.uuid4().hex[:16]

    def layer_context(self) -> LayerContext:
        dev = cfg.get_optional_string(self.config, "oryx.gpu.device") or "auto"
        return LayerContext(self.config, dist.init_from_env(device=dev), self.layer_name)

    def build_input_consumer(self) -> tlog.TopicConsumer:
        tlog.maybe_create_topic(self.input_root, self.input_topic, self.input_partitions)
        topic = tlog.Topic(self.input_root, self.input_topic)
        self._input_topic = topic
        start = "latest"
        if self.has_id:
            offsets = tlog.get_offsets(self.input_root, self.input_topic, self.group_id,
                                       topic.partitions)
            latest = topic.end_offsets()
            start = {p: offsets.get(p, latest[p]) for p in range(topic.partitions)}
            log.info("Resuming %s from offsets %s", self.group_id, start)
        self._input_consumer = tlog.TopicConsumer(topic, start=start, group=self.group_id)
        return self._input_consumer

    def commit_input_offsets(self) -> None:
        """``UpdateOffsetsFn``: persist the consumed offsets when the layer has an id."""
        if self.has_id and self._input_consumer is not None:
            self._input_consumer.commit()

    def close_input(self) -> None:
        if self._input_consumer is not None:
            self._input_consumer.close()
            self._input_consumer = None
        if self._input_topic is not None:
            self._input_topic.close()
            self._input_topic = None
