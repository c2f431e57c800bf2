"""The batch layer: periodic full retraining over all history.

Equivalent of ``BatchLayer`` + ``BatchUpdateFunction`` + ``SaveToHDFSFunction`` +
``DeleteOldDataFn`` + ``UpdateOffsetsFn`` (``[lambda]/batch/BatchLayer.java:58-184``,
``[lambda]/batch/BatchUpdateFunction.java:86-171``, ``SaveToHDFSFunction.java:59-76``,
``[lambda]/DeleteOldDataFn.java:42-76``, ``[lambda]/UpdateOffsetsFn.java:56-67``).  Every
``generation-interval-sec``:

1. drain the input topic since the last interval (the interval's new data);
2. if non-empty: read all past data (``data-dir/*/part-*``), open a *synchronous* producer on
   the update topic and call the update class's ``run_update`` (the update runs before the
   save, so past data never includes the current interval);
3. save the new data as ``data-dir/oryx-<ms>.data/part-00000.txt`` (the messages, one per
   line, when no record has a key -- the common case, read back without per-record
   decoding) or ``part-00000`` (JSON lines ``[key,message]``);
4. commit input offsets (when ``oryx.id`` is set);
5. delete data (and model) dirs older than ``max-age-data-hours`` (``max-age-model-hours``).

Sharded data path (one rank per GPU; update classes with ``sharded_data = True``, i.e. the ALS,
k-means and RDF apps): rank 0 announces only the generation (timestamp, seed and the input
offset range of every partition); each rank reads ITS share of every partition's offset range
straight from the log, reads only its share of the past part files, runs the update on its
share (the apps exchange what they need by key with all-to-alls -- the reference's Spark
shuffles) and writes its own ``part-<rank>`` file, like the reference's per-partition
``SaveToHDFSFunction`` / ``BatchUpdateFunction`` (``[lambda]/batch/SaveToHDFSFunction.java:
59-76``, ``BatchUpdateFunction.java:103-130``).  No record crosses ranks in the layer.
Other update classes get the interval's records from rank 0 (broadcast) as before.
"""

from __future__ import annotations

import json
import logging
import os
import re
import shutil
import threading
import time
from typing import List, Optional, Tuple

import numpy as np

from .. import hostbuf, tracing
from ..api import BatchLayerUpdate, Dataset
from ..transport.producer import LogTopicProducer
from ..utils import config as cfg
from ..parallel import dist
from ..textlines import LineConcat, TextLines, concat_lines
from ..utils import faults, ioutils, lang, rng
from .common import AbstractLayer, IntervalTimer, drain_dataset, read_text_parallel

__all__ = ["BatchLayer", "save_interval_data", "read_past_data", "delete_old_data",
           "read_log_share", "save_interval_part"]

log = logging.getLogger(__name__)

_TS_RE = re.compile(r"-(\d+)\.")


def _write_part(path_no_ext: str, records) -> str:
    """Write one part file; keyless single-line messages as plain text (``.txt``) -- a
    :class:`TextLines` buffer is written as it is."""
    if isinstance(records, Dataset) and records.keyless:
        vals = records.values()
        if isinstance(vals, TextLines):
            path = path_no_ext + ".txt"
            with open(path + ".w", "wb") as f:
                f.write(memoryview(vals.joined()))
            os.replace(path + ".w", path)
            return path
        text = "\n".join(vals)
        if text.count("\n") == len(vals) - 1:
            path = path_no_ext + ".txt"
            with open(path + ".w", "w", encoding="utf-8") as f:
                f.write(text)
                f.write("\n")
            os.replace(path + ".w", path)
            return path
    with open(path_no_ext + ".w", "w", encoding="utf-8") as f:
        for k, m in records:
            f.write(json.dumps([k, m], separators=(",", ":")))
            f.write("\n")
    os.replace(path_no_ext + ".w", path_no_ext)
    return path_no_ext


def _write_text_parts(tmp: str, buf) -> bool:
    """A large keyless text buffer as part-00000.txt, part-00001.txt, ... cut at
    :func:`~oryx_amd.textlines.part_edges`, written concurrently (one write() per file: the
    files scale on the box's filesystem, one big file does not -- 22.5 GB took 2.2 s and was
    the k-means generation's critical path).  False when one file is all there is."""
    from concurrent.futures import ThreadPoolExecutor
    from ..textlines import part_edges
    if not isinstance(buf, np.ndarray):
        buf = np.frombuffer(buf, dtype=np.uint8)
    edges = part_edges(buf)
    if len(edges) <= 2:
        return False

    def write(j):
        path = os.path.join(tmp, "part-%05d.txt" % j)
        with open(path + ".w", "wb") as f:
            f.write(memoryview(buf[edges[j]:edges[j + 1]]))
        os.replace(path + ".w", path)

    with ThreadPoolExecutor(max_workers=len(edges) - 1) as ex:
        list(ex.map(write, range(len(edges) - 1)))
    return True


def save_interval_data(data_dir: str, timestamp: int, records,
                       split: bool = False, publish: bool = True) -> Optional[str]:
    """The interval's records as ``oryx-<ts>.data/part-*``; ``split``: a large keyless text
    interval as several part files (:func:`_write_text_parts`).  ``publish=False`` leaves them
    in ``oryx-<ts>.data.tmp`` (past-data readers skip it) for :func:`_finish_interval_dir` or
    :func:`_discard_interval_dir` to settle once the interval's update has succeeded or
    failed."""
    if not records or not len(records):
        return None
    d = os.path.join(ioutils.to_local_path(data_dir), "oryx-%d.data" % timestamp)
    tmp = d + ".tmp"
    os.makedirs(tmp, exist_ok=True)
    vals = records.values() if split and isinstance(records, Dataset) and records.keyless \
        else None
    if not (isinstance(vals, TextLines) and _write_text_parts(tmp, vals.joined())):
        _write_part(os.path.join(tmp, "part-00000"), records)
    if not publish:
        return tmp
    os.replace(tmp, d)
    return d


def save_interval_part(data_dir: str, timestamp: int, records, rank: int) -> str:
    """This rank's share of an interval: ``oryx-<ts>.data.tmp/part-<rank>`` (the directory is
    renamed into place by rank 0 once every rank has written)."""
    d = os.path.join(ioutils.to_local_path(data_dir), "oryx-%d.data.tmp" % timestamp)
    os.makedirs(d, exist_ok=True)
    _write_part(os.path.join(d, "part-%05d" % rank), records)
    return d


def _finish_interval_dir(data_dir: str, timestamp: int) -> None:
    root = ioutils.to_local_path(data_dir)
    tmp = os.path.join(root, "oryx-%d.data.tmp" % timestamp)
    if os.path.isdir(tmp):
        os.replace(tmp, os.path.join(root, "oryx-%d.data" % timestamp))


def _discard_interval_dir(data_dir: str, timestamp: int) -> None:
    """Drop an interval's unpublished data (its update failed: the offsets stay uncommitted,
    so the next interval re-reads these records and saves them then -- saving them now too
    would put them in the past data twice)."""
    tmp = os.path.join(ioutils.to_local_path(data_dir), "oryx-%d.data.tmp" % timestamp)
    if os.path.isdir(tmp):
        shutil.rmtree(tmp, ignore_errors=True)


def read_past_data(data_dir: str, rank: int = 0, world: int = 1) -> Dataset:
    """All past records, or with ``world > 1`` this rank's share: part file j of the sorted
    listing belongs to rank ``j % world``."""
    from concurrent.futures import ThreadPoolExecutor
    pairs: List[Tuple[Optional[str], str]] = []
    texts = []
    paths = [p for p in sorted(ioutils.list_files(data_dir, "*/part-*"))
             if ".tmp" not in os.path.dirname(p) and not p.endswith(".w")]
    mine = [p for j, p in enumerate(paths) if j % world == rank]
    txt = [p for p in mine if p.endswith(".txt")]
    # the .txt files' bytes are the message buffers (no per-line strings), keyed by the
    # file's identity so apps can reuse their parse of it (models/als/history.py,
    # models/features.py); several files are read at once, 16 preads in flight in all
    per = max(1, 16 // max(1, len(txt)))

    def load(path):
        st = os.stat(path)
        return TextLines(hostbuf.read_text_file(path, per)).with_key(
            ("part", os.path.abspath(path), st.st_size, st.st_mtime_ns))

    loaded = {}
    if txt:
        with ThreadPoolExecutor(max_workers=min(16, len(txt))) as ex:
            loaded = dict(zip(txt, ex.map(load, txt)))
    for path in mine:
        if path in loaded:
            texts.append(loaded[path])
            continue
        with open(path, "r", encoding="utf-8") as f:
            for line in f:
                if line.strip():
                    k, m = json.loads(line)
                    pairs.append((k, m))
    # several part files stay a lazy concatenation: the feature parsers take them part by part
    # (cached / adopted parses), others get the joined buffer when they ask for its bytes
    values = LineConcat(texts) if len(texts) > 1 and not pairs else concat_lines(texts)
    if not pairs:
        return Dataset.from_values(values)
    return Dataset([(None, v) for v in values] + pairs)


def read_log_share(root: str, topic_name: str, starts: List[int], ends: List[int], rank: int,
                   world: int) -> Dataset:
    """Records of this rank's contiguous share of every partition's [start, end) range."""
    from ..transport import log as tlog
    out: List[Tuple[Optional[str], str]] = []
    texts = []
    topic = tlog.Topic(root, topic_name)
    readers = []
    try:
        for p, (lo, hi) in enumerate(zip(starts, ends)):
            n = hi - lo
            a, b = lo + n * rank // world, lo + n * (rank + 1) // world
            if b > a:
                readers.append((topic.reader(p, a), b))
        for (r, b), lines in zip(readers, read_text_parallel(readers)):
            if lines is not None:
                texts.append(lines)
                continue
            while r.position < b:
                recs = r.poll(min(65536, b - r.position), 100)
                if not recs:
                    break
                for off, _, k, v in recs:
                    if off >= b:
                        break
                    out.append((k, v))
    finally:
        for r, _ in readers:
            r.close()
        topic.close()
    values = concat_lines(texts)
    if not out:
        return Dataset.from_values(values)
    return Dataset([(None, v) for v in values] + out)


def delete_old_data(directory: str, max_age_hours: int, pattern: re.Pattern = _TS_RE,
                    now_ms: Optional[int] = None) -> List[str]:
    """Delete subdirectories whose embedded timestamp is older than ``max_age_hours``."""
    if max_age_hours < 0:
        return []
    now = int(time.time() * 1000) if now_ms is None else now_ms
    cutoff = now - max_age_hours * 3600 * 1000
    deleted = []
    root = ioutils.to_local_path(directory)
    if not os.path.isdir(root):
        return deleted
    for name in os.listdir(root):
        m = pattern.search(name)
        if not m:
            continue
        if int(m.group(1)) < cutoff:
            ioutils.delete_recursively(os.path.join(root, name))
            deleted.append(name)
    return deleted


class _Background:
    """``fn(*args)`` on a thread; ``wait`` joins it, ``raise_error`` re-raises its exception."""

    def __init__(self, fn, *args):
        self.error: Optional[BaseException] = None
        self.seconds = 0.0

        def run():
            t0 = time.perf_counter()
            try:
                fn(*args)
            except BaseException as e:   # noqa: BLE001 -- re-raised by join
                self.error = e
            self.seconds = time.perf_counter() - t0
        self._t = threading.Thread(target=run, name="oryx-save-data", daemon=True)
        self._t.start()

    def wait(self) -> None:
        self._t.join()

    def raise_error(self) -> None:
        if self.error is not None:
            raise self.error


class BatchLayer(AbstractLayer):
    layer_name = "BatchLayer"
    config_group = "batch"

    def __init__(self, config, update: Optional[BatchLayerUpdate] = None):
        super().__init__(config)
        self.data_dir = config.get_string("oryx.batch.storage.data-dir")
        self.model_dir = config.get_string("oryx.batch.storage.model-dir")
        self.max_data_age_hours = config.get_int("oryx.batch.storage.max-age-data-hours")
        self.max_model_age_hours = config.get_int("oryx.batch.storage.max-age-model-hours")
        self.update_class = cfg.get_optional_string(config, "oryx.batch.update-class")
        # per-interval JSON lines (new; the reference only logs)
        self.timings_file = cfg.get_optional_string(config, "oryx.metrics.timings-file")
        self._update = update
        self._timer: Optional[IntervalTimer] = None
        self._context = None
        self._released = False
        self.intervals_run = 0
        self.last_phases = {}
        self.warm_up_s: Optional[float] = None

    def load_update_instance(self) -> BatchLayerUpdate:
        if self._update is not None:
            return self._update
        if not self.update_class:
            raise ValueError("oryx.batch.update-class is not set")
        return lang.load_instance_of(self.update_class, None, self.config)

    def warm_up(self) -> Optional[float]:
        """The update's start-up warm-up (``BatchLayerUpdate.warm_up``: one tiny build on
        this process's device, so the first generation does not pay first-call costs --
        kernel code objects loaded on first launch, the caching allocator's first blocks);
        local to this rank, no collectives.  Seconds taken, or None."""
        fn = getattr(self._update, "warm_up", None)
        if fn is None or self.warm_up_s is not None:
            return self.warm_up_s
        t0 = time.perf_counter()
        try:
            fn(self._context)
        except Exception as e:   # noqa: BLE001 -- a failed warm-up only costs the first build
            log.warning("Batch update warm-up failed: %s", e)
        self.warm_up_s = time.perf_counter() - t0
        log.info("Batch update warmed up in %.3fs", self.warm_up_s)
        return self.warm_up_s

    def start(self) -> "BatchLayer":
        ioutils.mkdirs(self.data_dir)
        ioutils.mkdirs(self.model_dir)
        self._update = self.load_update_instance()
        self._context = self.layer_context()
        self.warm_up()
        self.build_input_consumer()
        self._timer = IntervalTimer(self.generation_interval_sec, self.run_interval,
                                    "OryxBatchLayer")
        self._timer.start()
        lang.close_at_shutdown(self)
        log.info("Batch layer started (interval %ds)", self.generation_interval_sec)
        return self

    def _sharded(self) -> bool:
        dctx = self._context.dist if self._context is not None else None
        return bool(dctx is not None and dctx.is_distributed and
                    getattr(self._update, "sharded_data", False))

    def run_interval(self, timestamp: Optional[int] = None) -> None:
        """One generation (also callable directly, e.g. from the CLI or tests)."""
        if self._input_consumer is None:
            self._update = self.load_update_instance()
            self._context = self.layer_context()
            self.build_input_consumer()
        ts = int(time.time() * 1000) if timestamp is None else timestamp
        t_start = time.perf_counter()
        if self._sharded():
            self._run_sharded_main(ts, t_start)
            return
        # where this interval starts: a failed update rewinds here, so the next interval
        # re-reads (and only then saves) the same records
        starts = [(r, r.position) for r in self._input_consumer.readers]
        records = drain_dataset(self._input_consumer)
        n_records = len(records)
        ph = self.last_phases = {"drain": time.perf_counter() - t_start}
        faults.point("batch.interval", timestamp=ts, records=len(records))
        dctx = self._context.dist if self._context is not None else None
        seed = rng.next_seed()
        if dctx is not None and dctx.is_distributed:
            # announce the generation to the follower ranks (they join the collectives)
            dist.broadcast_object({"ts": ts, "records": records, "seed": seed}, dctx,
                                  control=True)
        if len(records):
            log.info("Beginning update at %d with %d new records", ts, len(records))
            new_data = records
            tp = time.perf_counter()
            past = read_past_data(self.data_dir)
            ph["read_past"] = time.perf_counter() - tp
            # the interval's data is written while the update runs (disk writes beside GPU /
            # parse work) into oryx-<ts>.data.tmp, and published -- renamed into the past
            # data -- only after the update has succeeded, as the reference saves only after
            # a successful update (BatchLayer.java:103-124); apps whose parsers adopt part
            # files by byte range take a large interval as several files, written
            # concurrently
            saver = _Background(save_interval_data, self.data_dir, ts, records,
                                bool(getattr(self._update, "split_interval_files", False)),
                                False)
            ok = False
            producer = None
            if self.update_topic and self.update_broker:
                producer = LogTopicProducer(self.update_broker, self.update_topic, self.config,
                                            async_=False, max_message=self.max_message)
            tp = time.perf_counter()
            try:
                with rng.shared_seed_scope(seed):
                    self._update.run_update(self._context, ts, new_data,
                                            past if len(past) else None, self.model_dir,
                                            producer)
                ok = True
            finally:
                if producer is not None:
                    producer.close()
                ph["update"] = time.perf_counter() - tp
                tp = time.perf_counter()
                saver.wait()
                if ok and saver.error is None:
                    _finish_interval_dir(self.data_dir, ts)
                else:
                    _discard_interval_dir(self.data_dir, ts)
                    for r, pos in starts:
                        r.seek(pos)
                # (the part of the save not hidden behind the update)
                ph["save_data"] = time.perf_counter() - tp
                ph["save_data_total"] = saver.seconds
            saver.raise_error()
            tp = time.perf_counter()
            del new_data, past
            records = None
            ph["release"] = time.perf_counter() - tp
        self.commit_input_offsets()
        rec = {"event": "batch_interval", "layer_id": self.id, "timestamp": ts,
               "records": n_records, "seconds": time.perf_counter() - t_start}
        tracing.record(rec)
        if self.timings_file:
            with open(self.timings_file, "a") as f:
                f.write(json.dumps(rec) + "\n")
        if self.max_data_age_hours >= 0:
            delete_old_data(self.data_dir, self.max_data_age_hours)
        if self.max_model_age_hours >= 0:
            delete_old_data(self.model_dir, self.max_model_age_hours,
                            pattern=re.compile(r"^(\d+)$"))
        self.intervals_run += 1

    # ------------------------------------------------------------------ sharded generations
    def _run_sharded_main(self, ts: int, t_start: float) -> None:
        cons = self._input_consumer
        ends = cons.topic.end_offsets()
        starts = [r.position for r in sorted(cons.readers, key=lambda r: r.partition)]
        seed = rng.next_seed()
        msg = {"ts": ts, "seed": seed, "starts": starts, "ends": ends, "sharded": True}
        dist.broadcast_object(msg, self._context.dist, control=True)
        n = self._run_sharded(msg)
        for r in cons.readers:
            r.seek(ends[r.partition])
        self.commit_input_offsets()
        rec = {"event": "batch_interval", "layer_id": self.id, "timestamp": ts,
               "records": n, "seconds": time.perf_counter() - t_start, "sharded": True}
        tracing.record(rec)
        if self.timings_file:
            with open(self.timings_file, "a") as f:
                f.write(json.dumps(rec) + "\n")
        if self.max_data_age_hours >= 0:
            delete_old_data(self.data_dir, self.max_data_age_hours)
        if self.max_model_age_hours >= 0:
            delete_old_data(self.model_dir, self.max_model_age_hours,
                            pattern=re.compile(r"^(\d+)$"))
        self.intervals_run += 1

    def _run_sharded(self, msg) -> int:
        """Every rank: read its share, update, save its part; returns the interval's total
        record count (all ranks)."""
        dctx = self._context.dist
        total = sum(e - s for s, e in zip(msg["starts"], msg["ends"]))
        if total <= 0:
            return 0
        ts = msg["ts"]
        t0 = time.perf_counter()
        records = read_log_share(self.input_root, self.input_topic, msg["starts"], msg["ends"],
                                 dctx.rank, dctx.world_size)
        ph = self.last_phases = {"drain": time.perf_counter() - t0}
        faults.point("batch.interval", timestamp=ts, records=len(records))
        log.info("Rank %d: update at %d with %d of %d new records", dctx.rank, ts,
                 len(records), total)
        tp = time.perf_counter()
        past = read_past_data(self.data_dir, dctx.rank, dctx.world_size)
        ph["read_past"] = time.perf_counter() - tp
        producer = None
        if self.update_topic and self.update_broker:
            producer = LogTopicProducer(self.update_broker, self.update_topic, self.config,
                                        async_=False, max_message=self.max_message)
        tp = time.perf_counter()
        try:
            with rng.shared_seed_scope(msg["seed"]):
                self._update.run_update(self._context, ts, records,
                                        past if len(past) else None, self.model_dir, producer)
        finally:
            if producer is not None:
                producer.close()
        ph["update"] = time.perf_counter() - tp
        tp = time.perf_counter()
        save_interval_part(self.data_dir, ts, records, dctx.rank)
        dist.barrier(dctx)
        if dctx.is_main:
            _finish_interval_dir(self.data_dir, ts)
        dist.barrier(dctx)
        ph["save_data"] = time.perf_counter() - tp
        return total

    def run_follower(self) -> int:
        """Non-zero ranks of a multi-GPU batch layer: wait for rank 0's announcements and run
        the same update (reading past data from the shared data dir) so every collective in
        the trainers has all participants.  Returns the number of generations joined."""
        self._update = self.load_update_instance()
        self._context = self.layer_context()
        self.warm_up()
        dctx = self._context.dist
        joined = 0
        while True:
            msg = dist.broadcast_object(None, dctx, control=True)
            if msg is None:
                return joined
            if msg.get("sharded"):
                if self._run_sharded(msg):
                    joined += 1
                continue
            if not len(msg["records"]):
                continue
            past = read_past_data(self.data_dir)
            recs = msg["records"]
            with rng.shared_seed_scope(msg["seed"]):
                self._update.run_update(self._context, msg["ts"],
                                        recs if isinstance(recs, Dataset) else Dataset(recs),
                                        past if len(past) else None, self.model_dir, None)
            joined += 1

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
        dctx = self._context.dist if getattr(self, "_context", None) is not None else None
        if dctx is not None and dctx.is_distributed and dctx.is_main and not self._released:
            self._released = True
            dist.broadcast_object(None, dctx, control=True)     # release the followers
        self.close_input()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.close()
        return False
