"""Python bindings for the native append-only log (``csrc/runtime/oryx_log.cpp``).

Provides Kafka-like primitives used by every layer:

* :class:`Topic` -- open/create a topic (partitions, max message size), append single or
  batched keyed records, begin/end offsets, retention;
* :class:`PartitionReader` / :class:`TopicConsumer` -- tail one or all partitions from an
  offset (``earliest`` / ``latest`` / committed group offset);
* :func:`get_offsets` / :func:`set_offsets` -- consumer-group offset store
  (the ZooKeeper role of ``[kafka]/KafkaUtils.java:123-161``);
* :func:`maybe_create_topic`, :func:`topic_exists`, :func:`delete_topic`
  (``[kafka]/KafkaUtils.java:57-115``).

Brokers: the reference's ``host:port`` broker strings are accepted; records go to the log
root directory ``oryx.transport.log-dir`` unless a broker is written ``log:/some/dir``.
"""

from __future__ import annotations

import ctypes
import os
import shutil
import struct
import threading
import time
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .. import hostbuf, native
from ..utils import faults

__all__ = ["Topic", "PartitionReader", "TopicConsumer", "Record", "get_offsets", "set_offsets",
           "maybe_create_topic", "topic_exists", "delete_topic", "log_root_for",
           "MessageTooLargeError", "DEFAULT_LOG_ROOT"]

DEFAULT_LOG_ROOT = os.environ.get("ORYX_LOG_DIR", "/tmp/Oryx/log")


class MessageTooLargeError(ValueError):
    pass


def _lib():
    return native.runtime()


def log_root_for(broker: Optional[str], config=None) -> str:
    """Resolve a broker string to a log directory."""
    if broker and broker.startswith("log:"):
        return broker[4:]
    if config is not None and config.has_path("oryx.transport.log-dir"):
        from ..utils.ioutils import to_local_path
        return to_local_path(config.get_string("oryx.transport.log-dir"))
    return DEFAULT_LOG_ROOT


def _b(s: Optional[str]) -> Optional[bytes]:
    if s is None:
        return None
    return s.encode("utf-8") if isinstance(s, str) else bytes(s)


def topic_exists(root: str, topic: str) -> bool:
    return bool(_lib().oryx_log_exists(_b(root), _b(topic)))


def maybe_create_topic(root: str, topic: str, partitions: int = 1,
                       max_message: int = 16777216, segment_bytes: int = 64 << 20) -> None:
    if not topic_exists(root, topic):
        Topic(root, topic, create_partitions=partitions, max_message=max_message,
              segment_bytes=segment_bytes).close()


def delete_topic(root: str, topic: str) -> None:
    path = os.path.join(root, topic)
    if os.path.isdir(path):
        shutil.rmtree(path, ignore_errors=True)


class Record(Tuple):
    pass


_HDR = struct.Struct("<qqii")


class Topic:
    """A handle on one topic of the log."""

    def __init__(self, root: str, name: str, create_partitions: int = 0,
                 max_message: int = 16777216, segment_bytes: int = 64 << 20):
        self.root = root
        self.name = name
        lib = _lib()
        self._h = lib.oryx_log_open(_b(root), _b(name), int(create_partitions),
                                    int(max_message), int(segment_bytes))
        if not self._h:
            raise FileNotFoundError(lib.oryx_log_last_error().decode())
        self.partitions = lib.oryx_log_num_partitions(self._h)
        self.max_message = lib.oryx_log_max_message(self._h)
        self._lock = threading.Lock()

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        with self._lock:
            if self._h:
                _lib().oryx_log_close(self._h)
                self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def partition_for(self, key: Optional[str]) -> int:
        kb = _b(key)
        return _lib().oryx_log_partition_for(self._h, kb, -1 if kb is None else len(kb))

    def append(self, key: Optional[str], value: str, partition: int = -1,
               timestamp_ms: int = -1, fsync: bool = False) -> int:
        return self.append_batch([(key, value)], partition, timestamp_ms, fsync)

    def append_batch(self, records: Sequence[Tuple[Optional[str], str]], partition: int = -1,
                     timestamp_ms: int = -1, fsync: bool = False) -> int:
        """Append many (key, value) records with one native call; returns the last offset."""
        if not records:
            return -1
        if faults.armed():
            act = faults.point("log.append", topic=self.name, partition=partition)
            if act == "drop":
                records = records[1:]
                if not records:
                    return -1
            elif act == "corrupt":
                # damage the first record's bytes on disk after its CRC was computed
                return self._append_corrupted(records, partition, timestamp_ms, fsync)
        k0 = records[0][0]
        if all(k == k0 for k, _ in records):
            return self.append_values([v for _, v in records], partition, timestamp_ms, fsync,
                                      key=k0)
        parts = []
        for k, v in records:
            kb = _b(k)
            vb = _b(v)
            parts.append(struct.pack("<iq", -1 if kb is None else len(kb), len(vb)))
            if kb is not None:
                parts.append(kb)
            parts.append(vb)
        buf = b"".join(parts)
        res = _lib().oryx_log_append_batch(self._h, int(partition), buf, len(buf),
                                           len(records), int(timestamp_ms), int(bool(fsync)),
                                           None)
        if res == -2:
            raise MessageTooLargeError(_lib().oryx_log_last_error().decode())
        if res < 0:
            raise IOError(_lib().oryx_log_last_error().decode())
        return res

    def append_values(self, values: Sequence[str], partition: int = -1,
                      timestamp_ms: int = -1, fsync: bool = False,
                      key: Optional[str] = None) -> int:
        """Append records that share one key (default none): one encode of the joined
        values, lengths computed in bulk (character counts when the text is ASCII)."""
        if not values:
            return -1
        text = "".join(values)
        blob = text.encode("utf-8")
        if len(blob) == len(text):
            lens = np.fromiter(map(len, values), dtype=np.int64, count=len(values))
        else:
            lens = np.fromiter((len(v.encode("utf-8")) for v in values), dtype=np.int64,
                               count=len(values))
        kb = _b(key)
        res = _lib().oryx_log_append_values(self._h, int(partition), kb,
                                            -1 if kb is None else len(kb), blob,
                                            lens.ctypes.data_as(ctypes.c_void_p), len(values),
                                            int(timestamp_ms), int(bool(fsync)))
        if res == -2:
            raise MessageTooLargeError(_lib().oryx_log_last_error().decode())
        if res < 0:
            raise IOError(_lib().oryx_log_last_error().decode())
        return res

    def append_block(self, block, key: Optional[str] = None, partition: int = -1,
                     timestamp_ms: int = -1, fsync: bool = False) -> int:
        """Append every message of a :class:`~oryx_amd.api.MessageBlock` with one key, straight
        from its buffer (no per-message Python strings)."""
        n = len(block)
        if n == 0:
            return -1
        if faults.armed():
            return self.append_values(list(block), partition, timestamp_ms, fsync, key=key)
        if key == "UP" and hasattr(block, "append_to"):
            # formats itself straight into the segment (ingest.DeferredUpBlock)
            res = block.append_to(self._h, int(partition), int(timestamp_ms), fsync)
            if res == -2:
                raise MessageTooLargeError(_lib().oryx_log_last_error().decode())
            if res < 0:
                raise IOError(_lib().oryx_log_last_error().decode())
            return res
        lens = np.ascontiguousarray(block.lengths(), dtype=np.int64)
        buf = block.buf
        if isinstance(buf, np.ndarray):
            ptr = ctypes.c_void_p(buf.ctypes.data)
        else:
            ptr = ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p)
        kb = _b(key)
        res = _lib().oryx_log_append_values_gap(self._h, int(partition), kb,
                                                -1 if kb is None else len(kb), ptr,
                                                lens.ctypes.data_as(ctypes.c_void_p), n,
                                                int(block.sep), int(timestamp_ms),
                                                int(bool(fsync)))
        if res == -2:
            raise MessageTooLargeError(_lib().oryx_log_last_error().decode())
        if res < 0:
            raise IOError(_lib().oryx_log_last_error().decode())
        return res

    def _append_corrupted(self, records, partition, timestamp_ms, fsync) -> int:
        p = partition if partition >= 0 else (0 if self.partitions == 1 else
                                              self.partition_for(records[0][0]))
        pdir = os.path.join(self.root, self.name, str(p))
        segs = sorted(f for f in os.listdir(pdir) if f.endswith(".log")) if \
            os.path.isdir(pdir) else []
        before = os.path.getsize(os.path.join(pdir, segs[-1])) if segs else 0
        res = self.append_batch(list(records), p, timestamp_ms, fsync)
        segs = sorted(f for f in os.listdir(pdir) if f.endswith(".log"))
        seg = os.path.join(pdir, segs[-1])
        start = before if os.path.getsize(seg) > before else 0
        with open(seg, "r+b") as f:
            f.seek(start + _FRAME_HEADER)        # first payload byte of the first record
            b = f.read(1)
            f.seek(start + _FRAME_HEADER)
            f.write(bytes([(b[0] if b else 0) ^ 0xFF]))
        return res

    def begin_offset(self, partition: int) -> int:
        return _lib().oryx_log_begin_offset(self._h, partition)

    def end_offset(self, partition: int) -> int:
        return _lib().oryx_log_end_offset(self._h, partition)

    def end_offsets(self) -> List[int]:
        return [self.end_offset(p) for p in range(self.partitions)]

    def retain(self, max_age_ms: int) -> int:
        cutoff = int(time.time() * 1000) - int(max_age_ms)
        return _lib().oryx_log_retain(self._h, cutoff)

    def reader(self, partition: int, offset: int) -> "PartitionReader":
        return PartitionReader(self, partition, offset)

    def segment_bases(self, partition: int) -> List[int]:
        """First offsets of the partition's segment files, ascending."""
        pdir = os.path.join(self.root, self.name, str(partition))
        out = []
        try:
            names = os.listdir(pdir)
        except OSError:
            return out
        for f in names:
            if f.endswith(".log") and f[:-4].isdigit():
                out.append(int(f[:-4]))
        return sorted(out)


_FRAME_HEADER = 32     # u32 magic, u32 crc, u64 offset, i64 ts, u32 key len, u32 value len
_FRAME = struct.Struct("<IIqqII")


class LogCorruptionError(IOError):
    """A record failed its CRC check with later records present (not a torn tail write)."""


_TLS = threading.local()


class PartitionReader:
    """Tails one partition from an offset (``-1`` = current end)."""

    def __init__(self, topic: Topic, partition: int, offset: int):
        self.topic = topic
        self.partition = partition
        self._r = _lib().oryx_reader_open(topic.handle, partition, int(offset))
        if not self._r:
            raise IOError(_lib().oryx_log_last_error().decode())
        self._cap = 1 << 20
        self._buf = ctypes.create_string_buffer(self._cap)
        self._used = ctypes.c_longlong(0)

    @property
    def position(self) -> int:
        return _lib().oryx_reader_position(self._r)

    def seek(self, offset: int) -> None:
        _lib().oryx_reader_seek(self._r, int(offset))

    def poll(self, max_records: int = 4096, timeout_ms: int = 100
             ) -> List[Tuple[int, int, Optional[str], str]]:
        """Returns up to ``max_records`` (offset, timestamp_ms, key, value) tuples."""
        n = self.poll_raw(max_records, timeout_ms)
        return self.decode_raw(0, n)

    def poll_raw(self, max_records: int = 4096, timeout_ms: int = 100,
                 min_buffer: int = 0) -> int:
        """Reads up to ``max_records`` records into this reader's raw buffer (layout: per
        record i64 offset, i64 timestamp, i32 key length, i32 value length, key, value) and
        returns how many; :meth:`raw_buffer` / :meth:`decode_raw` read them.  ``min_buffer``
        grows the buffer first (bulk loads fetch many large records per call)."""
        lib = _lib()
        if min_buffer > self._cap:
            self._cap = int(min_buffer)
            self._buf = ctypes.create_string_buffer(self._cap)
        while True:
            n = lib.oryx_reader_poll(self._r, self._buf, self._cap, int(max_records),
                                     int(timeout_ms), ctypes.byref(self._used))
            if n == -3:
                raise LogCorruptionError(lib.oryx_log_last_error().decode())
            if n < -3:
                need = -n - 16
                self._cap = max(self._cap * 2, need + 1024)
                self._buf = ctypes.create_string_buffer(self._cap)
                continue
            if n < 0:
                raise IOError(lib.oryx_log_last_error().decode())
            return n

    def raw_buffer(self) -> Tuple[int, int]:
        """(address, bytes used) of the last :meth:`poll_raw`."""
        return ctypes.addressof(self._buf), self._used.value

    def decode_raw(self, start: int, count: int) -> List[Tuple[int, int, Optional[str], str]]:
        """``count`` records of the raw buffer from byte ``start`` as (offset, timestamp_ms,
        key, value) tuples."""
        out = []
        if not count:
            return out
        raw = ctypes.string_at(ctypes.addressof(self._buf) + start, self._used.value - start)
        pos = 0
        n = count
        for _ in range(n):
            off, ts, kl, vl = _HDR.unpack_from(raw, pos)
            pos += 24
            if kl >= 0:
                key = raw[pos:pos + kl].decode("utf-8")
                pos += kl
            else:
                key = None
            val = raw[pos:pos + vl].decode("utf-8")
            pos += vl
            out.append((off, ts, key, val))
        return out

    def poll_frames(self, max_records: int = 1 << 15, min_buffer: int = 64 << 20) -> int:
        """Complete records from the position read in the log's frame layout into this
        reader's frame buffer with one read (CRCs checked on the native threads); never
        waits.  :meth:`frame_buffer` / :meth:`decode_frames` read them."""
        import numpy as np
        lib = _lib()
        buf = getattr(self, "_frames", None)
        if buf is None or len(buf) < min_buffer:
            buf = self._frames = np.empty(int(min_buffer), dtype=np.uint8)
        while True:
            n = lib.oryx_reader_poll_frames(self._r, ctypes.c_void_p(buf.ctypes.data), len(buf),
                                            int(max_records), ctypes.byref(self._used))
            if n == -3:
                raise LogCorruptionError(lib.oryx_log_last_error().decode())
            if n < -3:
                need = -n - 16
                buf = self._frames = np.empty(max(2 * len(buf), need + 1024), dtype=np.uint8)
                continue
            if n < 0:
                raise IOError(lib.oryx_log_last_error().decode())
            return n

    def frame_buffer(self) -> Tuple[int, int]:
        """(address, bytes used) of the last :meth:`poll_frames`."""
        return self._frames.ctypes.data, self._used.value

    def decode_frames(self, start: int, count: int) -> List[Tuple[int, int, Optional[str], str]]:
        """``count`` frames of the frame buffer from byte ``start`` as (offset, timestamp_ms,
        key, value) tuples."""
        out = []
        raw = self._frames[start:self._used.value].tobytes() if count else b""
        pos = 0
        for _ in range(count):
            _, _, off, ts, kl, vl = _FRAME.unpack_from(raw, pos)
            pos += _FRAME_HEADER
            if kl != 0xFFFFFFFF:
                key = raw[pos:pos + kl].decode("utf-8")
                pos += kl
            else:
                key = None
            out.append((off, ts, key, raw[pos:pos + vl].decode("utf-8")))
            pos += vl
        return out

    def read_text_lines(self, end_offset: int):
        """As :meth:`read_text` but the values stay one buffer: (:class:`TextLines` or None,
        records read).  No per-record Python string is created: the records are read
        natively straight into one array sized by the segment bytes left to read."""
        import numpy as np
        from ..textlines import TextLines
        lib = _lib()
        start = self.position
        if start >= end_offset:
            return TextLines(b"", 0), 0
        cap = max(int(lib.oryx_reader_text_bound(self._r, int(end_offset))), 1 << 16)
        # (from 8 MB: a drain reads a partition as one buffer per 64 MB segment, freed in bulk
        # after the concatenation -- on the reaper thread, not the layer's)
        buf = hostbuf.empty(cap, min_bytes=8 << 20)
        used_total = total = 0
        used = ctypes.c_longlong(0)
        flags = ctypes.c_int(0)
        while self.position < end_offset:
            n = lib.oryx_reader_read_text(self._r, int(end_offset),
                                          ctypes.c_void_p(buf.ctypes.data + used_total),
                                          cap - used_total, ctypes.byref(used),
                                          ctypes.byref(flags))
            if n == -3:
                raise LogCorruptionError(lib.oryx_log_last_error().decode())
            if n < 0:
                raise IOError(lib.oryx_log_last_error().decode())
            if flags.value & 3:
                self.seek(start)
                return None, 0
            if flags.value & 4:
                # more was appended since the bound was taken: grow
                cap = max(2 * cap, used_total + int(used.value))
                grown = hostbuf.empty(cap, min_bytes=8 << 20)
                grown[:used_total] = buf[:used_total]
                buf = grown
                continue
            if n == 0:
                break
            used_total += int(used.value)
            total += n
        return TextLines(buf[:used_total], total), total

    def text_bound(self, end_offset: int) -> int:
        """Upper bound of the bytes :meth:`read_text_into` writes up to ``end_offset``."""
        if self.position >= end_offset:
            return 0
        return int(_lib().oryx_reader_text_bound(self._r, int(end_offset)))

    def read_text_into(self, end_offset: int, addr: int, cap: int):
        """As :meth:`read_text_lines`, into ``cap`` bytes at ``addr`` (a slice of the caller's
        buffer): (bytes written, records read), or None -- position unchanged -- when a record
        has a key or a multi-line value, or the text does not fit."""
        lib = _lib()
        start = self.position
        used_total = total = 0
        used = ctypes.c_longlong(0)
        flags = ctypes.c_int(0)
        while self.position < end_offset:
            n = lib.oryx_reader_read_text(self._r, int(end_offset),
                                          ctypes.c_void_p(addr + used_total),
                                          cap - used_total, ctypes.byref(used),
                                          ctypes.byref(flags))
            if n == -3:
                raise LogCorruptionError(lib.oryx_log_last_error().decode())
            if n < 0:
                raise IOError(lib.oryx_log_last_error().decode())
            if flags.value & 7:
                self.seek(start)
                return None
            if n == 0:
                break
            used_total += int(used.value)
            total += n
        return used_total, total

    def read_text(self, end_offset: int) -> Tuple[Optional[List[str]], int]:
        """Values of every record up to ``end_offset`` (exclusive) in one bulk native read.

        Returns (values, records read); values is None when a record has a key or a value
        contains a newline (the position is then back where it started: use :meth:`poll`).
        """
        lib = _lib()
        start = self.position
        chunks: List[bytes] = []
        total = 0
        # one reusable 16 MB buffer per thread (zeroing a fresh one per call costs more than
        # the read); a record larger than that gets a private one
        buf = getattr(_TLS, "text_buf", None)
        if buf is None:
            buf = _TLS.text_buf = ctypes.create_string_buffer(16 << 20)
        cap = len(buf)
        used = ctypes.c_longlong(0)
        flags = ctypes.c_int(0)
        while self.position < end_offset:
            n = lib.oryx_reader_read_text(self._r, int(end_offset), buf, cap,
                                          ctypes.byref(used), ctypes.byref(flags))
            if n == -3:
                raise LogCorruptionError(lib.oryx_log_last_error().decode())
            if n < 0:
                raise IOError(lib.oryx_log_last_error().decode())
            if flags.value & 3:
                self.seek(start)
                return None, 0
            if flags.value & 4:
                # the next record alone is larger than the buffer: the native call reported
                # the size it needs
                cap = max(int(used.value), 2 * cap)
                buf = ctypes.create_string_buffer(cap)
                continue
            if n == 0:
                break
            chunks.append(ctypes.string_at(buf, used.value))
            total += n
        if not chunks:
            return [], 0
        text = b"".join(chunks).decode("utf-8")
        vals = text.split("\n")
        vals.pop()                     # trailing separator
        return vals, total

    def close(self) -> None:
        if self._r:
            _lib().oryx_reader_close(self._r)
            self._r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def get_offsets(root: str, topic: str, group: str, partitions: int) -> Dict[int, int]:
    out = {}
    lib = _lib()
    for p in range(partitions):
        o = lib.oryx_offsets_get(_b(root), _b(topic), _b(group), p)
        if o >= 0:
            out[p] = o
    return out


def set_offsets(root: str, topic: str, group: str, offsets: Dict[int, int]) -> None:
    if not offsets:
        return
    n = len(offsets)
    parts = (ctypes.c_int * n)(*offsets.keys())
    offs = (ctypes.c_longlong * n)(*offsets.values())
    if _lib().oryx_offsets_set(_b(root), _b(topic), _b(group), n, parts, offs) != 0:
        raise IOError(_lib().oryx_log_last_error().decode())


class TopicConsumer:
    """Consumes all partitions of a topic, round-robin.

    ``start``: ``"earliest"`` (replay from the beginning, as speed/serving do for the update
    topic), ``"latest"``, or a dict partition->offset (resume); a ``group`` makes
    :meth:`commit` persist offsets.
    """

    def __init__(self, topic: Topic, start="latest", group: Optional[str] = None):
        self.topic = topic
        self.group = group
        self.readers: List[PartitionReader] = []
        for p in range(topic.partitions):
            if isinstance(start, dict):
                off = start.get(p, topic.end_offset(p))
            elif start == "earliest":
                off = topic.begin_offset(p)
            else:
                off = topic.end_offset(p)
            self.readers.append(PartitionReader(topic, p, off))
        self._closed = False

    def positions(self) -> Dict[int, int]:
        return {r.partition: r.position for r in self.readers}

    def poll(self, max_records: int = 4096, timeout_ms: int = 100
             ) -> List[Tuple[int, int, int, Optional[str], str]]:
        """(partition, offset, ts, key, value) tuples; waits up to timeout for any record."""
        out = []
        deadline = time.monotonic() + timeout_ms / 1000.0
        while True:
            for r in self.readers:
                for rec in r.poll(max_records, 0):
                    out.append((r.partition,) + rec)
            if out or time.monotonic() >= deadline or self._closed:
                return out
            if len(self.readers) == 1:
                rem = max(0, int((deadline - time.monotonic()) * 1000))
                for rec in self.readers[0].poll(max_records, rem):
                    out.append((0,) + rec)
                return out
            time.sleep(0.002)

    def __iter__(self) -> Iterator[Tuple[Optional[str], str]]:
        while not self._closed:
            for _, _, _, k, v in self.poll():
                yield k, v

    def commit(self) -> None:
        if self.group:
            set_offsets(self.topic.root, self.topic.name, self.group, self.positions())

    def close(self) -> None:
        self._closed = True
        for r in self.readers:
            r.close()
