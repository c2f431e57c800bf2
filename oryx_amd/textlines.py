"""Newline-delimited messages held as one byte buffer (the batch layer's bulk data form).

The reference moves an interval's messages and its whole history through Spark as
partitioned binary SequenceFiles (``[lambda]/batch/BatchUpdateFunction.java:103-130``,
``SaveToHDFSFunction.java:59-76``): no per-record object until an app parses them.  Here the
same role is played by :class:`TextLines`: the messages of a log drain, of a part file or of a
train/test split stay in ONE UTF-8 buffer in which every line ends with ``b"\\n"``; the native
parsers (``ingest.parse_ratings`` and friends) read that buffer directly, part files are that
buffer written out, and selections (train/test masks, shares) are gathered natively.  It is a
read-only ``Sequence[str]``, so any code that iterates or indexes it still works -- decoding
then happens lazily, once.
"""

from __future__ import annotations

import collections.abc
import ctypes
from typing import Iterable, List, Optional, Sequence, Union

import numpy as np

from . import hostbuf, native

__all__ = ["TextLines", "LineSelection", "LineConcat", "concat_lines", "as_buffer",
           "part_edges"]

_NL = 10


def _addr(buf) -> int:
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data
    if isinstance(buf, bytearray):
        return ctypes.addressof((ctypes.c_char * len(buf)).from_buffer(buf))
    return ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value


class TextLines(collections.abc.Sequence):
    """``n`` messages in ``buf`` (bytes / bytearray / uint8 array), each followed by ``\\n``.

    ``n`` may be given (the log's bulk read knows it); the line index (end offsets) is built
    natively on first indexed access.
    """

    __slots__ = ("buf", "_n", "_ends", "_strs", "segments", "__weakref__")

    def __init__(self, buf, n: Optional[int] = None, ends: Optional[np.ndarray] = None):
        if isinstance(buf, memoryview):
            buf = bytes(buf)
        self.buf = buf
        self._ends = ends
        self._strs: Optional[List[str]] = None
        if n is None:
            n = len(self.ends()) if len(buf) else 0
        self._n = int(n)
        # provenance of consecutive byte ranges: [(key, n_lines, n_bytes)], key None for data
        # without a stable identity; a keyed range is the content of e.g. one past part file
        # (``layers.batch.read_past_data``), so a parse of it can be reused across generations
        # (``models.als.history``).  None: one unkeyed range.
        self.segments: Optional[List[tuple]] = None

    def with_key(self, key) -> "TextLines":
        """Mark the whole buffer as one keyed segment (returns self)."""
        self.segments = [(key, self._n, len(self.buf))]
        return self

    def segment_list(self) -> List[tuple]:
        return self.segments if self.segments is not None else [(None, self._n, len(self.buf))]

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_strings(cls, strs: Iterable[str]) -> "TextLines":
        strs = list(strs)
        if not strs:
            return cls(b"", 0)
        data = ("\n".join(strs) + "\n").encode("utf-8")
        return cls(data, len(strs))

    @classmethod
    def from_bytes(cls, data: bytes) -> "TextLines":
        """Text (e.g. a part file); a missing final newline is added."""
        if data and data[-1:] != b"\n":
            data = bytes(data) + b"\n"
        return cls(data)

    # ------------------------------------------------------------------ sequence
    def __len__(self) -> int:
        return self._n

    def nbytes(self) -> int:
        return len(self.buf)

    def ends(self) -> np.ndarray:
        """Offset of every line's ``\\n`` (int64, native threaded scan)."""
        if self._ends is None:
            n_buf = len(self.buf)
            if n_buf == 0:
                self._ends = np.zeros(0, dtype=np.int64)
            else:
                cap = getattr(self, "_n", None) or max(1, n_buf // 8)
                while True:
                    out = np.empty(int(cap), dtype=np.int64)
                    got = native.runtime().oryx_line_ends(_addr(self.buf), n_buf,
                                                          out.ctypes.data, int(cap))
                    if got >= 0:
                        self._ends = out[:got]
                        break
                    cap = -got
        return self._ends

    def _decode_all(self) -> List[str]:
        if self._strs is None:
            text = bytes(self.buf).decode("utf-8") if not isinstance(self.buf, str) else self.buf
            parts = text.split("\n")
            if parts and parts[-1] == "":
                parts.pop()
            self._strs = parts
        return self._strs

    def __getitem__(self, j):
        if isinstance(j, slice):
            idx = np.arange(self._n)[j]
            return self.take(idx)
        if self._strs is not None:
            return self._strs[j]
        n = self._n
        if j < 0:
            j += n
        if not 0 <= j < n:
            raise IndexError(j)
        if self._ends is None and j in (0, n - 1):
            # first / last line without indexing the whole buffer
            b = bytes(memoryview(self.buf)[:1 << 20]) if j == 0 else None
            if j == 0 and b is not None and b"\n" in b:
                return b[:b.index(b"\n")].decode("utf-8")
            if j == n - 1:
                mv = memoryview(self.buf)
                tail = bytes(mv[max(0, len(mv) - (1 << 20)):len(mv) - 1])
                if b"\n" in tail or len(tail) == len(mv) - 1:
                    return tail[tail.rfind(b"\n") + 1:].decode("utf-8")
        e = self.ends()
        b = int(e[j - 1]) + 1 if j else 0
        return bytes(memoryview(self.buf)[b:int(e[j])]).decode("utf-8")

    def __iter__(self):
        return iter(self._decode_all())

    def __add__(self, other):
        return concat_lines([self, other])

    def __radd__(self, other):
        return concat_lines([other, self])

    def __eq__(self, other):
        if isinstance(other, TextLines):
            return self._n == other._n and bytes(self.buf) == bytes(other.buf)
        if isinstance(other, (list, tuple)):
            return list(self) == list(other)
        return NotImplemented

    def __repr__(self):
        return "TextLines[%d lines, %d bytes]" % (self._n, len(self.buf))

    # ------------------------------------------------------------------ bulk
    def joined(self):
        """The whole buffer: every message followed by ``\\n`` (what native parsers take)."""
        return self.buf

    def take(self, sel) -> "TextLines":
        """Lines selected by a boolean mask or an index array, in that order (native gather)."""
        sel = np.asarray(sel)
        idx = np.flatnonzero(sel) if sel.dtype == bool else sel.astype(np.int64)
        if len(idx) == self._n and (len(idx) == 0 or (idx[0] == 0 and
                                                      np.all(np.diff(idx) == 1))):
            return self
        if len(idx) == 0:
            return TextLines(b"", 0)
        e = self.ends()
        starts = np.r_[0, e[:-1] + 1]
        size = int((e[idx] - starts[idx] + 1).sum())
        out = hostbuf.empty(size)
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        native.runtime().oryx_gather_lines(_addr(self.buf), e.ctypes.data, idx.ctypes.data,
                                           len(idx), out.ctypes.data)
        return TextLines(out, len(idx))


class _Lazy(TextLines):
    """A :class:`TextLines` whose bytes are built only when something reads them: every
    accessor goes through :meth:`materialize`.  Parsers that understand the subclasses
    (``models.features.FeatureHistory``) work from their parts instead."""

    __slots__ = ("_mat",)

    def materialize(self) -> TextLines:
        if self._mat is None:
            self._mat = self._build()
        return self._mat

    def _build(self) -> TextLines:
        raise NotImplementedError

    buf = property(lambda self: self.materialize().buf)
    segments = property(lambda self: self.segment_list_or_none())

    def segment_list_or_none(self) -> Optional[List[tuple]]:
        return self.materialize().segments

    def ends(self) -> np.ndarray:
        return self.materialize().ends()

    def nbytes(self) -> int:
        return self.materialize().nbytes()

    def segment_list(self) -> List[tuple]:
        return self.materialize().segment_list()

    def with_key(self, key) -> "TextLines":
        return self.materialize().with_key(key)

    def __getitem__(self, j):
        return self.materialize()[j]

    def __iter__(self):
        return iter(self.materialize())

    def _decode_all(self) -> List[str]:
        return self.materialize()._decode_all()

    def take(self, sel) -> "TextLines":
        return self.materialize().take(sel)

    def __repr__(self):
        return "%s[%d lines]" % (type(self).__name__, self._n)


class LineSelection(_Lazy):
    """Lines ``index`` (increasing) of ``parent``, gathered into a buffer of their own only if
    one is asked for.  The random train / test split of the feature apps
    (``MLUpdate.split_new_data_to_train_test``) returns these: their parser parses the parent
    once and selects rows on the device, so the split copies no text and the parse of the
    whole interval is the one a later generation adopts for its part file."""

    __slots__ = ("parent", "index")

    def __init__(self, parent: TextLines, index: np.ndarray):
        self.parent = parent
        self.index = np.ascontiguousarray(index, dtype=np.int64)
        self._n = len(self.index)
        self._ends = None
        self._strs = None
        self._mat = None

    def _build(self) -> TextLines:
        return self.parent.take(self.index)


class LineConcat(_Lazy):
    """``parts`` one after another (the train selection followed by past part files),
    concatenated only if a buffer is asked for."""

    __slots__ = ("parts",)

    def __init__(self, parts: Sequence[TextLines]):
        flat: List[TextLines] = []
        for p in parts:
            flat.extend(p.parts if isinstance(p, LineConcat) else [p])
        self.parts = flat
        self._n = sum(len(p) for p in flat)
        self._ends = None
        self._strs = None
        self._mat = None

    def segment_list_or_none(self) -> Optional[List[tuple]]:
        # (from the parts, without joining them, when none of them is lazy)
        if any(isinstance(p, _Lazy) for p in self.parts):
            return self.materialize().segments
        if all(p.segments is None for p in self.parts):
            return None
        return [seg for p in self.parts for seg in p.segment_list()]

    def segment_list(self) -> List[tuple]:
        segs = self.segment_list_or_none()
        return segs if segs is not None else self.materialize().segment_list()

    def _build(self) -> TextLines:
        return concat_lines([p.materialize() if isinstance(p, _Lazy) else p
                             for p in self.parts])


def concat_lines(parts: Sequence[Union[TextLines, Sequence[str], None]]):
    """Concatenation that stays a :class:`TextLines` when every non-empty part is one (else a
    plain list of strings); a :class:`LineConcat` when a part is a lazy selection."""
    parts = [p for p in parts if p is not None and len(p)]
    if not parts:
        return TextLines(b"", 0)
    if len(parts) == 1 and isinstance(parts[0], TextLines):
        return parts[0]
    if all(isinstance(p, TextLines) for p in parts) and \
            any(isinstance(p, _Lazy) for p in parts):
        return LineConcat(parts)
    if all(isinstance(p, TextLines) for p in parts):
        bufs = [np.frombuffer(p.buf, dtype=np.uint8) if not isinstance(p.buf, np.ndarray)
                else np.ascontiguousarray(p.buf) for p in parts]
        lens = np.array([len(b) for b in bufs], dtype=np.int64)
        out = hostbuf.empty(int(lens.sum()))
        ptrs = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
        # threaded native copy (hundreds of MB per drain)
        native.runtime().oryx_concat_buffers(ptrs.ctypes.data, lens.ctypes.data, len(bufs),
                                             out.ctypes.data)
        res = TextLines(out, sum(len(p) for p in parts))
        if any(p.segments is not None for p in parts):
            res.segments = [seg for p in parts for seg in p.segment_list()]
        return res
    out: List[str] = []
    for p in parts:
        out.extend(p)
    return out


def as_buffer(lines) -> Optional[object]:
    """The newline-terminated byte buffer of ``lines`` when it is a :class:`TextLines`."""
    return lines.joined() if isinstance(lines, TextLines) else None


# A large interval is saved as several part files written concurrently (one write() per file
# scales with the files on the box's filesystem; one file does not: scripts/write_probe.py).
PART_FILE_BYTES = 1 << 30
MAX_PART_FILES = 16
SPLIT_MIN_BYTES = 8 << 30


def part_edges(buf, nbytes: Optional[int] = None) -> List[int]:
    """Byte offsets [0, ..., nbytes] splitting a newline-terminated buffer into the part files
    it is saved as (from SPLIT_MIN_BYTES): ceil(nbytes / PART_FILE_BYTES) pieces (at most
    MAX_PART_FILES), each cut
    just after the first newline at or past its even share.  The batch layer's save and the
    feature parsers' adoption of part files (models/features.py) both use this, so a saved
    interval's files are byte ranges the parser of that interval can name."""
    b = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    n = len(b) if nbytes is None else int(nbytes)
    parts = 1 if n < SPLIT_MIN_BYTES else min(MAX_PART_FILES, max(1, -(-n // PART_FILE_BYTES)))
    edges = [0]
    for j in range(1, parts):
        p = max(edges[-1], n * j // parts)
        q = -1
        step = 1 << 20
        while p < n and q < 0:
            w = b[p:min(n, p + step)]
            hit = np.flatnonzero(w == 10)
            if len(hit):
                q = p + int(hit[0]) + 1
            p += step
        if q <= edges[-1] or q >= n:
            continue
        edges.append(q)
    edges.append(n)
    return edges
