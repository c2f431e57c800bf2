"""Native ingest helpers: dictionary-encoded rating parsing and fast JSON row formatting.

Thin bindings over ``csrc/runtime/oryx_ingest.cpp`` (see its header for the reference call
sites it replaces).
"""

from __future__ import annotations

import ctypes
import threading
import json
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import hostbuf, native

__all__ = ["IdDict", "parse_ratings", "format_float_rows", "format_als_updates",
           "parse_up_batch"]


class IdDict:
    """Collision-free string -> dense int64 dictionary (insertion order)."""

    def __init__(self):
        self._lib = native.runtime()
        self._h = self._lib.oryx_dict_new()
        # (object array with spare capacity, keys filled): a numpy object array is not a
        # cyclic-GC container, so a 20M-key cache adds nothing to a full collection's walk
        # (a list of 20M strings cost the serving process ~0.5 s per gen-2 pass)
        self._keys_cache: Tuple[np.ndarray, int] = (np.empty(0, dtype=object), 0)
        # key_list is called from many serving threads at once: one of them extends the cache
        self._keys_lock = threading.Lock()

    def __del__(self):
        try:
            self._lib.oryx_dict_free(self._h)
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def __len__(self) -> int:
        return int(self._lib.oryx_dict_size(self._h))

    def clear(self) -> "IdDict":
        """Empty the dictionary, keeping its native table's capacity (reused per batch)."""
        self._lib.oryx_dict_clear(self._h)
        with self._keys_lock:
            self._keys_cache = (np.empty(0, dtype=object), 0)
        return self

    def encode(self, keys: Sequence[str]) -> np.ndarray:
        buf = b"\0".join(k.encode("utf-8") for k in keys) + b"\0"
        out = np.empty(len(keys), dtype=np.int64)
        self._lib.oryx_dict_encode(self._h, buf, len(buf), len(keys),
                                   out.ctypes.data_as(ctypes.c_void_p))
        return out

    def encode_nums(self, values) -> np.ndarray:
        """Encode canonical decimal keys given as int values (< 2^24) in order: the same codes
        as encoding ``[str(v) for v in values]``, without building the strings."""
        vals = np.ascontiguousarray(values, dtype=np.int32)
        out = np.empty(len(vals), dtype=np.int64)
        vp = ctypes.c_void_p
        rc = self._lib.oryx_dict_encode_nums(self._h, vals.ctypes.data_as(vp), len(vals),
                                             out.ctypes.data_as(vp))
        if rc < 0:
            raise ValueError("numeric key out of range")
        return out

    def merge_from(self, other: "IdDict") -> np.ndarray:
        """Insert ``other``'s keys (in its code order); returns the codes they have here."""
        out = np.empty(len(other), dtype=np.int64)
        n = self._lib.oryx_dict_merge(self._h, other._h, out.ctypes.data_as(ctypes.c_void_p))
        if n != len(out):
            raise ValueError("dictionary merge failed")
        return out

    def get(self, key: str) -> int:
        b = key.encode("utf-8")
        return int(self._lib.oryx_dict_get(self._h, b, len(b)))

    # ---- blob forms (keys as one uint8 buffer + int64 end offsets; no Python strings)
    def owners(self, world: int, start: int = 0) -> np.ndarray:
        """``zlib.crc32(key) % world`` of every key from code ``start`` on (int64)."""
        out = np.empty(max(0, len(self) - start), dtype=np.int64)
        if len(out):
            self._lib.oryx_dict_owners(self._h, int(start), int(world), _ptr(out))
        return out

    def encode_blob(self, blob: np.ndarray, ends: np.ndarray) -> np.ndarray:
        """Insert the keys of a blob in order; returns their codes."""
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        ends = np.ascontiguousarray(ends, dtype=np.int64)
        out = np.empty(len(ends), dtype=np.int64)
        if len(ends):
            self._lib.oryx_dict_encode_blob(self._h, _ptr(blob), _ptr(ends), len(ends),
                                            _ptr(out))
        return out

    def find_blob(self, blob: np.ndarray, ends: np.ndarray) -> np.ndarray:
        """Codes of the keys of a blob (-1 when absent); inserts nothing."""
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        ends = np.ascontiguousarray(ends, dtype=np.int64)
        out = np.empty(len(ends), dtype=np.int64)
        if len(ends):
            self._lib.oryx_dict_find_blob(self._h, _ptr(blob), _ptr(ends), len(ends),
                                          _ptr(out))
        return out

    def keys_blob(self, codes: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        """(blob, ends) of the keys of ``codes`` in that order (default: every key)."""
        if codes is None:
            codes = np.arange(len(self), dtype=np.int64)
        codes = np.ascontiguousarray(codes, dtype=np.int64)
        ends = np.empty(len(codes), dtype=np.int64)
        if not len(codes):
            return np.zeros(0, dtype=np.uint8), ends
        cap = max(16 * len(codes), 1 << 12)
        while True:
            blob = np.empty(cap, dtype=np.uint8)
            used = self._lib.oryx_dict_keys_blob_sel(self._h, _ptr(codes), len(codes),
                                                     _ptr(blob), cap, _ptr(ends))
            if used >= 0:
                return blob[:used], ends
            cap = -used

    @classmethod
    def from_blob(cls, blob: np.ndarray, ends: np.ndarray) -> "IdDict":
        d = cls()
        d.encode_blob(blob, ends)
        return d

    def keys(self) -> List[str]:
        """Every key in code order (a copy)."""
        return list(self.key_list())

    def key_list(self) -> np.ndarray:
        """Every key in code order: a read-only view of the dictionary's own cached object
        array (no copy -- per-request lookups of a few codes in a 1M-key dictionary must not
        copy it); indexes, slices and iterates like a list."""
        n = len(self)
        arr, have = self._keys_cache
        if have >= n:
            return arr[:n]
        with self._keys_lock:
            arr, have = self._keys_cache
            if have < n:
                new = self._fetch_keys(have, n)
                if len(arr) < n:
                    # 1/8 headroom (at least double once filled): growing copies every key
                    # reference with the GIL held -- at 20M keys a 30-40 ms stall of every
                    # serving thread, which an exact-size cache paid on the first new key
                    # after a model load (profiles/r6_traffic_20m_250_lsh03_v4.json)
                    grown = np.empty(max(n + n // 8, 2 * len(arr), 1024), dtype=object)
                    grown[:have] = arr[:have]
                    arr = grown
                arr[have:n] = new
                # published as one tuple: readers see the old or the whole new state
                self._keys_cache = (arr, n)
        return arr[:n]

    def _fetch_keys(self, have: int, n: int) -> List[str]:
        """Keys ``have`` .. ``n - 1`` in code order (one native call)."""
        ends = np.empty(n - have, dtype=np.int64)
        cap = 1 << 16
        while True:
            buf = ctypes.create_string_buffer(cap)
            used = self._lib.oryx_dict_keys_blob(self._h, have, n, buf, cap,
                                                 ends.ctypes.data_as(ctypes.c_void_p))
            if used >= 0:
                break
            cap = -used + 1
        raw = ctypes.string_at(buf, used)
        starts = np.r_[0, ends[:-1]].tolist()
        if used == (ends[-1] if len(ends) else 0) and raw.isascii():
            text = raw.decode("ascii")
            return [text[a:b] for a, b in zip(starts, ends.tolist())]
        return [raw[a:b].decode("utf-8") for a, b in zip(starts, ends.tolist())]


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def blob_strings(blob: np.ndarray, ends: np.ndarray) -> List[str]:
    """Python strings of a key blob (only where strings are really needed)."""
    raw = bytes(memoryview(np.ascontiguousarray(blob, dtype=np.uint8)))
    e = np.asarray(ends, dtype=np.int64).tolist()
    s = [0] + e[:-1]
    if raw.isascii():
        text = raw.decode("ascii")
        return [text[a:b] for a, b in zip(s, e)]
    return [raw[a:b].decode("utf-8") for a, b in zip(s, e)]


def blob_hash64(blob: np.ndarray, ends: np.ndarray, seed: int = 0) -> np.ndarray:
    """uint64 hash of every key of a (blob, ends) pair (native FNV-1a + splitmix64)."""
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.int64)
    out = np.empty(len(ends), dtype=np.uint64)
    if len(ends):
        from . import native
        native.runtime().oryx_blob_hash64(_ptr(blob), _ptr(ends), len(ends),
                                          int(seed) & ((1 << 64) - 1), _ptr(out))
    return out


def strings_blob(keys: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    """(blob, ends) of Python strings."""
    enc = [k.encode("utf-8") for k in keys]
    ends = np.cumsum(np.fromiter((len(e) for e in enc), dtype=np.int64, count=len(enc)))
    blob = np.frombuffer(b"".join(enc), dtype=np.uint8) if enc else np.zeros(0, np.uint8)
    return blob, ends


def parse_ratings(lines, users: IdDict, items: IdDict, default_ts: int,
                  strict: bool = False) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Parse rating lines (str list, newline-joined bytes or a :class:`TextLines` buffer)
    -> (u, i, strength, ts) arrays."""
    from .textlines import TextLines
    if isinstance(lines, TextLines):
        buf = lines.joined()
        n_max = len(lines) + 1
        if isinstance(buf, np.ndarray):
            data = ctypes.cast(ctypes.c_void_p(buf.ctypes.data), ctypes.c_char_p)
            n_bytes = buf.nbytes
        else:
            data, n_bytes = bytes(buf), len(buf)
        return _parse_ratings_buf(data, n_bytes, n_max, users, items, default_ts, strict)
    if isinstance(lines, (bytes, bytearray)):
        data = bytes(lines)
        n_max = data.count(b"\n") + 1
    else:
        data = "\n".join(lines).encode("utf-8")
        n_max = len(lines) + 1
    return _parse_ratings_buf(data, len(data), n_max, users, items, default_ts, strict)


def parse_timestamps(lines, default_ts: int = 0) -> np.ndarray:
    """Timestamps of the rating lines :func:`parse_ratings` accepts (same rows), without
    encoding any ID -- what a time-based train/test split needs."""
    from .textlines import TextLines
    if isinstance(lines, TextLines):
        buf = lines.joined()
        n_max = len(lines) + 1
        if isinstance(buf, np.ndarray):
            data = ctypes.cast(ctypes.c_void_p(buf.ctypes.data), ctypes.c_char_p)
            n_bytes = buf.nbytes
        else:
            data, n_bytes = bytes(buf), len(buf)
    else:
        data = (bytes(lines) if isinstance(lines, (bytes, bytearray))
                else "\n".join(lines).encode("utf-8"))
        n_bytes = len(data)
        n_max = data.count(b"\n") + 1
    return _parse_ratings_buf(data, n_bytes, n_max, None, None, default_ts, False)[3]


def _lines_ptr(lines):
    buf = lines.joined()
    if not isinstance(buf, np.ndarray):
        buf = np.frombuffer(bytes(buf), dtype=np.uint8)
    return buf, ctypes.c_void_p(buf.ctypes.data), int(buf.nbytes)


def ts_range(lines, default_ts: int = 0) -> Optional[Tuple[int, int]]:
    """(min, max) timestamp of a :class:`~oryx_amd.textlines.TextLines` buffer's rating
    lines (native, threaded), or None without any parsable line."""
    buf, ptr, n = _lines_ptr(lines)
    lo, hi = ctypes.c_longlong(0), ctypes.c_longlong(0)
    rows = native.runtime().oryx_ts_range(ptr, n, int(default_ts), ctypes.byref(lo),
                                          ctypes.byref(hi))
    return (int(lo.value), int(hi.value)) if rows > 0 else None


def split_by_time(lines, boundary: int, default_ts: int = 0):
    """(lines with timestamp < boundary, the rest) of a TextLines buffer, both TextLines in
    the original order; unparsable lines are dropped (native, threaded, one pass)."""
    from .textlines import TextLines
    buf, ptr, n = _lines_ptr(lines)
    lo = np.empty(n + 1, dtype=np.uint8)
    hi = np.empty(n + 1, dtype=np.uint8)
    c = [ctypes.c_longlong(0) for _ in range(4)]
    native.runtime().oryx_split_by_time(ptr, n, int(default_ts), int(boundary), _ptr(lo),
                                        _ptr(hi), *[ctypes.byref(x) for x in c])
    return TextLines(lo[:c[2].value], int(c[0].value)), TextLines(hi[:c[3].value],
                                                                  int(c[1].value))


def _parse_ratings_buf(data, n_bytes: int, n_max: int, users: "IdDict", items: "IdDict",
                       default_ts: int, strict: bool):
    u = np.empty(n_max, dtype=np.int64)
    i = np.empty(n_max, dtype=np.int64)
    s = np.empty(n_max, dtype=np.float64)
    t = np.empty(n_max, dtype=np.int64)
    vp = ctypes.c_void_p
    n = native.runtime().oryx_parse_ratings(
        data, int(n_bytes), users.handle if users is not None else None,
        items.handle if items is not None else None, u.ctypes.data_as(vp),
        i.ctypes.data_as(vp), s.ctypes.data_as(vp), t.ctypes.data_as(vp), n_max,
        int(default_ts), int(bool(strict)))
    if n < 0:
        raise ValueError("Bad input line %d" % (-n - 1))
    return u[:n], i[:n], s[:n], t[:n]


def _ids_blob(ids: Sequence[str]):
    enc = [i.encode("utf-8") for i in ids]
    ends = np.cumsum(np.fromiter((len(e) for e in enc), dtype=np.int64, count=len(enc)))
    return b"".join(enc), ends


class RowMap:
    """Native ``id -> row`` map mirroring a feature store's index, so a batch's dictionary of
    IDs translates to store rows in one call (no per-ID Python lookups)."""

    def __init__(self):
        self._lib = native.runtime()
        self._h = self._lib.oryx_rowmap_new()

    def __del__(self):
        try:
            if self._h:
                self._lib.oryx_rowmap_free(self._h)
                self._h = None
        except Exception:
            pass

    def __len__(self) -> int:
        return int(self._lib.oryx_rowmap_size(self._h))

    def set(self, ids: Sequence[str], rows) -> None:
        if not len(ids):
            return
        blob, ends = _ids_blob(ids)
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        vp = ctypes.c_void_p
        self._lib.oryx_rowmap_set(self._h, blob, ends.ctypes.data_as(vp),
                                  rows.ctypes.data_as(vp), len(ids))

    def remove(self, ids: Sequence[str]) -> None:
        if not len(ids):
            return
        blob, ends = _ids_blob(ids)
        self._lib.oryx_rowmap_remove(self._h, blob, ends.ctypes.data_as(ctypes.c_void_p),
                                     len(ids))

    def key_suffixes(self, n_rows: int) -> np.ndarray:
        """int64 [n_rows]: the trailing decimal digits of the key at each row (-1: no key
        there, or no digits), in one native pass over the map."""
        out = np.empty(max(int(n_rows), 0), dtype=np.int64)
        if len(out):
            self._lib.oryx_rowmap_key_suffixes(self._h, out.ctypes.data_as(ctypes.c_void_p),
                                               len(out))
        return out

    def translate(self, d: "IdDict") -> np.ndarray:
        """Row of every key of ``d`` in code order (-1: not in the map)."""
        out = np.empty(len(d), dtype=np.int64)
        if len(out):
            self._lib.oryx_rowmap_translate(self._h, d.handle,
                                            out.ctypes.data_as(ctypes.c_void_p))
        return out


class SpeedBatch:
    """One speed-layer micro-batch parsed against the stores' id -> row maps
    (``csrc/runtime/oryx_ingest.cpp`` ``oryx_speed_*``): lines are parsed on the native
    threads with each user / item resolved straight to its store row (no per-batch
    dictionary), pairs aggregated in time order, and the UP messages assembled from the
    events' own key bytes.  Reused across batches (its native buffers keep their capacity)."""

    def __init__(self):
        self._lib = native.runtime()
        self._h = self._lib.oryx_speed_new()
        self._buf = None
        self._gen = 0        # bumped by every parse (deferred blocks check it)

    def __del__(self):
        try:
            if self._h:
                self._lib.oryx_speed_free(self._h)
                self._h = None
        except Exception:
            pass

    def parse(self, lines, xmap: "RowMap", ymap: "RowMap", default_ts: int = 0) -> int:
        """Parse ``lines`` (TextLines, bytes or strings; kept referenced until the next
        parse: the events' keys point into it).  Returns the number of events."""
        from .textlines import TextLines
        if isinstance(lines, TextLines):
            buf = lines.joined()
            if not isinstance(buf, np.ndarray):
                buf = np.frombuffer(bytes(buf), dtype=np.uint8)
        elif isinstance(lines, (bytes, bytearray)):
            buf = np.frombuffer(bytes(lines), dtype=np.uint8)
        else:
            buf = np.frombuffer("\n".join(lines).encode("utf-8"), dtype=np.uint8)
        self._buf = buf
        self._gen += 1
        return int(self._lib.oryx_speed_parse(self._h, _ptr(buf), int(buf.nbytes), xmap._h,
                                              ymap._h, int(default_ts)))

    def counts(self) -> Tuple[int, int, int, int]:
        """(events, new users, new items, aggregated pairs)."""
        out = np.zeros(4, dtype=np.int64)
        self._lib.oryx_speed_counts(self._h, _ptr(out))
        return tuple(int(x) for x in out)

    def aggregate(self, implicit: bool) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(user rows, item rows, values) of the aggregated pairs (rows -1: not in the
        store)."""
        n = self.counts()[0]
        u = np.empty(max(n, 1), dtype=np.int64)
        i = np.empty(max(n, 1), dtype=np.int64)
        v = np.empty(max(n, 1), dtype=np.float64)
        m = int(self._lib.oryx_speed_aggregate(self._h, int(bool(implicit)), _ptr(u), _ptr(i),
                                               _ptr(v)))
        return u[:m], i[:m], v[:m]

    def new_keys(self, which: int) -> Tuple[np.ndarray, np.ndarray]:
        """(blob, ends) of the batch's user (0) / item (1) keys the stores lack."""
        cnt = self.counts()[1 + which]
        ends = np.empty(cnt, dtype=np.int64)
        cap = 16 * cnt + 64
        while True:
            out = np.empty(cap, dtype=np.uint8)
            used = self._lib.oryx_speed_new_keys(self._h, int(which), _ptr(out), cap, _ptr(ends))
            if used >= 0:
                return out[:used], ends
            cap = -used

    def assemble(self, lo: int, hi: int, xrows, yrows, vx: np.ndarray, vy: np.ndarray,
                 with_known: bool):
        """UP messages of the aggregated pairs [lo, hi) (``xrows`` / ``yrows``: RowText of
        every pair's updated rows) as one :class:`~oryx_amd.api.MessageBlock`."""
        from .api import MessageBlock
        n = int(hi) - int(lo)
        if n <= 0:
            return MessageBlock(b"", np.zeros(0, dtype=np.int64))
        lo = int(lo)
        vx, vy, xe, ye, xptr, yptr = _row_args(xrows, yrows, vx, vy, lo, int(hi))
        cap = int(xe[-1]) + int(ye[-1]) + n * 256
        ends = np.empty(2 * n, dtype=np.int64)
        n_msgs = ctypes.c_longlong(0)
        while True:
            out = _host_buffer(cap)
            used = self._lib.oryx_speed_assemble(
                self._h, lo, int(hi), xptr, _ptr(xe), yptr, _ptr(ye), _ptr(vx), _ptr(vy),
                int(bool(with_known)), _ptr(out), cap, _ptr(ends), ctypes.byref(n_msgs))
            if used >= 0:
                break
            cap = -used + 1
        return MessageBlock(out[:used], ends[:n_msgs.value].copy())


    def deferred(self, lo: int, hi: int, xrows, yrows, vx: np.ndarray, vy: np.ndarray,
                 with_known: bool) -> "DeferredUpBlock":
        """The same messages as :meth:`assemble`, not yet formatted: a block that the native
        log formats straight into its segment when appended (:meth:`DeferredUpBlock.
        append_to`), or into a buffer on first access otherwise.  Valid until the next
        :meth:`parse`."""
        return DeferredUpBlock(self, int(lo), int(hi), xrows, yrows, vx, vy, with_known)


def _row_args(xrows, yrows, vx, vy, lo, hi):
    vx = np.ascontiguousarray(vx[lo:hi], dtype=np.uint8)
    vy = np.ascontiguousarray(vy[lo:hi], dtype=np.uint8)
    xb = int(xrows.ends[lo - 1]) if lo else 0
    yb = int(yrows.ends[lo - 1]) if lo else 0
    xe = np.ascontiguousarray(xrows.ends[lo:hi] - xb, dtype=np.int64)
    ye = np.ascontiguousarray(yrows.ends[lo:hi] - yb, dtype=np.int64)
    xptr = ctypes.c_void_p(_buf_ptr(xrows.blob).value + xb)
    yptr = ctypes.c_void_p(_buf_ptr(yrows.blob).value + yb)
    return vx, vy, xe, ye, xptr, yptr


from .api import MessageBlock as _MessageBlock  # noqa: E402


class DeferredUpBlock(_MessageBlock):
    """A speed-layer micro-batch's UP messages (``SpeedBatch.deferred``) held as the parsed
    batch plus the GPU-formatted row text: appended to a native log topic it is formatted by
    the log's writer threads straight into the segment, CRCs included
    (``oryx_speed_append`` -> ``oryx_log_append_fill``), so the row bytes are copied once
    after the GPU's; any other use materialises the ordinary :class:`MessageBlock` buffer."""

    __slots__ = ("_sb", "_gen", "_lo", "_hi", "_rows", "_with_known", "_n", "_block")

    def __init__(self, sb: SpeedBatch, lo: int, hi: int, xrows, yrows, vx, vy,
                 with_known: bool):
        self._sb, self._gen, self._lo, self._hi = sb, sb._gen, lo, hi
        self._rows = (xrows, yrows, vx, vy)
        self._with_known = bool(with_known)
        self._n = int(np.count_nonzero(vx[lo:hi])) + int(np.count_nonzero(vy[lo:hi])) \
            if hi > lo else 0
        self._block = None
        self._cache = None

    def _check(self):
        if self._sb._gen != self._gen:
            raise RuntimeError("deferred UP block used after its speed batch was re-parsed")

    def materialize(self) -> _MessageBlock:
        if self._block is None:
            self._check()
            xrows, yrows, vx, vy = self._rows
            self._block = self._sb.assemble(self._lo, self._hi, xrows, yrows, vx, vy,
                                            self._with_known)
        return self._block

    buf = property(lambda self: self.materialize().buf)
    ends = property(lambda self: self.materialize().ends)
    sep = property(lambda self: 1)

    def __len__(self) -> int:
        return self._n

    def append_to(self, handle, partition: int = -1, timestamp_ms: int = -1,
                  fsync: bool = False) -> int:
        """Append as key-``UP`` records to the native topic ``handle``; the native result
        (last offset, -1 error, -2 a message over the topic's maximum, nothing written)."""
        if self._n == 0:
            return -1
        self._check()
        sb = self._sb
        xrows, yrows, vx, vy = self._rows
        vx, vy, xe, ye, xptr, yptr = _row_args(xrows, yrows, vx, vy, self._lo, self._hi)
        n_msgs = ctypes.c_longlong(0)
        return int(sb._lib.oryx_speed_append(
            sb._h, handle, int(partition), self._lo, self._hi, xptr, _ptr(xe), yptr, _ptr(ye),
            _ptr(vx), _ptr(vy), int(self._with_known), int(timestamp_ms), int(bool(fsync)),
            ctypes.byref(n_msgs)))


def format_leaf_updates(trees, id_blob, id_ends, idx, counts, nc: int, means=None):
    """RDF speed-layer update messages as a :class:`~oryx_amd.api.MessageBlock` (native):
    classification (``nc`` > 0, ``counts`` [n, nc]) ``[tree,ID,{"c":count,...}]`` over the
    nonzero classes, regression (``nc`` == 0, ``means`` / ``counts`` [n])
    ``[tree,ID,mean,count]``; ``ID`` = entry ``idx[j]`` of the pre-quoted JSON ID blob."""
    from .api import MessageBlock
    trees = np.ascontiguousarray(trees, dtype=np.int64)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    id_ends = np.ascontiguousarray(id_ends, dtype=np.int64)
    n = len(trees)
    if n == 0:
        return MessageBlock(b"", np.zeros(0, dtype=np.int64))
    mp = None
    if means is not None:
        means = np.ascontiguousarray(means, dtype=np.float64)
        mp = _ptr(means)
    ends = np.empty(n, dtype=np.int64)
    cap = 1 << 16
    while True:
        out = np.empty(cap, dtype=np.uint8)
        used = native.runtime().oryx_format_leaf_updates(
            n, _ptr(trees), _buf_ptr(id_blob), _ptr(id_ends), _ptr(idx), _ptr(counts), int(nc),
            mp, _ptr(out), cap, _ptr(ends))
        if used >= 0:
            return MessageBlock(out[:used], ends)
        cap = -used


def f64_repr_slots(values):
    """(slots uint8 [n, 24], lens uint8 [n]): Python repr text of each double of a 1-D
    device tensor formatted on the GPU (``csrc/kernels/fmt64.hip``), or of a host array by the
    native host formatter (the reference the device output is held to)."""
    import torch
    if torch.is_tensor(values) and values.is_cuda:
        v = values.detach().to(torch.float64).contiguous().reshape(-1)
        n = v.numel()
        slots = torch.empty((max(n, 1), 24), dtype=torch.uint8, device=v.device)
        lens = torch.empty(max(n, 1), dtype=torch.uint8, device=v.device)
        native.check(native.require_kernels().oryx_format_f64_slots(
            v.data_ptr(), n, slots.data_ptr(), lens.data_ptr(), native.stream_ptr(v.device)),
            "oryx_format_f64_slots")
        # both into one pinned block, one wait
        host = torch.empty(25 * n, dtype=torch.uint8, pin_memory=True)
        host[:24 * n].copy_(slots[:n].reshape(-1), non_blocking=True)
        host[24 * n:].copy_(lens[:n], non_blocking=True)
        torch.cuda.current_stream(v.device).synchronize()
        h = host.numpy()
        return h[:24 * n].reshape(n, 24), h[24 * n:]
    v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1)
    n = len(v)
    slots = np.empty((n, 24), dtype=np.uint8)
    lens = np.empty(n, dtype=np.uint8)
    if n:
        native.runtime().oryx_format_f64_repr_host(_ptr(v), n, _ptr(slots), _ptr(lens))
    return slots, lens


def format_cluster_updates(ids, centers, counts, device_centers=None):
    """k-means speed-layer update messages ``[id,[center...],count]`` (one per row of
    ``centers`` [n, d] float64) as a :class:`~oryx_amd.api.MessageBlock`, byte-identical to
    ``text.join_json([id, [float(v) ...], count])`` (native, threaded).  ``device_centers``:
    the same values as a device tensor -- their text is then formatted on the GPU
    (:func:`f64_repr_slots`) and only assembled on the host."""
    from .api import MessageBlock
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    n = len(ids)
    if n == 0:
        return MessageBlock(b"", np.zeros(0, dtype=np.int64))
    if device_centers is not None and native.kernels_available():
        d = int(device_centers.shape[1])
        slots, lens = f64_repr_slots(device_centers)
        ends = np.empty(n, dtype=np.int64)
        cap = n * (25 * d + 48)
        out = _host_buffer(cap)
        used = native.runtime().oryx_format_cluster_updates_slots(
            _ptr(ids), _ptr(slots), _ptr(lens), _ptr(counts), n, d, _ptr(out), cap, _ptr(ends))
        if used < 0:
            raise RuntimeError("cluster update text larger than its bound")
        return MessageBlock(out[:used], ends)
    centers = np.ascontiguousarray(centers, dtype=np.float64)
    d = centers.shape[1]
    ends = np.empty(n, dtype=np.int64)
    cap = n * (52 + 25 * d)
    while True:
        # (a reused pinned block on a GPU host: a fresh 6 MB array faulted in its pages on
        # every speed-layer micro-batch)
        out = _host_buffer(cap)
        used = native.runtime().oryx_format_cluster_updates(
            _ptr(ids), _ptr(centers), _ptr(counts), n, d, _ptr(out), cap, _ptr(ends))
        if used >= 0:
            return MessageBlock(out[:used], ends)
        cap = -used


def parse_up_batch(messages: Sequence[str], k: int, known_dict: Optional["IdDict"] = None):
    """Bulk-parse ALS ``UP`` messages ``["X"|"Y", id, [k floats], [known ids]?]``.

    Returns (kinds uint8 [n] -- 0 X, 1 Y, 2 unparseable --, ids list, vectors fp32 [n, k],
    known lists per message (None when absent)).  One native pass (threaded) instead of a
    JSON parse per message (the serving / speed model load of millions of rows).
    """
    n = len(messages)
    enc = [m.encode("utf-8") for m in messages]
    blob = b"".join(enc)
    ends = np.cumsum(np.fromiter((len(b) for b in enc), dtype=np.int64, count=n))
    kinds = np.empty(n, dtype=np.uint8)
    vecs = np.empty((n, k), dtype=np.float32)
    id_ends = np.empty(n, dtype=np.int64)
    kcnt = np.empty(n, dtype=np.int64)
    vp = ctypes.c_void_p
    native.runtime().oryx_parse_up_batch(blob, ends.ctypes.data_as(vp), n, int(k),
                                         kinds.ctypes.data_as(vp), vecs.ctypes.data_as(vp),
                                         id_ends.ctypes.data_as(vp), kcnt.ctypes.data_as(vp))
    if known_dict is not None:
        ids, known = _up_ids_codes(id_ends, kcnt, known_dict)
    else:
        ids, known = _up_texts(id_ends, kcnt, len(blob))
    return kinds, ids, vecs, known


def _known_mode(model):
    """What an UP parse should do with known items for ``model``: its item dictionary
    (codes), False (the model keeps none: skip them) or None (string lists)."""
    kd = getattr(model, "known_items_dict", None)
    if kd is not None:
        return kd
    return None if hasattr(model, "add_known_items") else False


def content_digest(buf, off: int, nbytes: int) -> bytes:
    """24-byte identity of ``buf[off:off + nbytes]`` (numpy uint8 array or bytes): the
    parallel native digest (``oryx_digest128``) plus the length."""
    out = np.empty(2, dtype=np.uint64)
    if isinstance(buf, np.ndarray):
        base = buf.ctypes.data
    else:
        base = ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value
    native.runtime().oryx_digest128(ctypes.c_void_p(base + int(off)), int(nbytes),
                                    out.ctypes.data_as(ctypes.c_void_p))
    return out.tobytes() + int(nbytes).to_bytes(8, "little")


PARSE_STATS = {"native_s": 0.0}


def parse_up_records(raw_ptr: int, used: int, nrec: int, k: int, max_n: int,
                     known_dict: Optional["IdDict"] = None, frames: bool = False):
    """The leading run of ``UP`` records of a raw log poll buffer (see
    ``oryx_parse_up_records``): returns (count, consumed bytes, kinds, ids, vectors, known) --
    count 0 when the first record is not a parseable ``UP``.  With ``known_dict`` the known
    items come back as :class:`KnownCodes` of that dictionary instead of string lists."""
    m = min(nrec, max_n)
    kinds = np.empty(m, dtype=np.uint8)
    vecs = np.empty((m, k), dtype=np.float32)
    id_ends = np.empty(m, dtype=np.int64)
    kcnt = np.empty(m, dtype=np.int64)
    consumed = ctypes.c_longlong(0)
    vp = ctypes.c_void_p
    fn = native.runtime().oryx_parse_up_frames if frames else \
        native.runtime().oryx_parse_up_records
    t0 = time.perf_counter()
    got = fn(
        ctypes.c_void_p(raw_ptr), int(used), int(nrec), int(k), int(max_n),
        kinds.ctypes.data_as(vp), vecs.ctypes.data_as(vp), id_ends.ctypes.data_as(vp),
        kcnt.ctypes.data_as(vp), ctypes.byref(consumed))
    PARSE_STATS["native_s"] += time.perf_counter() - t0
    if got <= 0:
        return 0, 0, None, None, None, None
    if known_dict is not None:
        ids, known = _up_ids_codes(id_ends[:got], kcnt[:got], known_dict)
    else:
        ids, known = _up_texts(id_ends[:got], kcnt[:got], int(used))
    return got, consumed.value, kinds[:got], ids, vecs[:got], known


def parse_feature_lines(data: bytes, k: int):
    """(ids, fp32 [n, k]) of factor part-file lines ``[id,[k floats]]`` (native, threaded),
    or None when a line does not parse that way."""
    if isinstance(data, np.ndarray):
        n_max = int(np.count_nonzero(data == 10)) + 1
    else:
        n_max = data.count(b"\n") + 1
    vecs = np.empty((n_max, k), dtype=np.float32)
    id_ends = np.empty(n_max, dtype=np.int64)
    vp = ctypes.c_void_p
    n = native.runtime().oryx_parse_feature_lines(_buf_ptr(data), len(data), int(k), n_max,
                                                  vecs.ctypes.data_as(vp),
                                                  id_ends.ctypes.data_as(vp))
    if n < 0:
        return None
    ids, _ = _up_texts(id_ends[:n], np.full(n, -1, dtype=np.int64), 16)
    return ids, vecs[:n]


class KnownCodes:
    """Known-item lists of parsed ``UP`` rows as codes of an :class:`IdDict`: row j's items
    are ``codes[offs[j]:offs[j + 1]]``; ``has[j]`` is False for a row without a list."""

    __slots__ = ("codes", "offs", "has")

    def __init__(self, codes: np.ndarray, counts: np.ndarray):
        self.codes = codes
        c = np.maximum(np.asarray(counts, dtype=np.int64), 0)
        self.offs = np.zeros(len(c) + 1, dtype=np.int64)
        np.cumsum(c, out=self.offs[1:])
        self.has = np.asarray(counts) >= 0

    def __len__(self) -> int:
        return len(self.has)

    def row(self, j: int) -> Optional[np.ndarray]:
        return self.codes[self.offs[j]:self.offs[j + 1]] if self.has[j] else None


def _up_ids_codes(id_ends: np.ndarray, kcnt: np.ndarray, known_dict: "IdDict"):
    """IDs (strings) and known items (:class:`KnownCodes`) of the last native UP parse."""
    n = len(id_ends)
    ids_cap = max(1, int(id_ends[-1]) if n else 0)
    ib = np.empty(ids_cap, dtype=np.uint8)
    lib = native.runtime()
    if lib.oryx_up_ids(ib.ctypes.data, ids_cap) < 0:
        raise RuntimeError("UP batch ids exceed their buffer")
    raw = ib[:int(id_ends[-1]) if n else 0].tobytes()
    starts = np.r_[0, id_ends[:-1]].tolist() if n else []
    if raw.isascii():
        text = raw.decode("ascii")
        ids = [text[a:b] for a, b in zip(starts, id_ends.tolist())]
    else:
        ids = [raw[a:b].decode("utf-8") for a, b in zip(starts, id_ends.tolist())]
    if known_dict is False:
        return ids, None
    total = int(np.maximum(kcnt, 0).sum()) if n else 0
    codes = np.empty(max(1, total), dtype=np.int64)
    got = lib.oryx_up_known_codes(known_dict.handle, codes.ctypes.data, total)
    if got != total:
        raise RuntimeError("UP known items: %d parsed, %d counted" % (got, total))
    return ids, KnownCodes(codes[:total].astype(np.int32), kcnt)


def _up_texts(id_ends: np.ndarray, kcnt: np.ndarray, bound: int):
    """IDs and known-item lists of the last native UP parse (thread-local texts)."""
    n = len(id_ends)
    ids_cap = max(1, int(id_ends[-1]) if n else 0)
    known_cap = max(16, bound)
    ib = np.empty(ids_cap, dtype=np.uint8)
    kb = np.empty(known_cap, dtype=np.uint8)
    vp = ctypes.c_void_p
    got = native.runtime().oryx_up_texts(ib.ctypes.data_as(vp), ids_cap,
                                         kb.ctypes.data_as(vp), known_cap)
    if got < 0:
        raise RuntimeError("UP batch texts exceed their buffers")
    raw = ib[:int(id_ends[-1]) if n else 0].tobytes()
    starts = np.r_[0, id_ends[:-1]].tolist() if n else []
    if raw.isascii():
        text = raw.decode("ascii")
        ids = [text[a:b] for a, b in zip(starts, id_ends.tolist())]
    else:
        ids = [raw[a:b].decode("utf-8") for a, b in zip(starts, id_ends.tolist())]
    known: List[Optional[List[str]]] = [None] * n
    pos_c = kcnt > 0
    total = int(kcnt[pos_c].sum()) if n else 0
    if total:
        flat = [x.decode("utf-8") for x in kb.tobytes().split(b"\0", total)[:total]]
        pos = 0
        for j, c in enumerate(kcnt.tolist()):
            if c > 0:
                known[j] = flat[pos:pos + c]
                pos += c
            elif c == 0:
                known[j] = []
    else:
        for j in np.nonzero(kcnt == 0)[0].tolist():
            known[j] = []
    return ids, known


def format_als_updates(users: IdDict, items: IdDict, u: np.ndarray, i: np.ndarray,
                       nx: np.ndarray, ny: np.ndarray, vx: np.ndarray, vy: np.ndarray,
                       with_known: bool) -> List[str]:
    """The speed layer's ``UP`` messages for folded-in events (see ``oryx_ingest.cpp``)."""
    n = len(u)
    if n == 0:
        return []
    k = int(nx.shape[1])
    u = np.ascontiguousarray(u, dtype=np.int64)
    i = np.ascontiguousarray(i, dtype=np.int64)
    nx = np.ascontiguousarray(nx, dtype=np.float32)
    ny = np.ascontiguousarray(ny, dtype=np.float32)
    vx = np.ascontiguousarray(vx, dtype=np.uint8)
    vy = np.ascontiguousarray(vy, dtype=np.uint8)
    vp = ctypes.c_void_p
    lib = native.runtime()
    return _run_message_writer(n * (k * 20 + 256), lambda out, cap: lib.oryx_format_als_updates(
        users.handle, items.handle, u.ctypes.data_as(vp), i.ctypes.data_as(vp),
        nx.ctypes.data_as(vp), ny.ctypes.data_as(vp), vx.ctypes.data_as(vp),
        vy.ctypes.data_as(vp), n, k, int(bool(with_known)), out, cap))


def assemble_als_updates(users: IdDict, items: IdDict, u: np.ndarray, i: np.ndarray,
                         xrows, yrows, vx: np.ndarray, vy: np.ndarray, with_known: bool,
                         lo: int = 0, hi: Optional[int] = None):
    """As :func:`format_als_updates` with the factor rows already formatted
    (:class:`~oryx_amd.ops.textfmt.RowText`, e.g. by the GPU formatter).  Returns a
    :class:`~oryx_amd.api.MessageBlock` (one buffer; producers append it natively).
    ``lo`` / ``hi``: only the events [lo, hi) (a chunk of a pipelined publish)."""
    from .api import MessageBlock
    hi = len(u) if hi is None else int(hi)
    lo = int(lo)
    n = hi - lo
    if n <= 0:
        return MessageBlock(b"", np.zeros(0, dtype=np.int64))
    u = np.ascontiguousarray(u[lo:hi], dtype=np.int64)
    i = np.ascontiguousarray(i[lo:hi], dtype=np.int64)
    vx = np.ascontiguousarray(vx[lo:hi], dtype=np.uint8)
    vy = np.ascontiguousarray(vy[lo:hi], dtype=np.uint8)
    xb = int(xrows.ends[lo - 1]) if lo else 0
    yb = int(yrows.ends[lo - 1]) if lo else 0
    xe = np.ascontiguousarray(xrows.ends[lo:hi] - xb, dtype=np.int64)
    ye = np.ascontiguousarray(yrows.ends[lo:hi] - yb, dtype=np.int64)
    vp = ctypes.c_void_p
    lib = native.runtime()
    cap = int(xe[-1]) + int(ye[-1]) + n * 256
    ends = np.empty(2 * n, dtype=np.int64)
    n_msgs = ctypes.c_longlong(0)
    xptr = vp(_buf_ptr(xrows.blob).value + xb)
    yptr = vp(_buf_ptr(yrows.blob).value + yb)
    while True:
        out = _host_buffer(cap)
        used = lib.oryx_assemble_als_updates(
            users.handle, items.handle, u.ctypes.data_as(vp), i.ctypes.data_as(vp),
            xptr, xe.ctypes.data_as(vp), yptr, ye.ctypes.data_as(vp), vx.ctypes.data_as(vp),
            vy.ctypes.data_as(vp), n, int(bool(with_known)), out.ctypes.data_as(vp), cap,
            ends.ctypes.data_as(vp), ctypes.byref(n_msgs))
        if used >= 0:
            break
        cap = -used + 1
    return MessageBlock(out[:used], ends[:n_msgs.value].copy())


def assemble_row_messages(kind: str, ids, rows, known=None, kidx=None):
    """Model rows as newline-separated JSON lines in one :class:`~oryx_amd.api.MessageBlock`
    (native, threaded): ``kind`` "Y" / "X" -> ``["Y",id,row]`` update messages (with
    ``known`` spans and ``kidx``: ``["X",id,row,known[kidx[e]]]``, rows with ``kidx < 0``
    skipped), "" -> ``[id,row]`` part-file lines.  ``ids``: list of str or (blob, ends);
    ``rows`` / ``known``: :class:`~oryx_amd.ops.textfmt.RowText`."""
    from .api import MessageBlock
    id_blob, id_ends = ids if isinstance(ids, tuple) else _ids_blob(ids)
    n = len(id_ends)
    if n != len(rows):
        raise ValueError("%d ids vs %d rows" % (n, len(rows)))
    if n == 0:
        return MessageBlock(b"", np.zeros(0, dtype=np.int64))
    vp = ctypes.c_void_p
    id_ends = np.ascontiguousarray(id_ends, dtype=np.int64)
    re = np.ascontiguousarray(rows.ends, dtype=np.int64)
    if known is not None:
        ke = np.ascontiguousarray(known.ends, dtype=np.int64)
        kidx = np.ascontiguousarray(kidx, dtype=np.int64)
        if len(kidx) != n or (len(kidx) and int(kidx.max()) >= len(ke)):
            raise ValueError("known index out of range")
        kargs = (_buf_ptr(known.blob), ke.ctypes.data_as(vp), kidx.ctypes.data_as(vp))
        extra = int(ke[-1]) if len(ke) else 0
    else:
        kargs = (None, None, None)
        extra = 0
    lib = native.runtime()
    cap = len(id_blob) * 2 + len(rows.blob) + extra + n * 16
    ends = np.empty(n, dtype=np.int64)
    n_msgs = ctypes.c_longlong(0)
    code = ord(kind) if kind else 0
    while True:
        out = _host_buffer(cap)
        used = lib.oryx_assemble_row_messages(
            code, _buf_ptr(id_blob), id_ends.ctypes.data_as(vp), _buf_ptr(rows.blob),
            re.ctypes.data_as(vp), n, *kargs, out.ctypes.data_as(vp), cap,
            ends.ctypes.data_as(vp), ctypes.byref(n_msgs))
        if used >= 0:
            break
        cap = -used + 1
    return MessageBlock(out[:used], ends[:n_msgs.value].copy())


def known_items_text(items: IdDict, uu: np.ndarray, ii: np.ndarray, n_users: int):
    """Per user code, the JSON array of its items' quoted names (``(uu, ii)`` code pairs
    sorted by user, items in the order given); a :class:`~oryx_amd.ops.textfmt.RowText`."""
    from .ops.textfmt import RowText
    uu = np.ascontiguousarray(uu, dtype=np.int64)
    ii = np.ascontiguousarray(ii, dtype=np.int64)
    if len(uu) and (int(ii.min()) < 0 or int(ii.max()) >= len(items) or
                    int(uu.min()) < 0 or int(uu.max()) >= n_users):
        raise ValueError("code out of range")
    vp = ctypes.c_void_p
    lib = native.runtime()
    ends = np.empty(n_users, dtype=np.int64)
    cap = 2 * n_users + 16 * len(uu) + 64
    while True:
        out = np.empty(cap, dtype=np.uint8)
        used = lib.oryx_known_items_text(items.handle, uu.ctypes.data_as(vp),
                                         ii.ctypes.data_as(vp), len(uu), n_users,
                                         out.ctypes.data_as(vp), cap, ends.ctypes.data_as(vp))
        if used >= 0:
            break
        cap = -used + 1
    return RowText(out[:used], ends)


def write_gzip(path: str, buf, level: int = 1) -> None:
    """``buf`` (bytes / uint8 array) to ``path`` as a multi-member gzip file, compressed on
    the native threads."""
    n = len(buf)
    rc = native.runtime().oryx_write_gzip(path.encode(), _buf_ptr(buf) if n else None, n,
                                          int(level))
    if rc != 0:
        raise OSError("cannot write %s (%s)" % (path, "zlib" if rc == -2 else "file error"))


def read_gzip(raw: bytes):
    """Decompressed contents of a gzip file (bytes, or a uint8 array for files written by
    :func:`write_gzip`, whose indexed members are inflated natively in parallel and
    CRC-checked); any other gzip goes through :mod:`gzip`."""
    lib = native.runtime()
    size = lib.oryx_gzip_indexed_size(raw, len(raw))
    if size < 0:
        import gzip
        return gzip.decompress(raw)
    out = hostbuf.empty(max(1, size))
    got = lib.oryx_gzip_indexed_inflate(raw, len(raw), out.ctypes.data_as(ctypes.c_void_p),
                                        size)
    if got != size:
        raise OSError("corrupt gzip member (CRC / size mismatch)")
    return out[:size]


def _host_buffer(n: int) -> np.ndarray:
    """A uint8 host buffer; on a GPU host from torch's caching pinned allocator, whose blocks
    are reused (already-faulted pages) once the previous holder is gone."""
    try:
        import torch
        if torch.cuda.is_available():
            return torch.empty(int(n), dtype=torch.uint8, pin_memory=True).numpy()
    except RuntimeError:
        pass
    return np.empty(int(n), dtype=np.uint8)


def _buf_ptr(b) -> ctypes.c_void_p:
    """Address of a bytes object or uint8 numpy array (kept alive by the caller)."""
    if isinstance(b, np.ndarray):
        return ctypes.c_void_p(b.ctypes.data)
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)


def _run_message_writer(cap: int, call) -> List[str]:
    """Runs a native '\\n'-separated message writer (retrying once with the size it asks
    for) and splits its output."""
    while True:
        out = np.empty(cap, dtype=np.uint8)
        used = call(out.ctypes.data_as(ctypes.c_void_p), cap)
        if used >= 0:
            break
        cap = -used + 1
    if used == 0:
        return []
    msgs = out[:used].tobytes().decode("ascii").split("\n")
    msgs.pop()
    return msgs


def format_float_rows_blob(mat: np.ndarray):
    """JSON array text of each row (shortest float32 round-trip digits, Jackson-like) as one
    :class:`~oryx_amd.ops.textfmt.RowText` (native, threaded)."""
    from .ops.textfmt import RowText
    mat = np.ascontiguousarray(mat, dtype=np.float32)
    n, k = mat.shape
    if n == 0:
        return RowText(b"", np.zeros(0, dtype=np.int64))
    cap = n * (2 + k * 18) + 16
    out = np.empty(cap, dtype=np.uint8)
    ends = np.empty(n, dtype=np.int64)
    vp = ctypes.c_void_p
    used = native.runtime().oryx_format_float_rows(mat.ctypes.data_as(vp), n, k, k,
                                                   out.ctypes.data_as(vp), cap,
                                                   ends.ctypes.data_as(vp))
    if used < 0:
        raise RuntimeError("format buffer too small")
    return RowText(out[:used].tobytes(), ends)


def format_float_rows(mat: np.ndarray) -> List[str]:
    """JSON array text of each row, shortest float32 round-trip digits (Jackson-like)."""
    mat = np.asarray(mat, dtype=np.float32)
    if mat.shape[0] == 0:
        return []
    return format_float_rows_blob(mat).rows()