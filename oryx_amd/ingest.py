"""Native ingest helpers: dictionary-encoded rating parsing and fast JSON row formatting.

Thin bindings over ``csrc/runtime/oryx_ingest.cpp`` (see its header for the reference call
sites it replaces).
"""

from __future__ import annotations

import ctypes
import json
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import native

__all__ = ["IdDict", "parse_ratings", "format_float_rows"]


class IdDict:
    """Collision-free string -> dense int64 dictionary (insertion order)."""

    def __init__(self):
        self._lib = native.runtime()
        self._h = self._lib.oryx_dict_new()
        self._keys_cache: List[str] = []

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

    def encode(self, keys: Sequence[str]) -> np.ndarray:
        buf = b"\0".join(k.encode("utf-8") for k in keys) + b"\0"
        out = np.empty(len(keys), dtype=np.int64)
        self._lib.oryx_dict_encode(self._h, buf, len(buf), len(keys),
                                   out.ctypes.data_as(ctypes.c_void_p))
        return out

    def get(self, key: str) -> int:
        b = key.encode("utf-8")
        return int(self._lib.oryx_dict_get(self._h, b, len(b)))

    def keys(self) -> List[str]:
        n = len(self)
        if len(self._keys_cache) < n:
            buf = ctypes.create_string_buffer(4096)
            for code in range(len(self._keys_cache), n):
                ln = self._lib.oryx_dict_key(self._h, code, buf, 4096)
                if ln > 4096:
                    big = ctypes.create_string_buffer(int(ln))
                    self._lib.oryx_dict_key(self._h, code, big, ln)
                    self._keys_cache.append(big.raw[:ln].decode("utf-8"))
                else:
                    self._keys_cache.append(buf.raw[:ln].decode("utf-8"))
        return self._keys_cache[:n]


def parse_ratings(lines, users: IdDict, items: IdDict, default_ts: int,
                  strict: bool = False) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Parse rating lines (str list or newline-joined bytes) -> (u, i, strength, ts) arrays."""
    if isinstance(lines, (bytes, bytearray)):
        data = bytes(lines)
        n_max = data.count(b"\n") + 1
    else:
        data = "\n".join(lines).encode("utf-8")
        n_max = len(lines) + 1
    u = np.empty(n_max, dtype=np.int64)
    i = np.empty(n_max, dtype=np.int64)
    s = np.empty(n_max, dtype=np.float64)
    t = np.empty(n_max, dtype=np.int64)
    vp = ctypes.c_void_p
    n = native.runtime().oryx_parse_ratings(
        data, len(data), users.handle, items.handle, u.ctypes.data_as(vp), i.ctypes.data_as(vp),
        s.ctypes.data_as(vp), t.ctypes.data_as(vp), n_max, int(default_ts), int(bool(strict)))
    if n < 0:
        raise ValueError("Bad input line %d" % (-n - 1))
    return u[:n], i[:n], s[:n], t[:n]


def format_float_rows(mat: np.ndarray) -> List[str]:
    """JSON array text of each row, shortest float32 round-trip digits (Jackson-like)."""
    mat = np.ascontiguousarray(mat, dtype=np.float32)
    n, k = mat.shape
    cap = n * (2 + k * 17) + 16
    out = ctypes.create_string_buffer(cap)
    ends = np.empty(n, dtype=np.int64)
    vp = ctypes.c_void_p
    used = native.runtime().oryx_format_float_rows(mat.ctypes.data_as(vp), n, k, k, out, cap,
                                                   ends.ctypes.data_as(vp))
    if used < 0:
        raise RuntimeError("format buffer too small")
    raw = out.raw[:used].decode("ascii")
    res = []
    start = 0
    for e in ends.tolist():
        res.append(raw[start:e])
        start = e
    return res
