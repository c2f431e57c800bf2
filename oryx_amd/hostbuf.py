"""Large host byte buffers whose memory is returned off the caller's thread
(``csrc/runtime/oryx_hostbuf.cpp``).

The batch layer's text -- a generation's drain, its train / test selections, concatenations
of new and past data -- lives in uint8 arrays of up to tens of GB.  Dropping the last reference
to a numpy-allocated one unmaps it right there, with the GIL held (~65 ms per GB with 4 KB
pages); the reference's Spark executors leave that to the JVM's background collector
(``[lambda]/batch/BatchUpdateFunction.java:103-130``).  :func:`empty` returns an array over a
native mapping instead; when the array and every view of it are gone, a finalizer queues the
unmap on the runtime's reaper thread and returns.

``ORYX_HOSTBUF=0`` turns this off (plain ``np.empty``); ``ORYX_HOSTBUF_MIN_MB`` (default 64)
is the smallest buffer that takes the native path.
"""

from __future__ import annotations

import ctypes
import os
import weakref
from typing import Optional

import numpy as np

from . import native

__all__ = ["empty", "read_text_file", "stats", "quiesce"]

_MIN = int(float(os.environ.get("ORYX_HOSTBUF_MIN_MB", "64")) * (1 << 20))
_ON = os.environ.get("ORYX_HOSTBUF", "1") != "0"


def empty(n: int, min_bytes: Optional[int] = None) -> np.ndarray:
    """An uninitialised (in fact zero-filled) uint8 array of ``n`` bytes (native from
    ``min_bytes``, default ``ORYX_HOSTBUF_MIN_MB``)."""
    n = int(n)
    if not _ON or n < (_MIN if min_bytes is None else min(_MIN, int(min_bytes))):
        return np.empty(n, dtype=np.uint8)
    lib = native.runtime()
    p = lib.oryx_hostbuf_alloc(n)
    if not p:
        return np.empty(n, dtype=np.uint8)
    raw = (ctypes.c_uint8 * n).from_address(p)
    # the array's base chain (memoryview -> ctypes array) keeps ``raw`` alive as long as any
    # view of the buffer exists; the finalizer runs once the last one is gone
    fin = weakref.finalize(raw, lib.oryx_hostbuf_free, p, n)
    fin.atexit = False
    return np.frombuffer(raw, dtype=np.uint8)


def prefault(buf: np.ndarray, threads: int = 16) -> None:
    """Faults ``buf``'s pages in from ``threads`` native threads (before concurrent writers)."""
    if len(buf):
        native.runtime().oryx_hostbuf_prefault(buf.ctypes.data, len(buf),
                                               min(threads, os.cpu_count() or 1))


def read_text_file(path: str, threads: int = 16) -> np.ndarray:
    """The bytes of a text file as a uint8 array ending with a newline (one is appended when
    the file lacks it), read by ``threads`` concurrent native preads into an :func:`empty`
    buffer."""
    size = os.path.getsize(path)
    out = empty(size + 1)
    got = int(native.runtime().oryx_read_file_parallel(
        os.fsencode(path), out.ctypes.data, size, max(1, min(threads, os.cpu_count() or 1))))
    if got < 0:
        raise OSError(-got, os.strerror(-got), path)
    if got == 0:
        return out[:0]
    if out[got - 1] != 10:
        out[got] = 10
        got += 1
    return out[:got]


def stats() -> dict:
    """Bytes queued for unmapping and bytes unmapped by the reaper so far."""
    out = (ctypes.c_longlong * 2)()
    native.runtime().oryx_hostbuf_stats(out)
    return {"pending_bytes": int(out[0]), "freed_bytes": int(out[1])}


def quiesce(timeout_s: float = -1.0) -> int:
    """Waits for queued unmaps (tests, memory-tight phases); returns the bytes still pending."""
    ms = -1 if timeout_s < 0 else int(timeout_s * 1e3)
    return int(native.runtime().oryx_hostbuf_quiesce(ms))
