"""Tracing: roctx ranges around phases, kernels and collectives, plus JSON timing records.

The reference has no tracing subsystem (only the Spark UI and ad-hoc
benchmark timing).  Here every batch phase, kernel launch site and collective is bracketed by
a named range that ``rocprofv3 --marker-trace`` shows on the timeline (``torch.cuda.nvtx``
maps onto roctx on ROCm builds), and :class:`Timer` records wall-clock spans into
per-interval JSON records (ratings/s, iteration ms, ...).
"""

from __future__ import annotations

import contextlib
import json
import logging
import os
import threading
import time
from typing import Dict, List, Optional

__all__ = ["range", "enabled", "Timer", "record", "records", "dump_records"]

log = logging.getLogger(__name__)

_enabled = os.environ.get("ORYX_TRACE", "0") not in ("", "0", "false")
_records: List[dict] = []
_lock = threading.Lock()


def enabled() -> bool:
    return _enabled


def set_enabled(flag: bool) -> None:
    global _enabled
    _enabled = bool(flag)


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx API name
    if not _enabled:
        yield
        return
    pushed = False
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:
        pushed = False
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if pushed:
            import torch
            torch.cuda.nvtx.range_pop()
        record({"range": name, "ms": (time.perf_counter() - t0) * 1e3})


class Timer:
    """``with Timer('phase') as t: ...`` -> ``t.ms``; also records when tracing is enabled."""

    def __init__(self, name: str, sync_device=None):
        self.name = name
        self.sync_device = sync_device
        self.ms = 0.0

    def __enter__(self):
        self._sync()
        self.t0 = time.perf_counter()
        return self

    def _sync(self):
        if self.sync_device is not None:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize(self.sync_device)

    def __exit__(self, *exc):
        self._sync()
        self.ms = (time.perf_counter() - self.t0) * 1e3
        if _enabled:
            record({"timer": self.name, "ms": self.ms})
        return False


def record(rec: dict) -> None:
    with _lock:
        _records.append(dict(rec, ts=time.time()))
        if len(_records) > 100000:
            del _records[:50000]


def records() -> List[dict]:
    with _lock:
        return list(_records)


def dump_records(path: str) -> None:
    with open(path, "w") as f:
        for r in records():
            f.write(json.dumps(r) + "\n")
