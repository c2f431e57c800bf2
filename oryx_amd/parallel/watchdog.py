"""Rank-health watchdog for collectives and long device loops.

The reference delegates failure handling to Spark task retries; a multi-GPU job here is one
process per GPU, and a rank that dies or wedges leaves its peers blocked inside an RCCL
collective (or a stream sync) forever.  Two mechanisms turn that into a fast, visible failure:

* :func:`guard` -- a deadline around one blocking region (a collective plus the sync that
  waits for it, a checkpoint write); and
* :func:`heartbeat` -- the training loops (ALS iterations, k-means Lloyd steps, RDF levels)
  report progress; silence for longer than the timeout means a hang somewhere below.

When a deadline passes, the watchdog logs every thread's stack (``faulthandler``), records a
tracing event, and runs the expiry action: by default it terminates the process with exit
code 86, which makes ``torch.distributed.run`` (``oryx-run batch --gpus N`` launches with
``--max-restarts``) tear down and restart the whole group; the restarted ALS trainer resumes
from its last factor checkpoint.  Timeout: ``oryx.gpu.collective-timeout-sec`` or the
``ORYX_WATCHDOG_TIMEOUT`` environment variable; 0 disables the watchdog.
"""

from __future__ import annotations

import contextlib
import faulthandler
import logging
import os
import sys
import threading
import time
from typing import Callable, Dict, Optional

from .. import tracing

__all__ = ["Watchdog", "get", "configure", "guard", "heartbeat", "EXIT_CODE"]

log = logging.getLogger(__name__)

EXIT_CODE = 86


def _default_expire(what: str) -> None:
    os._exit(EXIT_CODE)


class Watchdog:
    def __init__(self, timeout_s: float, on_expire: Optional[Callable[[str], None]] = None,
                 poll_s: float = 0.5):
        self.timeout_s = float(timeout_s)
        self.on_expire = on_expire or _default_expire
        self.poll_s = poll_s
        self._lock = threading.Lock()
        self._deadlines: Dict[int, tuple] = {}
        self._next = 0
        self._beat: Optional[tuple] = None        # (name, last time)
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.expired: Optional[str] = None

    @property
    def enabled(self) -> bool:
        return self.timeout_s > 0

    def _start(self) -> None:
        if self._thread is None or not self._thread.is_alive():
            self._stop.clear()
            self._thread = threading.Thread(target=self._run, name="oryx-watchdog",
                                            daemon=True)
            self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    @contextlib.contextmanager
    def guard(self, name: str, timeout_s: Optional[float] = None):
        if not self.enabled:
            yield
            return
        t = self.timeout_s if timeout_s is None else float(timeout_s)
        with self._lock:
            key = self._next
            self._next += 1
            self._deadlines[key] = (name, time.monotonic() + t)
        self._start()
        try:
            yield
        finally:
            with self._lock:
                self._deadlines.pop(key, None)

    def heartbeat(self, name: str) -> None:
        if not self.enabled:
            return
        with self._lock:
            self._beat = (name, time.monotonic())
        self._start()

    def end_heartbeats(self) -> None:
        with self._lock:
            self._beat = None

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            now = time.monotonic()
            what = None
            with self._lock:
                for name, deadline in self._deadlines.values():
                    if now > deadline:
                        what = "guard '%s' exceeded %.1fs" % (name, self.timeout_s)
                        break
                if what is None and self._beat is not None:
                    name, last = self._beat
                    if now - last > self.timeout_s:
                        what = "no heartbeat since '%s' for %.1fs" % (name, now - last)
            if what is not None:
                self._fire(what)
                return

    def _fire(self, what: str) -> None:
        self.expired = what
        rank = os.environ.get("RANK", "0")
        log.error("Watchdog expired on rank %s: %s; thread stacks follow", rank, what)
        try:
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        except Exception:  # pragma: no cover - stderr may be closed
            pass
        tracing.record({"event": "watchdog_expired", "rank": rank, "what": what})
        self.on_expire(what)


_global: Optional[Watchdog] = None


def get() -> Watchdog:
    global _global
    if _global is None:
        _global = Watchdog(float(os.environ.get("ORYX_WATCHDOG_TIMEOUT", "0") or 0))
    return _global


def configure(timeout_s: float, on_expire: Optional[Callable[[str], None]] = None
              ) -> Watchdog:
    """Replace the process watchdog (a config value overrides the environment)."""
    global _global
    if _global is not None:
        _global.stop()
    _global = Watchdog(timeout_s, on_expire)
    return _global


def guard(name: str, timeout_s: Optional[float] = None):
    return get().guard(name, timeout_s)


def heartbeat(name: str) -> None:
    get().heartbeat(name)
