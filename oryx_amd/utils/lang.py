"""Concurrency and reflection utilities.

* ``AutoLock`` / ``AutoReadWriteLock`` (``[common]/lang/AutoLock.java:39-109``,
  ``[common]/lang/AutoReadWriteLock.java:37-86``) -> context-manager locks; the RW lock is
  writer-preferring.
* ``ExecUtils.doInParallel`` / ``collectInParallel`` (``[common]/lang/ExecUtils.java:43-119``).
* ``LoggingCallable`` (``[common]/lang/LoggingCallable.java:31-86``) -> :func:`logging_callable`.
* ``ClassUtils`` (``[common]/lang/ClassUtils.java:24-133``) -> :func:`load_instance_of`, which
  also maps the reference's Java class names (``com.cloudera.oryx.app...ALSUpdate``) onto this
  framework's classes so existing deployment files keep working.
* ``OryxShutdownHook`` / ``JVMUtils.closeAtShutdown`` (``[common]/lang/OryxShutdownHook.java:32-58``)
  -> :func:`close_at_shutdown` (LIFO close at interpreter exit).
"""

from __future__ import annotations

import atexit
import concurrent.futures as cf
import importlib
import inspect
import logging
import threading
from contextlib import contextmanager
from typing import Any, Callable, Iterable, List, Optional, Sequence

__all__ = ["AutoLock", "AutoReadWriteLock", "do_in_parallel", "collect_in_parallel",
           "logging_callable", "load_class", "load_instance_of", "close_at_shutdown",
           "JAVA_CLASS_ALIASES", "class_exists", "get_used_memory"]

log = logging.getLogger(__name__)


class AutoLock:
    """A reentrant lock usable as ``with lock:``; ``auto_lock()`` mirrors the reference API."""

    def __init__(self, lock: Optional[threading.RLock] = None):
        self._lock = lock or threading.RLock()

    def __enter__(self):
        self._lock.acquire()
        return self

    def __exit__(self, *exc):
        self._lock.release()
        return False

    def auto_lock(self) -> "AutoLock":
        return self

    def acquire(self, blocking=True, timeout=-1):
        return self._lock.acquire(blocking, timeout)

    def release(self):
        self._lock.release()


class AutoReadWriteLock:
    """Writer-preferring read/write lock with ``read()`` / ``write()`` context managers."""

    def __init__(self):
        self._cond = threading.Condition(threading.Lock())
        self._readers = 0
        self._writer: Optional[int] = None
        self._writer_depth = 0
        self._waiting_writers = 0

    @contextmanager
    def read(self):
        me = threading.get_ident()
        with self._cond:
            if self._writer == me:   # write lock holders may also read
                self._writer_depth += 1
                reentrant = True
            else:
                reentrant = False
                while self._writer is not None or self._waiting_writers:
                    self._cond.wait()
                self._readers += 1
        try:
            yield self
        finally:
            with self._cond:
                if reentrant:
                    self._writer_depth -= 1
                else:
                    self._readers -= 1
                    if self._readers == 0:
                        self._cond.notify_all()

    @contextmanager
    def write(self):
        me = threading.get_ident()
        with self._cond:
            if self._writer == me:
                self._writer_depth += 1
            else:
                self._waiting_writers += 1
                while self._writer is not None or self._readers:
                    self._cond.wait()
                self._waiting_writers -= 1
                self._writer = me
                self._writer_depth = 1
        try:
            yield self
        finally:
            with self._cond:
                self._writer_depth -= 1
                if self._writer_depth == 0:
                    self._writer = None
                    self._cond.notify_all()

    # reference-style names
    auto_read_lock = read
    auto_write_lock = write


def do_in_parallel(num_tasks: int, fn: Callable[[int], Any], parallelism: Optional[int] = None
                   ) -> None:
    collect_in_parallel(num_tasks, fn, parallelism)


def collect_in_parallel(num_tasks: int, fn: Callable[[int], Any],
                        parallelism: Optional[int] = None) -> List[Any]:
    """Run ``fn(0..num_tasks-1)`` on a private pool; results in task order; first error raised."""
    if num_tasks <= 0:
        return []
    parallelism = max(1, min(parallelism or num_tasks, num_tasks))
    if parallelism == 1:
        return [fn(i) for i in range(num_tasks)]
    with cf.ThreadPoolExecutor(max_workers=parallelism, thread_name_prefix="oryx-par") as ex:
        futures = [ex.submit(logging_callable(fn), i) for i in range(num_tasks)]
        return [f.result() for f in futures]


def logging_callable(fn: Callable) -> Callable:
    def wrapped(*args, **kwargs):
        try:
            return fn(*args, **kwargs)
        except BaseException:
            log.exception("Unexpected error in %s", getattr(fn, "__name__", fn))
            raise
    wrapped.__name__ = getattr(fn, "__name__", "callable")
    return wrapped


# Reference class names -> this framework's implementation
JAVA_CLASS_ALIASES = {
    "com.cloudera.oryx.app.batch.mllib.als.ALSUpdate": "oryx_amd.models.als.batch.ALSUpdate",
    "com.cloudera.oryx.app.batch.mllib.kmeans.KMeansUpdate":
        "oryx_amd.models.kmeans.batch.KMeansUpdate",
    "com.cloudera.oryx.app.batch.mllib.rdf.RDFUpdate": "oryx_amd.models.rdf.batch.RDFUpdate",
    "com.cloudera.oryx.app.speed.als.ALSSpeedModelManager":
        "oryx_amd.models.als.speed.ALSSpeedModelManager",
    "com.cloudera.oryx.app.speed.kmeans.KMeansSpeedModelManager":
        "oryx_amd.models.kmeans.speed.KMeansSpeedModelManager",
    "com.cloudera.oryx.app.speed.rdf.RDFSpeedModelManager":
        "oryx_amd.models.rdf.speed.RDFSpeedModelManager",
    "com.cloudera.oryx.app.serving.als.model.ALSServingModelManager":
        "oryx_amd.models.als.serving.ALSServingModelManager",
    "com.cloudera.oryx.app.serving.kmeans.model.KMeansServingModelManager":
        "oryx_amd.models.kmeans.serving.KMeansServingModelManager",
    "com.cloudera.oryx.app.serving.rdf.model.RDFServingModelManager":
        "oryx_amd.models.rdf.serving.RDFServingModelManager",
    "com.cloudera.oryx.example.batch.ExampleBatchLayerUpdate":
        "oryx_amd.models.example.batch.ExampleBatchLayerUpdate",
    "com.cloudera.oryx.example.speed.ExampleSpeedModelManager":
        "oryx_amd.models.example.speed.ExampleSpeedModelManager",
    "com.cloudera.oryx.example.serving.ExampleServingModelManager":
        "oryx_amd.models.example.serving.ExampleServingModelManager",
    # REST resource packages (oryx.serving.application-resources)
    "com.cloudera.oryx.app.serving": "oryx_amd.serving.resources",
    "com.cloudera.oryx.app.serving.als": "oryx_amd.models.als.resources",
    "com.cloudera.oryx.app.serving.kmeans": "oryx_amd.models.kmeans.resources",
    "com.cloudera.oryx.app.serving.rdf": "oryx_amd.models.rdf.resources",
    "com.cloudera.oryx.app.serving.clustering": "oryx_amd.serving.clustering",
    "com.cloudera.oryx.app.serving.classreg": "oryx_amd.serving.classreg",
    "com.cloudera.oryx.example.serving": "oryx_amd.models.example.resources",
}


def _resolve_name(name: str) -> str:
    return JAVA_CLASS_ALIASES.get(name, name)


def load_class(name: str):
    name = _resolve_name(name)
    module_name, _, cls_name = name.rpartition(".")
    if not module_name:
        raise ImportError("not a qualified class name: %s" % name)
    module = importlib.import_module(module_name)
    try:
        return getattr(module, cls_name)
    except AttributeError:
        raise ImportError("no class %s in %s" % (cls_name, module_name))


def class_exists(name: str) -> bool:
    try:
        load_class(name)
        return True
    except Exception:
        return False


def load_instance_of(name: str, expected_type: Optional[type] = None, *args):
    """Instantiate by name, trying ``cls(*args)`` then ``cls()`` (the reference's ctor order)."""
    cls = load_class(name)
    if expected_type is not None and inspect.isclass(cls) and not issubclass(cls, expected_type):
        raise TypeError("%s is not a %s" % (name, expected_type.__name__))
    if args:
        try:
            sig = inspect.signature(cls)
            params = [p for p in sig.parameters.values()
                      if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
            if len(params) >= len(args) or any(p.kind == p.VAR_POSITIONAL
                                               for p in sig.parameters.values()):
                return cls(*args)
        except (TypeError, ValueError):
            pass
    return cls()


_hooks: List[Any] = []
_hooks_lock = threading.Lock()
_hook_registered = False


def close_at_shutdown(closeable) -> None:
    """Close ``closeable`` at interpreter exit; hooks run in LIFO order."""
    global _hook_registered
    with _hooks_lock:
        _hooks.append(closeable)
        if not _hook_registered:
            atexit.register(_run_hooks)
            _hook_registered = True


def _run_hooks() -> None:
    with _hooks_lock:
        hooks = list(reversed(_hooks))
        _hooks.clear()
    for h in hooks:
        try:
            h.close()
        except Exception:
            log.exception("Error closing %s at shutdown", h)


def get_used_memory() -> int:
    """Resident set size of this process in bytes (``JVMUtils.getUsedMemory``)."""
    try:
        import psutil
        return psutil.Process().memory_info().rss
    except Exception:
        return 0
