"""Test-only fault injection (the reference has none).

Instrumented call sites name a *fault point* and call :func:`point`; an armed fault at that
point fires when its conditions match the call's attributes:

* ``raise``   -- raise :class:`InjectedFault` (a crashed update / rank),
* ``exit``    -- ``os._exit(code)`` with no cleanup (a killed rank; default code 43),
* ``hang``    -- sleep ``seconds`` (a stuck collective / kernel; exercises the watchdog),
* ``device_lost`` -- the rank's GPU is reported lost and the rank leaves the group (exit 87;
  the shrink-world supervisor of ``parallel/elastic.py`` relaunches on fewer GPUs),
* anything else (``corrupt``, ``drop``, ...) is returned to the call site, which applies it
  to the data it is handling (e.g. the log writer corrupts or drops a record).

Faults are armed programmatically (:func:`arm`) or from the environment, so that a spawned
rank inherits them::

    ORYX_FAULTS="als.iteration:raise@iteration=5,rank=1;log.append:corrupt@count=1"

Each spec is ``point:action[@cond=value,...]``; ``count=N`` fires N times (default 1, 0 =
unlimited), ``code=N`` / ``seconds=S`` parameterise ``exit`` / ``hang``; other conditions
must equal (as strings) the attributes passed to :func:`point` (plus ``restart``, the
elastic agent's restart count, so ``@restart=0`` fires on the first attempt only).  Points:
``als.iteration`` (iteration, rank), ``batch.interval`` (timestamp), ``log.append`` (topic,
partition), ``speed.interval``, ``serving.update``, ``rdf.level`` (depth, rank),
``kmeans.iteration`` (iteration, rank).
"""

from __future__ import annotations

import logging
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

__all__ = ["InjectedFault", "arm", "disarm_all", "point", "armed"]

log = logging.getLogger(__name__)

_CONTROL = ("count", "code", "seconds")


class InjectedFault(RuntimeError):
    """Raised by an armed ``raise`` fault."""


@dataclass
class _Fault:
    point: str
    action: str
    conditions: Dict[str, str] = field(default_factory=dict)
    count: int = 1
    code: int = 43
    seconds: float = 3600.0
    fired: int = 0


_lock = threading.Lock()
_faults: List[_Fault] = []
_env_loaded = False


def _parse(spec: str) -> List[_Fault]:
    out = []
    for item in spec.split(";"):
        item = item.strip()
        if not item:
            continue
        head, _, conds = item.partition("@")
        name, _, action = head.partition(":")
        f = _Fault(name.strip(), (action or "raise").strip())
        for kv in conds.split(","):
            if not kv.strip():
                continue
            k, _, v = kv.partition("=")
            k, v = k.strip(), v.strip()
            if k == "count":
                f.count = int(v)
            elif k == "code":
                f.code = int(v)
            elif k == "seconds":
                f.seconds = float(v)
            else:
                f.conditions[k] = v
        out.append(f)
    return out


def _ensure_env() -> None:
    global _env_loaded
    if _env_loaded:
        return
    with _lock:
        if not _env_loaded:
            spec = os.environ.get("ORYX_FAULTS", "")
            if spec:
                _faults.extend(_parse(spec))
                log.warning("Fault injection armed from ORYX_FAULTS: %s", spec)
            _env_loaded = True


def arm(spec_or_point: str, action: Optional[str] = None, count: int = 1, code: int = 43,
        seconds: float = 3600.0, **conditions) -> None:
    """``arm("als.iteration", "raise", iteration=3)`` or ``arm("p:raise@iteration=3")``."""
    _ensure_env()
    with _lock:
        if action is None:
            _faults.extend(_parse(spec_or_point))
        else:
            _faults.append(_Fault(spec_or_point, action, {k: str(v) for k, v in
                                                          conditions.items()},
                                  count, code, seconds))


def disarm_all() -> None:
    global _env_loaded
    with _lock:
        _faults.clear()
        _env_loaded = True      # do not re-read the environment after an explicit reset


def armed() -> bool:
    _ensure_env()
    return bool(_faults)


def point(name: str, **attrs) -> Optional[str]:
    """Fire the first armed fault matching ``name`` and ``attrs``; returns a data action
    (``corrupt``, ``drop``, ...) for the call site, or None."""
    if not _faults and _env_loaded:
        return None
    _ensure_env()
    # restart attempt of an elastic (torch.distributed.run) group, so a spec can fire on the
    # first attempt only: "...@restart=0"
    attrs.setdefault("restart", os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    # and of the shrink-world supervisor (parallel/elastic.py): "...@attempt=0"
    attrs.setdefault("attempt", os.environ.get("ORYX_ELASTIC_ATTEMPT", "0"))
    hit = None
    with _lock:
        for f in _faults:
            if f.point != name or (f.count and f.fired >= f.count):
                continue
            if all(str(attrs.get(k)) == v for k, v in f.conditions.items()):
                f.fired += 1
                hit = f
                break
    if hit is None:
        return None
    log.warning("Injected fault %s:%s at %s", hit.point, hit.action, attrs)
    if hit.action == "raise":
        raise InjectedFault("injected fault at %s %s" % (name, attrs))
    if hit.action == "exit":
        os._exit(hit.code)
    if hit.action == "hang":
        time.sleep(hit.seconds)
        return None
    if hit.action == "device_lost":
        from ..parallel import elastic
        elastic.report_device_lost("injected at %s %s" % (name, attrs))
    return hit.action
