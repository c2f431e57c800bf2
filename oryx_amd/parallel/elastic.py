"""Shrink-world recovery for multi-GPU jobs (re-init of the
communicators on a shrunken world, 8 -> 4 GPUs).

The reference delegates failures to Spark/YARN (task retries, dynamic allocation).  Here a
job is one process per GPU under ``torch.distributed.run``; a rank whose GPU fails cannot be
brought back in place, so recovery happens one level up:

* a rank that hits a device failure (a HIP runtime error -- launch failure, illegal access,
  ECC, hang -- or the ``device_lost`` fault-injection action) records its physical device in
  the supervisor's directory (:func:`report_device_lost`) and exits with
  :data:`DEVICE_LOST_EXIT`; the surviving ranks' collectives then fail (or their watchdog
  fires) and the launcher ends the group;
* :func:`supervise` runs the group; when it ends with lost devices recorded, the supervisor
  drops them from the device pool and relaunches on the largest power-of-two subset of the
  healthy devices that is smaller than the old world (8 -> 4 after one loss: a balanced ring
  over the xGMI mesh), with ``HIP_VISIBLE_DEVICES`` restricted to that subset.  Fresh
  processes mean fresh RCCL communicators over the shrunken world (the equivalent of
  ``ncclCommAbort`` + re-init without trusting any state of the failed group).
* the work resumes where it can: the batch layer re-runs the uncommitted interval (input
  offsets are committed only after an update completes) and the ALS trainer resumes from its
  world-size independent factor checkpoint (``ALSTrainer.save_checkpoint``).

Failures that record no lost device are left to ``--max-restarts`` (same-size restarts by the
launcher) and then reported, as before.
"""

from __future__ import annotations

import logging
import os
import subprocess
import tempfile
from typing import Callable, List, Optional, Sequence

__all__ = ["DEVICE_LOST_EXIT", "ENV_DIR", "report_device_lost", "is_device_failure",
           "next_world", "supervise", "physical_device"]

log = logging.getLogger(__name__)

DEVICE_LOST_EXIT = 87
ENV_DIR = "ORYX_ELASTIC_DIR"
ENV_ATTEMPT = "ORYX_ELASTIC_ATTEMPT"

# HIP runtime / driver messages that mean the device (not the program) is gone
_DEVICE_ERRORS = ("hipErrorLaunchFailure", "hipErrorIllegalAddress",
                  "hipErrorECCNotCorrectable", "hipErrorNoDevice", "illegal memory access",
                  "unspecified launch failure", "GPU Hang", "HSA_STATUS_ERROR",
                  "device-side assert", "ECC error", "uncorrectable ECC",
                  "no ROCm-capable device")


def physical_device(local_rank: Optional[int] = None) -> str:
    """The physical id of this rank's GPU: its entry in ``HIP_VISIBLE_DEVICES`` /
    ``CUDA_VISIBLE_DEVICES`` (or the local rank when neither is set)."""
    lr = int(os.environ.get("LOCAL_RANK", "0")) if local_rank is None else int(local_rank)
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if vis:
        ids = [v.strip() for v in vis.split(",") if v.strip()]
        if lr < len(ids):
            return ids[lr]
    return str(lr)


def report_device_lost(reason: str = "") -> None:
    """Record this rank's GPU as lost for the supervisor and leave the group (no cleanup: the
    device may not answer)."""
    d = os.environ.get(ENV_DIR)
    dev = physical_device()
    log.error("Device %s lost (%s): leaving the group for a shrink-world restart", dev,
              reason or "reported")
    if d:
        try:
            with open(os.path.join(d, "lost-%s" % dev), "w") as fh:
                fh.write(reason)
        except OSError:
            pass
    os._exit(DEVICE_LOST_EXIT)


def is_device_failure(exc: BaseException) -> bool:
    msg = str(exc)
    return any(p in msg for p in _DEVICE_ERRORS)


def next_world(healthy: int, current: int, min_world: int = 1) -> int:
    """The largest power of two <= ``healthy`` and < ``current`` (0 when below ``min_world``)."""
    w = 1
    while w * 2 <= healthy and w * 2 < current:
        w *= 2
    if w > healthy or w >= current or w < min_world:
        return 0
    return w


def _initial_pool(n: int) -> List[str]:
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if vis:
        ids = [v.strip() for v in vis.split(",") if v.strip()]
        if len(ids) >= n:
            return ids
    return [str(i) for i in range(n)]


def supervise(build_cmd: Callable[[int], Sequence[str]], world: int,
              min_world: int = 1, max_shrinks: int = 3, env: Optional[dict] = None,
              devices: Optional[Sequence[str]] = None) -> int:
    """Run ``build_cmd(world)`` (a launcher command for ``world`` ranks) and shrink on device
    loss as described in the module docstring.  Returns the final exit code."""
    pool = list(devices) if devices is not None else _initial_pool(world)
    base_env = dict(os.environ if env is None else env)
    attempt = 0
    while True:
        with tempfile.TemporaryDirectory(prefix="oryx_elastic_") as d:
            run_env = dict(base_env, **{ENV_DIR: d, ENV_ATTEMPT: str(attempt)})
            if attempt > 0:
                run_env["HIP_VISIBLE_DEVICES"] = ",".join(pool[:world])
                run_env.pop("CUDA_VISIBLE_DEVICES", None)
            log.info("Elastic attempt %d: %d ranks on devices %s", attempt, world,
                     ",".join(pool[:world]))
            rc = subprocess.call(list(build_cmd(world)), env=run_env)
            lost = sorted(f[len("lost-"):] for f in os.listdir(d) if f.startswith("lost-"))
        if rc == 0:
            return 0
        if not lost:
            return rc
        pool = [p for p in pool if p not in lost]
        new = next_world(len(pool), world, min_world)
        if new == 0 or attempt >= max_shrinks:
            log.error("Devices %s lost; cannot shrink below %d ranks (healthy: %d)",
                      ",".join(lost), world, len(pool))
            return rc
        log.warning("Devices %s lost: restarting on %d of the %d healthy devices (was %d)",
                    ",".join(lost), new, len(pool), world)
        world = new
        attempt += 1
