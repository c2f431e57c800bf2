"""Self-launch of one rank per GPU for scripts run as ``python script.py --gpus N``.

The driver may start a bench either under ``torch.distributed.run`` (``WORLD_SIZE`` set) or as
a plain process with ``--gpus N``.  In the second case the script must not silently run one
rank: :func:`relaunch_if_needed` starts ``torch.distributed.run --nproc-per-node N`` on the
same script as a CHILD process (never ``exec`` -- nothing here has touched the GPU yet, but a
child keeps that true by construction) and the parent exits with the child's status.

A ``WORLD_SIZE`` that disagrees with ``--gpus`` is an error (exit 2): a weak-scaling number
reported for the wrong rank count is worse than none.
"""

from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import List, Optional

__all__ = ["relaunch_if_needed", "free_port"]


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch_if_needed(script: str, argv: List[str], gpus: int,
                       env_extra: Optional[dict] = None) -> Optional[int]:
    """Return None when this process should run as a rank, else the exit code to return.

    ``script`` is the path of the running script, ``argv`` its arguments (passed through
    unchanged to every rank).
    """
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            print("error: --gpus %d but WORLD_SIZE=%s" % (gpus, ws), file=sys.stderr)
            return 2
        return None
    if gpus <= 1:
        return None
    port = os.environ.get("ORYX_MASTER_PORT") or str(free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % gpus, "--master-addr=127.0.0.1",
           "--master-port=%s" % port, script] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.setdefault("OMP_NUM_THREADS", "4")
    if env_extra:
        env.update(env_extra)
    return subprocess.call(cmd, env=env)
