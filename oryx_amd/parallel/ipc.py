"""One-shot all-reduce of small fp32 tensors through peer-mapped exchange buffers (SURVEY.md
section 5.8; kernel: ``csrc/kernels/ipc_allreduce.hip``).

The batch layer's latency-bound reductions -- the k x k YtY Gramian each ALS half-step and the
K x (d + 1) centroid sums / counts each Lloyd step, the stand-ins for MLlib's shuffles
(``[mllib]/als/ALSUpdate.java:116-124``, ``[mllib]/kmeans/KMeansUpdate.java:116-117``) -- are
tens of KB to a few MB.  A ring all-reduce over 8 GPUs takes 2 (W - 1) dependent steps; the
one-shot form reads every peer's payload directly over the point-to-point xGMI links in one
step.  Every rank of the node allocates one uncached exchange buffer, exports it with
``hipIpcGetMemHandle``, and maps every peer's (``hipIpcOpenMemHandle``); handles travel over
the gloo control group.

Safety: the reducer runs a self-test against ``torch.distributed.all_reduce`` when it is
created (all ranks agree on the verdict); a peer that never arrives makes the kernel stop
waiting after 120 s, set an error flag and write NaN instead of the sum (``check()`` raises
and clears the flag) instead of hanging the GPU.  Tensors larger than the slot capacity,
non-fp32 tensors and multi-node worlds use RCCL.

It is on by default for multi-rank CUDA (RCCL) worlds on one node and for a forced world of
one (``ORYX_FORCE_COLLECTIVES=1``) when the self-test passes; ``ORYX_IPC_ALLREDUCE=0`` turns
it off.
"""

from __future__ import annotations

import ctypes
import logging
import os
from typing import List, Optional

import torch
import torch.distributed as tdist

from .. import native

log = logging.getLogger(__name__)

__all__ = ["IpcAllReduce", "maybe_create"]


class IpcAllReduce:
    def __init__(self, ctx, cap_bytes: int = 8 << 20):
        self.ctx = ctx
        self.lib = native.require_kernels()
        self.W = ctx.world_size
        self.rank = ctx.rank
        self.cap = int(cap_bytes) // 4
        hdr = int(self.lib.oryx_ipc_header_floats())
        nbytes = (hdr + 2 * self.cap) * 4
        self._own = None
        self._opened: List[int] = []
        mine: Optional[bytes] = None
        try:
            own = ctypes.c_void_p()
            native.check(self.lib.oryx_ipc_alloc(nbytes, ctypes.byref(own)), "oryx_ipc_alloc")
            self._own = own.value
            hs = int(self.lib.oryx_ipc_handle_size())
            h = (ctypes.c_char * hs)()
            native.check(self.lib.oryx_ipc_handle(ctypes.c_void_p(self._own), h),
                         "oryx_ipc_handle")
            mine = bytes(h)
        except Exception as e:   # noqa: BLE001 -- still take part in the exchange below
            log.warning("IPC exchange buffer unavailable on rank %d: %s", self.rank, e)
        # every rank takes part in the exchange, so a failure on one rank cannot leave the
        # others waiting in it
        handles: List[Optional[bytes]] = [None] * self.W
        group = ctx.control if ctx.control is not None else ctx.group
        if self.W > 1:
            tdist.all_gather_object(handles, mine, group=group)
        else:
            handles = [mine]
        if any(hb is None for hb in handles):
            self.close()
            raise RuntimeError("IPC exchange buffers missing on some rank")
        ptrs = []
        for r, hb in enumerate(handles):
            if r == self.rank:
                ptrs.append(self._own)
                continue
            p = ctypes.c_void_p()
            native.check(self.lib.oryx_ipc_open(hb, ctypes.byref(p)), "oryx_ipc_open")
            self._opened.append(p.value)
            ptrs.append(p.value)
        self._peers = (ctypes.c_void_p * self.W)(*ptrs)
        self.err = torch.zeros(1, dtype=torch.int32, device=ctx.device)
        self.epoch = 0
        self.calls = 0

    def close(self) -> None:
        for p in self._opened:
            self.lib.oryx_ipc_close(ctypes.c_void_p(p))
        self._opened = []
        if self._own:
            self.lib.oryx_ipc_free(ctypes.c_void_p(self._own))
            self._own = None

    def fits(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                and 0 < t.numel() <= self.cap)

    def all_reduce_(self, t: torch.Tensor, timeout_s: float = 120.0) -> torch.Tensor:
        """In-place sum over the ranks (stream-ordered on the current stream)."""
        self.epoch += 1
        self.calls += 1
        rc = self.lib.oryx_ipc_allreduce_f32(
            ctypes.c_void_p(t.data_ptr()), t.numel(), self._peers, self.W, self.rank,
            self.epoch & 0xFFFFFFFF, self.cap, float(timeout_s),
            ctypes.c_void_p(self.err.data_ptr()), ctypes.c_void_p(native.stream_ptr(t.device)))
        native.check(rc, "oryx_ipc_allreduce_f32")
        return t

    def check(self) -> None:
        """Raise if some call timed out waiting for a peer (synchronises the stream).

        The error flag is sticky on the device -- every call after a timeout returns NaN --
        until this method reports it; it is cleared when raising, so a caller that recovers
        (e.g. an elastic restart of the collective) starts from a clean flag."""
        e = int(self.err.item())
        if e:
            self.err.zero_()
            raise RuntimeError("IPC all-reduce: rank %d never arrived (results since the "
                               "timeout are NaN)" % (e - 1))

    def self_test(self) -> bool:
        """Sum rank-dependent probes both ways; True when every rank matched RCCL."""
        ok = True
        try:
            for n in (1, 257, 4096 + 3):
                base = torch.arange(n, dtype=torch.float32, device=self.ctx.device)
                a = base * (self.rank + 1) + 0.25 * self.rank
                b = a.clone()
                # short deadline: a mapping that does not work must not stall start-up
                self.all_reduce_(a, timeout_s=5.0)
                if self.W > 1 or self.ctx.forced:
                    tdist.all_reduce(b, group=self.ctx.group)
                self.check()
                ok = ok and bool(torch.equal(a, b))
        except Exception as e:   # noqa: BLE001 -- any failure disables the path
            log.warning("IPC all-reduce self-test failed on rank %d: %s", self.rank, e)
            ok = False
        flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=self.ctx.device)
        if self.W > 1 or self.ctx.forced:
            tdist.all_reduce(flag, group=self.ctx.group)
        return int(flag.item()) == 0


def _single_node(ctx) -> bool:
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    return lw is None or int(lw) == ctx.world_size


def maybe_create(ctx) -> Optional[IpcAllReduce]:
    """The node's reducer when enabled and its self-test passes (collective: every rank of
    ``ctx`` calls it); else None."""
    mode = os.environ.get("ORYX_IPC_ALLREDUCE", "1")
    # "any": also under a gloo world (several ranks sharing one GPU in the multi-rank GPU
    # tests, where RCCL refuses duplicate devices)
    if mode == "0" or ctx.device.type != "cuda" or (ctx.backend != "nccl" and mode != "any"):
        return None
    if ctx.world_size > 16 or ctx.group is not None:
        return None
    if not (ctx.world_size > 1 or ctx.forced):
        return None
    # every rank takes the same decision (LOCAL_WORLD_SIZE is node-uniform under torchrun)
    if not _single_node(ctx):
        return None
    try:
        red = IpcAllReduce(ctx)
    except Exception as e:   # noqa: BLE001
        log.warning("IPC all-reduce unavailable on rank %d: %s", ctx.rank, e)
        red = None
    # agree: all ranks created it
    flag = torch.tensor([0 if red is not None else 1], dtype=torch.int32, device=ctx.device)
    tdist.all_reduce(flag, group=ctx.group)
    if int(flag.item()) != 0:
        if red is not None:
            red.close()
        return None
    if not red.self_test():
        red.close()
        return None
    log.info("IPC one-shot all-reduce enabled (%d ranks)", ctx.world_size)
    return red
