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
and clears the flag) instead of hanging the GPU.  Every staged payload carries its call's
epoch, element count and per-workgroup checksums, which the reducers verify: ranks whose
collective sequences diverged, or a slot read stale, raise at ``check()`` too.  Tensors larger than the slot capacity,
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

__all__ = ["IpcAllReduce", "IpcAllGather", "maybe_create", "maybe_create_gather"]


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
            if e > 2000:
                why = "rank %d's staged payload failed its checksum" % (e - 2001)
            elif e > 1000:
                why = ("rank %d's slot holds another call's payload (epoch / size mismatch: "
                       "the ranks disagree on their sequence of collectives)" % (e - 1001))
            else:
                why = "rank %d never arrived" % (e - 1)
            raise RuntimeError("IPC all-reduce: %s (results since then are NaN)" % why)

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


class IpcAllGather:
    """Peer-push all-gather of replicated row matrices (kernel: ``ipc_allgather.hip``).

    :meth:`buffer` hands out a matrix that every rank holds a peer mapping of (collective:
    every rank calls it with the same name and shape; the mapping is made once and kept while
    the shape stays).  An exchange is :meth:`begin` (this rank may be overwritten from now on),
    one :meth:`push` per row range (its solved rows into every rank's copy, on a side stream,
    after the kernels already queued on the current stream) and :meth:`end` (the current
    stream waits for the side stream and for every peer's rows).  Waits are bounded; a timeout
    sets the error flag that :meth:`check` raises on."""

    GROUPS = 32            # workgroups per pushed range

    def __init__(self, ctx, timeout_s: float = 120.0):
        self.ctx = ctx
        self.lib = native.require_kernels()
        self.W, self.rank = ctx.world_size, ctx.rank
        self.timeout_s = float(timeout_s)
        lim = (ctypes.c_int * 4)()
        self.lib.oryx_ipc_gather_limits(lim)
        self.max_ranks, self.max_mats, self.max_chunks, self.max_groups = list(lim)
        if self.W > self.max_ranks:
            raise RuntimeError("IPC all-gather: %d ranks > %d" % (self.W, self.max_ranks))
        self.group = ctx.control if ctx.control is not None else ctx.group
        self._hs = int(self.lib.oryx_ipc_handle_size())
        # flag buffers: own (uncached, zeroed) and every peer's mapping of theirs
        own = ctypes.c_void_p()
        native.check(self.lib.oryx_ipc_alloc(int(self.lib.oryx_ipc_gather_flag_bytes()),
                                             ctypes.byref(own)), "oryx_ipc_alloc")
        self._flags_own = own.value
        self._opened: List[int] = []
        h = (ctypes.c_char * self._hs)()
        native.check(self.lib.oryx_ipc_handle(ctypes.c_void_p(self._flags_own), h),
                     "oryx_ipc_handle")
        ptrs = self._exchange(bytes(h), 0, self._flags_own)
        self._flags = (ctypes.c_void_p * self.W)(*ptrs)
        self.err = torch.zeros(1, dtype=torch.int32, device=ctx.device)
        self.side = torch.cuda.Stream(device=ctx.device)
        self._mats = {}        # name -> dict(t, m, epoch, dst, opened)
        self.pushes = 0
        self.self_test_info: dict = {}

    def _exchange(self, handle: bytes, offset: int, own_ptr: int) -> List[int]:
        """All ranks' (handle, offset) -> one pointer per rank (own one as is, peers' opened)."""
        allh: List[Optional[tuple]] = [None] * self.W
        if self.W > 1:
            tdist.all_gather_object(allh, (handle, int(offset)), group=self.group)
        else:
            allh = [(handle, int(offset))]
        out = []
        for r, (hb, off) in enumerate(allh):
            if r == self.rank:
                out.append(own_ptr)
                continue
            p = ctypes.c_void_p()
            native.check(self.lib.oryx_ipc_open(hb, ctypes.byref(p)), "oryx_ipc_open")
            self._opened.append(p.value)
            out.append(p.value + off)
        return out

    def buffer(self, name: str, shape, dtype) -> torch.Tensor:
        """The replicated matrix ``name`` (collective on first use or a new shape)."""
        shape = tuple(int(x) for x in shape)
        e = self._mats.get(name)
        if e is not None and tuple(e["t"].shape) == shape and e["t"].dtype == dtype:
            return e["t"]
        if e is None and len(self._mats) >= self.max_mats:
            raise RuntimeError("IPC all-gather: more than %d matrices" % self.max_mats)
        m = e["m"] if e is not None else len(self._mats)
        if e is not None:
            # this rank's last pushes through the old mappings have finished before they are
            # closed, and every peer unmaps the old copy before any rank frees it
            self.side.synchronize()
            for p in e["opened"]:
                self.lib.oryx_ipc_close(ctypes.c_void_p(p))
                self._opened.remove(p)
            if self.W > 1:
                tdist.barrier(group=self.group)
        t = torch.empty(shape, dtype=dtype, device=self.ctx.device)
        h = (ctypes.c_char * self._hs)()
        off = ctypes.c_longlong()
        native.check(self.lib.oryx_ipc_handle_range(ctypes.c_void_p(t.data_ptr()), h,
                                                    ctypes.byref(off)), "oryx_ipc_handle_range")
        before = list(self._opened)
        ptrs = self._exchange(bytes(h), off.value, t.data_ptr())
        opened = [p for p in self._opened if p not in before]
        self._mats[name] = {"t": t, "m": m, "epoch": e["epoch"] if e is not None else 0,
                            "dst": (ctypes.c_void_p * self.W)(*ptrs), "opened": opened}
        return t

    def owns(self, t: torch.Tensor) -> Optional[str]:
        for name, e in self._mats.items():
            if e["t"].data_ptr() == t.data_ptr() and e["t"].shape == t.shape:
                return name
        return None

    def begin(self, name: str) -> None:
        e = self._mats[name]
        e["epoch"] += 1
        native.check(self.lib.oryx_ipc_gather_ready(
            ctypes.c_void_p(self._flags_own), e["m"], e["epoch"] & 0xFFFFFFFF,
            ctypes.c_void_p(native.stream_ptr(self.ctx.device))), "oryx_ipc_gather_ready")
        e["side_ready"] = False

    def push(self, name: str, src: torch.Tensor, row0: int, chunks: int, c: int) -> None:
        """Push ``src`` (contiguous rows) into row ``row0`` of every rank's copy, as range
        ``c`` of ``chunks`` of this exchange."""
        e = self._mats[name]
        t = e["t"]
        row_bytes = t.stride(0) * t.element_size()
        cur = torch.cuda.current_stream(self.ctx.device)
        self.side.wait_stream(cur)
        src = src.contiguous()
        with torch.cuda.stream(self.side):
            native.check(self.lib.oryx_ipc_gather_push(
                ctypes.c_void_p(src.data_ptr()), src.numel() * src.element_size(), e["dst"],
                int(row0) * row_bytes, self._flags, self.W, self.rank, e["m"], int(chunks),
                int(c), self.GROUPS, e["epoch"] & 0xFFFFFFFF, self.timeout_s,
                ctypes.c_void_p(self.err.data_ptr()),
                ctypes.c_void_p(native.stream_ptr(self.ctx.device))),
                "oryx_ipc_gather_push")
        # the source rows must outlive the side stream's read of them
        src.record_stream(self.side)
        self.pushes += 1

    def end(self, name: str, chunks: int) -> None:
        e = self._mats[name]
        cur = torch.cuda.current_stream(self.ctx.device)
        cur.wait_stream(self.side)
        native.check(self.lib.oryx_ipc_gather_wait(
            ctypes.c_void_p(self._flags_own), self.W, e["m"], int(chunks), self.GROUPS,
            e["epoch"] & 0xFFFFFFFF, self.timeout_s, ctypes.c_void_p(self.err.data_ptr()),
            ctypes.c_void_p(native.stream_ptr(self.ctx.device))), "oryx_ipc_gather_wait")

    def check(self) -> None:
        e = int(self.err.item())
        if e:
            self.err.zero_()
            raise RuntimeError("IPC all-gather: rank %d never arrived" % (e - 1))

    def _probe(self, buf: torch.Tensor, ref: torch.Tensor, out: torch.Tensor) -> None:
        native.check(self.lib.oryx_ipc_xcd_probe(
            ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(ref.data_ptr()),
            buf.numel() * buf.element_size() // 16, ctypes.c_void_p(out.data_ptr()),
            ctypes.c_void_p(native.stream_ptr(self.ctx.device))), "oryx_ipc_xcd_probe")

    def self_test(self) -> bool:
        """Gather rank-dependent rows both ways (peer push and torch.distributed); True when
        every rank matched bitwise.  Three exchanges into the same buffer.  Before each push
        round every XCD reads the whole destination (``ipc_xcd_probe``: the old rows then sit in
        every XCD's L2 and in CUs' L1s), and after the exchange every XCD reads it again and
        compares it with the reference: a stale line anywhere fails the test (see the
        coherence note in ``ipc_allgather.hip``).  The verdict is kept in
        :attr:`self_test_info` (reported by ``bench.py``)."""
        ok = True
        name = "__selftest__"
        info = {"rounds": 0, "stale_units": 0, "pre_mismatch_units": 0, "xcd_mask": 0}
        try:
            W, rows, cols = self.W, 1000, 64
            C = 3
            cr = -(-rows // C)
            out = self.buffer(name, (C * W * cr, cols), torch.bfloat16)
            base = torch.arange(C * cr * cols, device=self.ctx.device, dtype=torch.float32)
            ref = torch.empty_like(out)
            probe = torch.zeros(4, dtype=torch.int32, device=self.ctx.device)
            for rnd in range(3):
                local = ((base % 251) * (self.rank + 1 + 7 * rnd) + self.rank - rnd) \
                    .to(torch.bfloat16).reshape(C * cr, cols)
                if rnd > 0:
                    # the previous round's rows, read through every XCD before the peers
                    # overwrite them (probe[2]: the copy must still hold them)
                    self._probe(out, ref, probe[2:4])
                self.begin(name)
                for c in range(C):
                    self.push(name, local[c * cr:(c + 1) * cr], (c * W + self.rank) * cr, C,
                              c)
                self.end(name, C)
                for c in range(C):
                    blk = local[c * cr:(c + 1) * cr].contiguous()
                    parts = list(ref[c * W * cr:(c + 1) * W * cr].chunk(W, 0))
                    if W > 1:
                        tdist.all_gather(parts, blk, group=self.ctx.group)
                    else:
                        parts[0].copy_(blk)
                self._probe(out, ref, probe[0:2])
                torch.cuda.synchronize(self.ctx.device)
                self.check()
                ok = ok and bool(torch.equal(out.view(torch.int16), ref.view(torch.int16)))
                info["rounds"] += 1
            p = probe.cpu().tolist()
            info.update(stale_units=p[0], pre_mismatch_units=p[2], xcd_mask=p[1] | p[3])
            ok = ok and p[0] == 0 and p[2] == 0
        except Exception as e:   # noqa: BLE001 -- any failure disables the path
            log.warning("IPC all-gather self-test failed on rank %d: %s", self.rank, e)
            info["error"] = str(e)
            ok = False
        info["xcds_read"] = bin(int(info["xcd_mask"])).count("1")
        flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=self.ctx.device)
        if self.W > 1:
            tdist.all_reduce(flag, group=self.ctx.group)
        info["ok"] = int(flag.item()) == 0
        info["ok_here"] = ok
        self.self_test_info = info
        return info["ok"]

    def close(self) -> None:
        # no push of this rank may still be writing through a mapping that is closed here
        self.side.synchronize()
        for p in self._opened:
            self.lib.oryx_ipc_close(ctypes.c_void_p(p))
        self._opened = []
        self._mats = {}
        if self._flags_own:
            self.lib.oryx_ipc_free(ctypes.c_void_p(self._flags_own))
            self._flags_own = None


def maybe_create_gather(ctx) -> Optional[IpcAllGather]:
    """The node's peer-push all-gather when enabled and its self-test passes (collective);
    else None.  ``ORYX_IPC_ALLGATHER``: 1 (default) on for one-node RCCL worlds, 0 off,
    ``any`` also under gloo (ranks sharing one GPU in tests)."""
    mode = os.environ.get("ORYX_IPC_ALLGATHER", "1")
    if mode == "0" or ctx.device.type != "cuda" or ctx.world_size < 2 or \
            (ctx.backend != "nccl" and mode != "any"):
        return None
    if ctx.world_size > 16 or ctx.group is not None or not _single_node(ctx):
        return None
    try:
        ag = IpcAllGather(ctx)
    except Exception as e:   # noqa: BLE001
        log.warning("IPC all-gather unavailable on rank %d: %s", ctx.rank, e)
        ag = None
    flag = torch.tensor([0 if ag is not None else 1], dtype=torch.int32, device=ctx.device)
    tdist.all_reduce(flag, group=ctx.group)
    if int(flag.item()) != 0:
        if ag is not None:
            ag.close()
        return None
    if not ag.self_test():
        ag.close()
        return None
    log.info("IPC peer-push all-gather enabled (%d ranks)", ctx.world_size)
    return ag


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
