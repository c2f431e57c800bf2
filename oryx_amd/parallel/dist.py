"""One process per GPU over ``torch.distributed`` (RCCL on ROCm via the ``nccl`` backend).

Every Spark shuffle the reference relies on becomes one of a few
collectives here: all-reduce of partial Gramians / centroid sums / split histograms, and
all-gather of factor-matrix row shards.  Single-process runs (world size 1) skip the
collectives entirely.  CPU multi-process tests use the ``gloo`` backend.

xGMI note: each MI355X has 7 point-to-point links; RCCL's multi-channel ring/tree algorithms
already stripe large all-gathers over all links, so factor exchanges are issued as ONE large
``all_gather_into_tensor`` per half-step (bucketed only when exceeding ``bucket_bytes``)
rather than many small ones, and small latency-bound reductions (k x k Gramians) are
batched into a single all-reduce.
"""

from __future__ import annotations

import atexit
import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as tdist

from . import watchdog

__all__ = ["DistContext", "init_from_env", "get_context", "shard_range", "padded_shard_size",
           "all_gather_rows", "all_gather_rows_async", "all_reduce_sum", "broadcast_object",
           "barrier", "run_info", "split_groups", "broadcast_tensor", "all_gather_list",
           "global_rank", "check_collectives"]


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    group: Optional[object] = None          # None: the default (world) group
    control: Optional[object] = None
    # global ranks of this context's members when it is a subgroup (rank / world_size are
    # then positions within it); None for the world
    group_ranks: Optional[List[int]] = None
    # ORYX_FORCE_COLLECTIVES=1: a world of one still initialises the process group and runs
    # every collective (exercises the RCCL code paths on a single GPU)
    forced: bool = False
    # one-shot peer-mapped all-reduce for small fp32 payloads (parallel/ipc.py), or None
    ipc: Optional[object] = None
    # peer-push all-gather of the replicated factor matrices (parallel/ipc.py), or None
    ipc_gather: Optional[object] = None
    # one process playing rank `rank` of a `world_size` world (bench.py --emulate-world): the
    # layouts are the real world's, collectives move nothing (an all-gather writes only this
    # rank's slot, an all-reduce is the identity)
    emulated: bool = False

    @property
    def is_distributed(self) -> bool:
        return (self.world_size > 1 or self.forced) and not self.emulated

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_context: Optional[DistContext] = None


def _pick_device(local_rank: int, device: Optional[str]) -> torch.device:
    if device and device not in ("auto", ""):
        if device == "cuda":
            return torch.device("cuda", local_rank)
        return torch.device(device)
    if torch.cuda.is_available():
        return torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


def init_from_env(device: Optional[str] = None, backend: Optional[str] = None,
                  timeout_s: float = 600.0) -> DistContext:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*)."""
    global _context
    if _context is not None:
        return _context
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = _pick_device(local_rank, device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    ctx = DistContext(rank, world, local_rank, dev)
    ctx.forced = world == 1 and os.environ.get("ORYX_FORCE_COLLECTIVES") == "1"
    if world > 1 or ctx.forced:
        if backend is None:
            backend = "nccl" if dev.type == "cuda" else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if ctx.forced:
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        if not tdist.is_initialized():
            kwargs = dict(backend=backend, rank=rank, world_size=world,
                          timeout=datetime.timedelta(seconds=timeout_s))
            restart = os.environ.get("TORCHELASTIC_RESTART_COUNT")
            if restart not in (None, "", "0") and "MASTER_PORT" in os.environ:
                # under torch.distributed.run the agent's TCPStore outlives a failed attempt;
                # keys of the dead attempt (gloo / RCCL peer addresses) would be read by the
                # restarted ranks, so each later attempt rendezvous under its own prefix
                base = tdist.TCPStore(os.environ["MASTER_ADDR"],
                                      int(os.environ["MASTER_PORT"]), world, False,
                                      timeout=datetime.timedelta(seconds=timeout_s))
                kwargs["store"] = tdist.PrefixStore("oryx/attempt_%s" % restart, base)
            if backend == "nccl":
                kwargs["device_id"] = dev
            tdist.init_process_group(**kwargs)
        ctx.backend = backend
        # control plane: a gloo group with a long timeout for the batch layer's per-interval
        # work announcements (rank 0 may wait hours between generations)
        ctx.control = tdist.new_group(backend="gloo",
                                      timeout=datetime.timedelta(days=30))
        # tear the groups down before interpreter exit: left to the process's static
        # destructors, a gloo / RCCL group can be destroyed while its worker threads are
        # still joinable (std::terminate, SIGABRT at exit)
        atexit.register(_destroy_groups)
        from . import ipc
        ctx.ipc = ipc.maybe_create(ctx)
        ctx.ipc_gather = ipc.maybe_create_gather(ctx)
    _context = ctx
    return ctx


def _destroy_groups() -> None:
    try:
        if tdist.is_initialized():
            tdist.destroy_process_group()
    except Exception:                                      # pragma: no cover - best effort
        pass


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_info(ctx: DistContext) -> dict:
    """World size, backend and every rank's device (gathered over the control group); the
    bench JSON carries it so a scaling point can be checked for its actual rank layout."""
    me = {"rank": ctx.rank, "device": str(ctx.device)}
    if ctx.device.type == "cuda":
        me["current_device"] = torch.cuda.current_device()
    if ctx.is_distributed and tdist.is_initialized():
        allv = [None] * tdist.get_world_size()
        tdist.all_gather_object(allv, me, group=ctx.control)
        ws = tdist.get_world_size()
        backend = tdist.get_backend()
    else:
        allv, ws, backend = [me], 1, None
    out = {"world_size": ws, "backend": backend, "ranks": allv,
           "ipc_allreduce": ctx.ipc is not None, "allgather": allgather_kind(ctx)}
    ag = ctx.ipc_gather
    if ag is not None:
        out["allgather_selftest"] = dict(getattr(ag, "self_test_info", {}))
    return out


def allgather_kind(ctx: DistContext) -> str:
    """Which exchange the replicated factor matrices go through."""
    if ctx.emulated:
        return "emulated (nothing moved)"
    if not ctx.is_distributed:
        return "none (one rank)"
    if ctx.ipc_gather is not None:
        return "ipc-push (peer-mapped, per-range epoch flags)"
    return "rccl" if ctx.backend == "nccl" else str(ctx.backend)


def get_context() -> DistContext:
    return _context if _context is not None else DistContext()


def set_context(ctx: Optional[DistContext]) -> None:
    global _context
    _context = ctx


def padded_shard_size(n: int, world: int) -> int:
    return (n + world - 1) // world if world > 1 else n


def shard_range(n: int, rank: int, world: int):
    """Contiguous [lo, hi) of ``n`` rows owned by ``rank`` (equal padded shards)."""
    s = padded_shard_size(n, world)
    lo = min(n, rank * s)
    hi = min(n, lo + s)
    return lo, hi


def all_gather_rows(local: torch.Tensor, n_total: int, ctx: DistContext,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Concatenate equal-size row shards from every rank (shards padded to the same size)."""
    if not ctx.is_distributed:
        if out is not None:
            out[:local.shape[0]].copy_(local)
            return out
        return local
    s = padded_shard_size(n_total, ctx.world_size)
    if local.shape[0] != s:
        pad = torch.zeros((s,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[:local.shape[0]] = local
        local = pad
    full = out if out is not None and out.shape[0] == s * ctx.world_size else torch.empty(
        (s * ctx.world_size,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    with watchdog.guard("all_gather_rows"):
        if ctx.backend == "gloo":
            parts = list(full.chunk(ctx.world_size, 0))
            tdist.all_gather(parts, local.contiguous(), group=ctx.group)
        else:
            tdist.all_gather_into_tensor(full, local.contiguous(), group=ctx.group)
    return full


def all_gather_rows_async(local: torch.Tensor, out: torch.Tensor, ctx: DistContext):
    """Start an all-gather of one equal-size row block per rank into ``out`` (rank-major,
    ``world_size * local.shape[0]`` rows); returns a work handle (``wait()``) or None.

    With RCCL the collective runs on the communicator's stream after the kernels already
    queued on the current stream (the producer of ``local``), so compute launched afterwards
    overlaps it; ``wait()`` makes the current stream wait for it.
    """
    if ctx.emulated:
        n = local.shape[0]
        out[ctx.rank * n:(ctx.rank + 1) * n].copy_(local)
        return None
    if not ctx.is_distributed:
        out.copy_(local)
        return None
    if ctx.backend == "gloo":
        parts = list(out.chunk(ctx.world_size, 0))
        return tdist.all_gather(parts, local.contiguous(), async_op=True, group=ctx.group)
    return tdist.all_gather_into_tensor(out, local.contiguous(), async_op=True,
                                        group=ctx.group)


def all_reduce_sum(t: torch.Tensor, ctx: DistContext) -> torch.Tensor:
    """In-place sum over the group.  Small fp32 device tensors on a one-node world go through
    the one-shot peer-mapped all-reduce (parallel/ipc.py); everything else through RCCL."""
    if ctx.is_distributed:
        if ctx.ipc is not None and ctx.ipc.fits(t):
            return ctx.ipc.all_reduce_(t)
        with watchdog.guard("all_reduce"):
            tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=ctx.group)
    return t


def check_collectives(ctx: DistContext) -> None:
    """Raise if a one-shot all-reduce or a peer-push all-gather timed out waiting for a peer
    (synchronises)."""
    if ctx.ipc is not None and ctx.ipc.calls:
        ctx.ipc.check()
    if ctx.ipc_gather is not None and ctx.ipc_gather.pushes:
        ctx.ipc_gather.check()


def global_rank(ctx: DistContext, rank: int) -> int:
    """The global rank of member ``rank`` of ``ctx``'s group."""
    return ctx.group_ranks[rank] if ctx.group_ranks is not None else rank


def broadcast_tensor(t: torch.Tensor, ctx: DistContext, src: int = 0) -> torch.Tensor:
    """In-place broadcast of ``t`` from group member ``src``."""
    if ctx.is_distributed:
        with watchdog.guard("broadcast"):
            tdist.broadcast(t, src=global_rank(ctx, src), group=ctx.group)
    return t


def all_gather_list(parts: List[torch.Tensor], t: torch.Tensor, ctx: DistContext) -> None:
    """``parts[r]`` <- member r's ``t`` (equal shapes)."""
    if not ctx.is_distributed:
        parts[0].copy_(t)
        return
    with watchdog.guard("all_gather"):
        tdist.all_gather(parts, t, group=ctx.group)


def broadcast_object(obj, ctx: DistContext, src: int = 0, control: bool = False):
    """Broadcast a picklable object from ``src``; ``control=True`` uses the long-timeout gloo
    control group (host-side announcements) instead of the default group."""
    if not ctx.is_distributed:
        return obj
    lst = [obj]
    if control and ctx.control is not None:
        # control announcements legitimately wait a whole batch interval: no deadline
        tdist.broadcast_object_list(lst, src=global_rank(ctx, src), group=ctx.control)
    else:
        with watchdog.guard("broadcast_object"):
            tdist.broadcast_object_list(lst, src=global_rank(ctx, src), group=ctx.group)
    return lst[0]


def barrier(ctx: DistContext) -> None:
    if ctx.is_distributed:
        with watchdog.guard("barrier"):
            if ctx.backend == "nccl":
                tdist.barrier(group=ctx.group, device_ids=[ctx.device.index])
            else:
                tdist.barrier(group=ctx.group)


def all_to_all_rows(send: torch.Tensor, send_counts: Sequence[int], ctx: DistContext
                    ) -> torch.Tensor:
    """Variable-size all-to-all of rows (the shuffle that repartitions ratings by item)."""
    if not ctx.is_distributed:
        return send
    with watchdog.guard("all_to_all_rows"):
        return _all_to_all_rows(send, send_counts, ctx)


def _all_to_all_rows(send: torch.Tensor, send_counts: Sequence[int], ctx: DistContext
                     ) -> torch.Tensor:
    counts = torch.tensor(list(send_counts), dtype=torch.int64, device=send.device)
    recv_counts = torch.empty_like(counts)
    if ctx.backend == "gloo":
        # gloo has no all_to_all: emulate with all_gather of counts and padded payloads
        allc = [torch.empty_like(counts) for _ in range(ctx.world_size)]
        tdist.all_gather(allc, counts, group=ctx.group)
        recv_counts = torch.stack([c[ctx.rank] for c in allc])
        maxn = int(torch.stack(allc).max())
        chunks = list(torch.split(send, list(send_counts)))
        outs = []
        for src in range(ctx.world_size):
            for dst in range(ctx.world_size):
                n = int(allc[src][dst])
                buf = torch.zeros((maxn,) + tuple(send.shape[1:]), dtype=send.dtype,
                                  device=send.device)
                if src == ctx.rank:
                    buf[:n] = chunks[dst]
                tdist.broadcast(buf, src=global_rank(ctx, src), group=ctx.group)
                if dst == ctx.rank:
                    outs.append(buf[:n].clone())
        return torch.cat(outs) if outs else send[:0]
    tdist.all_to_all_single(recv_counts, counts, group=ctx.group)
    recv = torch.empty((int(recv_counts.sum()),) + tuple(send.shape[1:]), dtype=send.dtype,
                       device=send.device)
    tdist.all_to_all_single(recv, send.contiguous(), output_split_sizes=recv_counts.tolist(),
                            input_split_sizes=list(send_counts), group=ctx.group)
    return recv


_subgroups: dict = {}


def split_groups(ctx: DistContext, n_groups: int):
    """Partition the world into ``n_groups`` disjoint, equal, contiguous blocks of ranks
    (``n_groups`` is lowered to the largest divisor of the world size not above it) and
    return (this rank's block index, a :class:`DistContext` over that block).

    Every rank must call this with the same ``n_groups`` (group creation is collective); the
    process groups are created once per block layout and reused.  A block of one rank is an
    ordinary single-process context (no collectives).  Contiguous blocks keep each block's
    ranks on neighbouring GPUs.
    """
    W = ctx.world_size
    n = max(1, min(int(n_groups), W))
    while W % n:
        n -= 1
    if not ctx.is_distributed or n == 1:
        return 0, ctx
    size = W // n
    key = (W, n)
    if key not in _subgroups:
        made = []
        for g in range(n):
            ranks = list(range(g * size, (g + 1) * size))
            # new_group is collective over the world even for groups a rank is not in
            pg = tdist.new_group(ranks=ranks, backend=ctx.backend)
            ctl = tdist.new_group(ranks=ranks, backend="gloo",
                                  timeout=datetime.timedelta(days=30))
            made.append((ranks, pg, ctl))
        _subgroups[key] = made
    g = ctx.rank // size
    ranks, pg, ctl = _subgroups[key][g]
    if size == 1:
        return g, DistContext(rank=0, world_size=1, local_rank=ctx.local_rank,
                              device=ctx.device, group_ranks=ranks)
    return g, DistContext(rank=ctx.rank - ranks[0], world_size=size, local_rank=ctx.local_rank,
                          device=ctx.device, backend=ctx.backend, group=pg, control=ctl,
                          group_ranks=ranks)
