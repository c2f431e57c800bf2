"""Distributed ALS trainer on MI355X (the batch layer's hot loop).

Replaces Spark MLlib's block ALS that the reference runs at
``[mllib]/als/ALSUpdate.java:116-124``:

* ratings are partitioned twice -- by user owner (CSR for the user half-step) and by item
  owner (CSR for the item half-step) -- with one variable-size all-to-all each (the Spark
  shuffle C2); the CSRs stay resident in HBM for all iterations;
* every rank keeps a replicated bf16 copy of both factor matrices (the gather operand of the
  fused solve kernel) and an fp32 master copy of its own row shard;
* per half-step: partial Gramians of the owned fp32 shard are all-reduced (k x k, one call),
  then the owned rows are solved in ``gather_chunks`` row ranges; as soon as a range is
  solved its bf16 rows are all-gathered asynchronously (RCCL, striped over the xGMI links)
  while the fused HIP kernel solves the next range, so only the last range's exchange is
  exposed.  The replicated bf16 factor matrices are laid out chunk-major
  ([chunk][rank][row], see :class:`RowLayout`) so that each range's all-gather writes one
  contiguous block; the CSR column indices are remapped to that layout once, in prepare();
* iteration order follows MLlib: items from users, then users from items.

With world size 1 no collectives are issued.  On CPU the exact fp32 reference solve runs.

Factor precision: ``"bf16"`` replicates bf16 factors (the BASELINE rank-64 bf16 config);
``"fp32"`` replicates every factor row as bf16 hi|lo pairs (``ops.als.to_split_bf16``: the
same bytes as fp32, ~2^-17 relative) and the solve kernels form the Gramian from
hi*hi + hi*lo + lo*hi MFMA products -- MLlib's fp32 factors at bf16 MFMA rates.  Confidence
weights c_i stay fp32 in both modes (c_i * y_i is itself split into hi + lo).

Checkpoint / resume (the reference only truncates MLlib lineage with
``setCheckpointInterval(5)``, ``[mllib]/als/ALSUpdate.java:120``): every N iterations each rank
writes its fp32 factor shards to ``<dir>/it<k>/rank<r>.safetensors``; once all ranks have
written, rank 0 atomically replaces ``<dir>/latest.json`` (iteration, world size, shapes and a
caller-supplied data fingerprint) and removes older iteration directories, so a crash at any
point leaves one complete checkpoint.  :meth:`ALSTrainer.train` resumes from it when the
fingerprint and layout match.  Warm start (an improvement the reference lacks): initial
factor rows may be given per row, with NaN rows drawn at random as usual.
"""

from __future__ import annotations

import json
import logging
import math
import os
import shutil
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from ...ops import als as als_ops
from ...parallel import dist, watchdog
from ...utils import faults
from ... import tracing

__all__ = ["ALSTrainer", "ALSFactors"]

log = logging.getLogger(__name__)


@dataclass
class ALSFactors:
    X: torch.Tensor   # fp32 [n_users, k]
    Y: torch.Tensor   # fp32 [n_items, k]


class RowLayout:
    """Row order of a replicated factor matrix gathered in chunks.

    ``n`` rows are sharded over ``W`` ranks in equal padded shards of ``s`` rows; each shard is
    cut into ``C`` ranges of ``cr`` rows.  Gathered row of global id ``r*s + l`` (rank r, local
    l = c*cr + o): ``(c*W + r)*cr + o``.  With C = 1 this is the plain rank-major layout and
    with W = 1 it is the identity.
    """

    def __init__(self, n: int, world: int, chunks: int):
        self.n, self.W = int(n), int(world)
        self.s = dist.padded_shard_size(self.n, self.W)
        self.C = max(1, min(int(chunks), self.s)) if self.s > 0 else 1
        self.cr = max(1, -(-self.s // self.C))

    @property
    def local_rows(self) -> int:
        return self.C * self.cr

    @property
    def rows(self) -> int:
        return self.C * self.W * self.cr

    def remap(self, ids: torch.Tensor) -> torch.Tensor:
        ids = ids.to(torch.int64)
        r = torch.div(ids, self.s, rounding_mode="floor")
        loc = ids - r * self.s
        c = torch.div(loc, self.cr, rounding_mode="floor")
        return (c * self.W + r) * self.cr + (loc - c * self.cr)

    def gather(self, local: torch.Tensor, ctx: dist.DistContext, overlap_with=None,
               out: Optional[torch.Tensor] = None, name: Optional[str] = None):
        """All-gather ``local`` ([local_rows, ...]) into the gathered layout; ``overlap_with``
        (callable c -> None) runs before each range's exchange is started.  ``out``: the
        previous gathered matrix, overwritten in place when its shape fits (the collectives
        are ordered after every kernel already queued on the current stream, i.e. after the
        last reads of the old rows), so the exchange allocates nothing per half-step.

        ``name`` ("X" / "Y"): with the node's peer-push all-gather (``ctx.ipc_gather``) the
        gathered matrix is that gatherer's peer-mapped buffer of this name, and each range's
        rows are written straight into every rank's copy as soon as they are solved."""
        ag = getattr(ctx, "ipc_gather", None)
        if ag is not None and name is not None and ctx.is_distributed:
            shape = (self.rows,) + tuple(local.shape[1:])
            full = ag.buffer(name, shape, local.dtype)
            # from here on the peers may overwrite this rank's copy: every kernel that read
            # its previous contents is already queued ahead on this stream
            ag.begin(name)
            for c in range(self.C):
                if overlap_with is not None:
                    overlap_with(c)
                ag.push(name, local[c * self.cr:(c + 1) * self.cr],
                        (c * self.W + ctx.rank) * self.cr, self.C, c)
            with watchdog.guard("all_gather_rows"):
                ag.end(name, self.C)
            return full
        if ctx.world_size == 1 and self.C == 1:
            # one process, one range: the local shard IS the gathered matrix (no copy)
            if overlap_with is not None:
                overlap_with(0)
            return local
        shape = (self.rows,) + tuple(local.shape[1:])
        if out is None or tuple(out.shape) != shape or out.dtype != local.dtype or \
                out.data_ptr() == local.data_ptr():
            out = torch.empty(shape, dtype=local.dtype, device=local.device)
            if ctx.emulated:
                # the other ranks' rows of an emulated world: copies of this rank's (sane
                # values for the solves that read them; an emulated exchange moves nothing)
                for c in range(self.C):
                    blk = local[c * self.cr:(c + 1) * self.cr]
                    out[c * self.W * self.cr:(c + 1) * self.W * self.cr].copy_(
                        blk.repeat((self.W,) + (1,) * (blk.dim() - 1)))
        handles = []
        for c in range(self.C):
            if overlap_with is not None:
                overlap_with(c)
            handles.append(dist.all_gather_rows_async(
                local[c * self.cr:(c + 1) * self.cr],
                out[c * self.W * self.cr:(c + 1) * self.W * self.cr], ctx))
        with watchdog.guard("all_gather_rows"):
            for h in handles:
                if h is not None:
                    h.wait()
        return out


# the batch layer's keyed init seed: fixed, as MLlib's ALS default seed is (a per-class
# constant), so a generation's factors do not depend on RNG call order or the world size
ALS_INIT_SEED = 0x0A15_5EED


def _u64_to_i64(c: int) -> int:
    return c - (1 << 64) if c >= (1 << 63) else c


_GOLD = _u64_to_i64(0x9E3779B97F4A7C15)
_MIX1 = _u64_to_i64(0xBF58476D1CE4E5B9)
_MIX2 = _u64_to_i64(0x94D049BB133111EB)


def _lsr(z: torch.Tensor, s: int) -> torch.Tensor:
    return (z >> s) & ((1 << (64 - s)) - 1)


def _mix64(z: torch.Tensor) -> torch.Tensor:
    """splitmix64 finalizer on int64 tensors (two's-complement wrapping arithmetic)."""
    z = z + _GOLD
    z = (z ^ _lsr(z, 30)) * _MIX1
    z = (z ^ _lsr(z, 27)) * _MIX2
    return z ^ _lsr(z, 31)


def keyed_unit_gaussian(keys: np.ndarray, k: int, kp: int, seed: int, device) -> torch.Tensor:
    """Unit-norm Gaussian rows [n, kp] (features past k zero) where row j depends only on
    (seed, keys[j]) -- a 64-bit hash of the row's ID -- and not on which rank holds the row or
    in which order: the same ID starts from the same vector at any world size (MLlib's ALS
    seeds its random init with a fixed default, ALSUpdate.java:116-124).  Box-Muller on two
    splitmix64 streams per (key, feature), computed on ``device``."""
    n = len(keys)
    out = torch.zeros((n, kp), dtype=torch.float32, device=device)
    if n == 0:
        return out
    h = torch.from_numpy(np.ascontiguousarray(keys, dtype=np.uint64).view(np.int64)).to(device)
    sd = _u64_to_i64((int(seed) * 0x2545F4914F6CDD1D) & ((1 << 64) - 1))
    f = torch.arange(k, dtype=torch.int64, device=device) * _GOLD
    z1 = _mix64(_mix64(h[:, None] ^ sd) ^ f)
    z2 = _mix64(z1 ^ _MIX2)
    u1 = (_lsr(z1, 11).double() + 0.5) * 2.0 ** -53
    u2 = _lsr(z2, 11).double() * 2.0 ** -53
    g = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * np.pi * u2)
    g = g / g.norm(dim=1, keepdim=True).clamp_min(1e-12)
    out[:, :k] = g.to(torch.float32)
    return out


def _unit_gaussian(n: int, k: int, kp: int, gen: torch.Generator, device) -> torch.Tensor:
    v = torch.randn((n, k), generator=gen, dtype=torch.float32, device="cpu")
    v = v / v.norm(dim=1, keepdim=True).clamp_min(1e-12)
    out = torch.zeros((n, kp), dtype=torch.float32)
    out[:, :k] = v
    return out.to(device)


class ALSTrainer:
    def __init__(self, features: int, lam: float, alpha: float, implicit: bool,
                 ctx: Optional[dist.DistContext] = None, seed: int = 0,
                 gather_chunks: Optional[int] = None, precision: str = "bf16",
                 init_seed: Optional[int] = None):
        if precision not in ("bf16", "fp32"):
            raise ValueError("precision must be bf16 or fp32, not %r" % (precision,))
        self.precision = precision
        self.split = precision == "fp32"
        self.k = int(features)
        self.kp = als_ops.padded_rank(self.k)
        self.lam = float(lam)
        self.alpha = float(alpha)
        self.implicit = bool(implicit)
        self.ctx = ctx or dist.get_context()
        self.device = self.ctx.device
        self.seed = int(seed)
        # keyed random init (init_factors with ID hashes): a fixed seed, as MLlib's default
        self.init_seed = int(init_seed) if init_seed is not None else self.seed
        self.timings: Dict[str, float] = {}
        self.fail_count = None
        self.events: Optional[list] = None
        # row ranges per half-step whose factor exchange overlaps the next range's solve
        self._explicit_chunks = bool(gather_chunks)
        # (a forced world of one has nothing to exchange: ranges there only add launch tails)
        self.gather_chunks = int(gather_chunks) if gather_chunks else (
            4 if self.ctx.world_size > 1 else 1)

    # ------------------------------------------------------------------ data
    def prepare(self, users: torch.Tensor, items: torch.Tensor, ratings: torch.Tensor,
                n_users: int, n_items: int) -> None:
        """Partition this rank's (user, item, rating) triples and build both CSRs.

        Each rank may hold any subset of the (unique) triples; together they form the data.
        """
        ctx = self.ctx
        dev = self.device
        self.n_users, self.n_items = int(n_users), int(n_items)
        W, R = ctx.world_size, ctx.rank
        self.su = dist.padded_shard_size(self.n_users, W)
        self.si = dist.padded_shard_size(self.n_items, W)
        # ids are owned round-robin (id % W, like MLlib's hash partitioner), not in contiguous
        # ranges: popularity is skewed towards some id ranges (the synthetic data: low item
        # ids), and a contiguous item shard put 43% of all ratings on rank 0 at 8 GPUs.
        # Internally a row lives at the padded global position owner * s + id // W; this rank's
        # rows are [u_lo, u_hi) of that space.
        self.u_lo, self.u_hi = R * self.su, R * self.su + self._owned(self.n_users)
        self.i_lo, self.i_hi = R * self.si, R * self.si + self._owned(self.n_items)
        users = users.to(dev, torch.int64)
        items = items.to(dev, torch.int64)
        ratings = ratings.to(dev, torch.float32)
        t0 = time.perf_counter()
        gu, gi = self._position(users, self.su), self._position(items, self.si)
        by_user = self._route(gu, gi, ratings, users % W)
        by_item = self._route(gu, gi, ratings, items % W)
        self._build_csrs(by_user, by_item)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self.timings["prepare_s"] = time.perf_counter() - t0

    def prepare_routed(self, by_user, by_item, n_users: int, n_items: int) -> None:
        """As :meth:`prepare` from triples already at their owners: ``by_user`` = (user,
        item, rating) of the users this rank owns (id % W == rank), ``by_item`` = those of
        the items it owns -- what the two all-to-alls deliver (bench.py --emulate-world builds
        one rank's share of a larger world this way)."""
        ctx = self.ctx
        dev = self.device
        self.n_users, self.n_items = int(n_users), int(n_items)
        W, R = ctx.world_size, ctx.rank
        self.su = dist.padded_shard_size(self.n_users, W)
        self.si = dist.padded_shard_size(self.n_items, W)
        self.u_lo, self.u_hi = R * self.su, R * self.su + self._owned(self.n_users)
        self.i_lo, self.i_hi = R * self.si, R * self.si + self._owned(self.n_items)
        conv = lambda t: (self._position(t[0].to(dev, torch.int64), self.su),
                          self._position(t[1].to(dev, torch.int64), self.si),
                          t[2].to(dev, torch.float32))
        t0 = time.perf_counter()
        self._build_csrs(conv(by_user), conv(by_item))
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self.timings["prepare_s"] = time.perf_counter() - t0

    def _build_csrs(self, by_user, by_item) -> None:
        W = self.ctx.world_size
        self.lay_u = RowLayout(self.n_users, W, self._chunks_for(self.n_users))
        self.lay_i = RowLayout(self.n_items, W, self._chunks_for(self.n_items))
        # column ids index the gathered (chunk-major) copy of the opposite factors
        self.csr_u = als_ops.build_csr(by_user[0], self.lay_i.remap(by_user[1]), by_user[2],
                                       self.u_hi - self.u_lo, self.lay_i.rows,
                                       row_offset=self.u_lo)
        self.csr_i = als_ops.build_csr(by_item[1], self.lay_u.remap(by_item[0]), by_item[2],
                                       self.i_hi - self.i_lo, self.lay_u.rows,
                                       row_offset=self.i_lo)
        self.csr_u_parts = self._row_parts(self.csr_u, self.lay_u)
        self.csr_i_parts = self._row_parts(self.csr_i, self.lay_i)
        self.local_nnz = self.csr_u.nnz

    # a factor matrix is exchanged in ranges only when the exchange is worth hiding and each
    # range still fills the GPU (small ranges leave CUs idle in every launch's tail)
    OVERLAP_MIN_BYTES = 16 << 20
    OVERLAP_MIN_ROWS = 8192
    OVERLAP_MIN_ROWS_W = 2048

    def _chunks_for(self, n_total: int) -> int:
        c = self.gather_chunks
        if c <= 1 or self._explicit_chunks:
            return max(1, c)
        shard = dist.padded_shard_size(n_total, self.ctx.world_size)
        if self.ctx.world_size > 1:
            # a real (or emulated) exchange: always in ranges, so all but the last range's
            # transfer hides behind the next range's solve; ranges of at least
            # OVERLAP_MIN_ROWS_W rows still fill the GPU's launches
            return max(1, min(c, shard // self.OVERLAP_MIN_ROWS_W))
        if n_total * self.kp * (4 if self.split else 2) < self.OVERLAP_MIN_BYTES or \
                shard // c < self.OVERLAP_MIN_ROWS:
            return 1
        return c

    @staticmethod
    def _row_parts(csr: als_ops.CSR, lay: RowLayout) -> List[als_ops.CSR]:
        if lay.C == 1:
            return [csr]
        return [csr.row_range(c * lay.cr, (c + 1) * lay.cr) for c in range(lay.C)]

    def _owned(self, n: int) -> int:
        """Ids of [0, n) this rank owns (id % W == rank)."""
        W, R = self.ctx.world_size, self.ctx.rank
        return max(0, (n - R + W - 1) // W)

    def _position(self, ids: torch.Tensor, s: int) -> torch.Tensor:
        """Padded global row of each id: owner * s + id // W."""
        W = self.ctx.world_size
        if W == 1:
            return ids
        return (ids % W) * s + torch.div(ids, W, rounding_mode="floor")

    def _original_order(self, full: torch.Tensor, n: int, s: int) -> torch.Tensor:
        """Rows of a rank-major gathered matrix ([W * s, ...]) back in id order ([n, ...])."""
        if self.ctx.world_size == 1:
            return full[:n]
        ids = torch.arange(n, device=full.device)
        return full[self._position(ids, s)]

    def _route(self, users, items, ratings, owner):
        """Send each (user row, item row, rating) to ``owner``: one variable-size all-to-all of
        12-byte int32 triples (the rating travels as its fp32 bits)."""
        ctx = self.ctx
        if not ctx.is_distributed:
            return users, items, ratings
        assert max(self.su, self.si) * ctx.world_size < 2 ** 31
        order = torch.argsort(owner, stable=True)
        counts = torch.bincount(owner, minlength=ctx.world_size).tolist()
        packed = torch.stack([users[order].to(torch.int32), items[order].to(torch.int32),
                              ratings[order].contiguous().view(torch.int32)], 1)
        recv = dist.all_to_all_rows(packed, counts, ctx)
        return (recv[:, 0].to(torch.int64), recv[:, 1].to(torch.int64),
                recv[:, 2].contiguous().view(torch.float32))

    # ------------------------------------------------------------------ factors
    def init_factors(self, x_init: Optional[torch.Tensor] = None,
                     y_init: Optional[torch.Tensor] = None,
                     x_keys: Optional[np.ndarray] = None,
                     y_keys: Optional[np.ndarray] = None) -> None:
        """Random unit-norm Gaussian rows (MLlib's init), or warm-start from given factors
        (full [n, k] matrices; rows containing NaN are initialised at random).  With
        ``x_keys`` / ``y_keys`` (uint64 ID hashes of this rank's local rows, in local row
        order) the random rows are keyed by ID (:func:`keyed_unit_gaussian`, seed
        ``init_seed``): independent of the world size and of row placement."""
        ctx, dev, k, kp = self.ctx, self.device, self.k, self.kp
        gen = torch.Generator(device="cpu")
        gen.manual_seed((self.seed * 1000003 + ctx.rank) & ((1 << 62) - 1))
        nu, ni = self.u_hi - self.u_lo, self.i_hi - self.i_lo
        # local shards padded to whole gather ranges (rows past the shard stay zero)
        self.X = torch.zeros((self.lay_u.local_rows, kp), dtype=torch.float32, device=dev)
        self.Y = torch.zeros((self.lay_i.local_rows, kp), dtype=torch.float32, device=dev)
        for keys, dst, n in ((x_keys, self.X, nu), (y_keys, self.Y, ni)):
            if keys is not None:
                keys = np.asarray(keys, dtype=np.uint64)
                m = min(n, len(keys))
                dst[:m] = keyed_unit_gaussian(keys[:m], k, kp, self.init_seed, dev)
                if m < n:
                    dst[m:n] = _unit_gaussian(n - m, k, kp, gen, dev)
            else:
                dst[:n] = _unit_gaussian(n, k, kp, gen, dev)
        for init, dst, lo, hi in ((x_init, self.X, self.u_lo, self.u_hi),
                                  (y_init, self.Y, self.i_lo, self.i_hi)):
            if init is None:
                continue
            rows = init[ctx.rank::ctx.world_size].to(dev, torch.float32)
            assert rows.shape[0] == hi - lo
            ok = ~torch.isnan(rows).any(1)
            dst[:hi - lo, :k] = torch.where(ok[:, None], rows, dst[:hi - lo, :k])
        # rows without any rating are never solved (the CSRs' work lists skip them) and must
        # not enter the other side's Gramian: they start, and stay, zero.  Only the sharded
        # generation's dense ids have such rows (ids a padded owner shard does not use).
        for csr, dst, n in ((self.csr_u, self.X, nu), (self.csr_i, self.Y, ni)):
            empty = csr.row_ptr[1:n + 1] == csr.row_ptr[:n]
            if n and bool(empty.any()):
                dst[:n][empty] = 0.0
        self._publish_factors()

    def _publish_factors(self) -> None:
        ctx = self.ctx
        self._graph = None            # captured launches hold the old buffers' addresses
        self.Xb_local = self._operand(self.X)
        self.Yb_local = self._operand(self.Y)
        self.Xb = self.lay_u.gather(self.Xb_local, ctx, name="X")
        self.Yb = self.lay_i.gather(self.Yb_local, ctx, name="Y")
        self.fail_count = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.iterations_done = 0

    def _operand(self, x: torch.Tensor) -> torch.Tensor:
        return als_ops.to_split_bf16(x) if self.split else x.to(torch.bfloat16)

    # ------------------------------------------------------------------ checkpoints
    # A checkpoint holds the FULL fp32 factors in global row order (not per-rank shards), so
    # it does not depend on the world size: a group that shrinks after losing a GPU (see
    # parallel/elastic.py) resumes from it with a different row sharding.
    def _layout(self, fingerprint: str, iteration: int) -> dict:
        return {"iteration": int(iteration), "format": "global-v1",
                "n_users": self.n_users, "n_items": self.n_items, "k": self.k,
                "fingerprint": str(fingerprint)}

    def save_checkpoint(self, directory: str, iteration: int, fingerprint: str = "",
                        background: bool = False) -> None:
        """Write the factors after ``iteration`` (collective: every rank calls it; rank 0
        writes one safetensors file and then ``latest.json``, both atomically).

        ``background``: rank 0 copies the factors to pinned host memory on a side stream and
        a thread writes the files while the iterations go on (the copy overlaps compute, the
        write overlaps everything); the next checkpoint or the end of the run waits for it
        (:meth:`_finish_checkpoint`).  A crash before the write lands leaves the previous
        checkpoint in place, which is all a checkpoint promises."""
        ctx = self.ctx
        self._finish_checkpoint()
        f = self.factors()
        if ctx.is_main:
            meta = self._layout(fingerprint, iteration)
            if background and f.X.is_cuda:
                import threading
                side = getattr(self, "_ckpt_stream", None)
                if side is None:
                    side = self._ckpt_stream = torch.cuda.Stream(device=f.X.device)
                # device copies the iterations cannot touch (at world 1 the factors are views
                # of the live matrices), taken in stream order
                X, Y = f.X.clone(), f.Y.clone()
                ready = torch.cuda.Event()
                ready.record(torch.cuda.current_stream(f.X.device))
                self._ckpt_cancel = threading.Event()
                cancel = self._ckpt_cancel

                def write():
                    # the device -> host copies run on the side stream (the copy engine,
                    # beside the iterations) and block only this thread
                    with torch.cuda.stream(side):
                        side.wait_event(ready)
                        hx, hy = X.cpu(), Y.cpu()
                    if not cancel.is_set():
                        self._write_checkpoint(directory, iteration, meta, hx, hy)
                self._ckpt_thread = threading.Thread(target=write, name="als-checkpoint",
                                                     daemon=True)
                self._ckpt_thread.start()
            else:
                self._write_checkpoint(directory, iteration, meta, f.X.detach().cpu(),
                                       f.Y.detach().cpu())
        if not background:
            dist.barrier(ctx)

    def _write_checkpoint(self, directory: str, iteration: int, meta: dict, X, Y) -> None:
        from safetensors.torch import save_file
        it_dir = os.path.join(directory, "it%d" % iteration)
        os.makedirs(it_dir, exist_ok=True)
        path = os.path.join(it_dir, "factors.safetensors")
        save_file({"X": X.contiguous(), "Y": Y.contiguous()}, path + ".tmp",
                  metadata={k: str(v) for k, v in meta.items()})
        os.replace(path + ".tmp", path)
        mpath = os.path.join(directory, "latest.json")
        with open(mpath + ".tmp", "w") as fh:
            json.dump(meta, fh)
        os.replace(mpath + ".tmp", mpath)
        for name in os.listdir(directory):
            if name.startswith("it") and name != "it%d" % iteration:
                shutil.rmtree(os.path.join(directory, name), ignore_errors=True)

    def _finish_checkpoint(self, cancel: bool = False) -> None:
        """Wait for a background checkpoint write (``cancel``: drop it if not yet begun)."""
        th = getattr(self, "_ckpt_thread", None)
        if th is None:
            return
        if cancel:
            self._ckpt_cancel.set()
        th.join()
        self._ckpt_thread = None

    def load_checkpoint(self, directory: str, fingerprint: str = "") -> int:
        """Restore the latest complete checkpoint if it matches this run (any world size);
        returns the iteration it was taken after, or 0 (collective; every rank gets the same
        answer and takes its own rows of the global factors)."""
        ctx = self.ctx
        iteration = 0
        if ctx.is_main:
            try:
                with open(os.path.join(directory, "latest.json")) as fh:
                    meta = json.load(fh)
                want = self._layout(fingerprint, meta.get("iteration", 0))
                path = os.path.join(directory, "it%d" % int(meta["iteration"]),
                                    "factors.safetensors")
                if meta == want and os.path.exists(path):
                    iteration = int(meta["iteration"])
                else:
                    log.info("Ignoring checkpoint in %s: layout or data differ", directory)
            except (OSError, ValueError, KeyError):
                iteration = 0
        iteration = int(dist.broadcast_object(iteration, ctx))
        if iteration <= 0:
            return 0
        from safetensors import safe_open
        path = os.path.join(directory, "it%d" % iteration, "factors.safetensors")
        with safe_open(path, framework="pt") as fh:
            xs, ys = fh.get_slice("X"), fh.get_slice("Y")
            if tuple(xs.get_shape()) != (self.n_users, self.k) or \
                    tuple(ys.get_shape()) != (self.n_items, self.k):
                raise ValueError("checkpoint factor shapes do not match the trainer")
            xr = xs[:][ctx.rank::ctx.world_size]
            yr = ys[:][ctx.rank::ctx.world_size]
        X = torch.zeros((self.lay_u.local_rows, self.kp), dtype=torch.float32)
        Y = torch.zeros((self.lay_i.local_rows, self.kp), dtype=torch.float32)
        X[:xr.shape[0], :self.k] = xr
        Y[:yr.shape[0], :self.k] = yr
        self.X = X.to(self.device)
        self.Y = Y.to(self.device)
        self._publish_factors()
        self.iterations_done = iteration
        log.info("Resumed ALS from %s after iteration %d (world size %d)", directory,
                 iteration, ctx.world_size)
        return iteration

    # ------------------------------------------------------------------ iterations
    def _mark(self, label: str) -> None:
        """Phase event for :meth:`phase_breakdown` (only while ``self.events`` is a list)."""
        if self.events is not None and self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.events.append((label, ev))

    def _half_step(self, parts, src_own_f32, src_full_bf16, dst_f32, dst_b_local, lay, name,
                   dst_full=None, mat=None):
        ctx = self.ctx
        yty = None
        self._mark(name + ".start")
        if self.implicit:
            with tracing.range(name + ".gramian"):
                yty = als_ops.gramian(src_own_f32)
                dist.all_reduce_sum(yty, ctx)
        self._mark(name + ".gramian")

        def solve(c):
            with tracing.range(name + ".solve"):
                als_ops.solve_rows(parts[c], src_full_bf16, yty, dst_f32, dst_b_local, self.k,
                                   self.lam, self.alpha, self.implicit,
                                   fail_count=self.fail_count, split=self.split)
            if c == lay.C - 1:
                self._mark(name + ".solve")
        # range c's bf16 rows are exchanged while range c+1 is solved
        with tracing.range(name + ".solve+allgather"):
            out = lay.gather(dst_b_local, ctx, overlap_with=solve, out=dst_full, name=mat)
        self._mark(name + ".exchange")
        return out

    def phase_breakdown(self, iterations: int = 3) -> Dict[str, float]:
        """Milliseconds per iteration (mean of ``iterations``) of each half-step's phases on this
        rank's stream: Gramian + YtY all-reduce, the solve launches (ranges after the first
        overlap the previous range's all-gather), and the exposed factor exchange after the
        last solve."""
        if self.device.type != "cuda":
            return {}
        self.events = []
        self.iterate(iterations)
        torch.cuda.synchronize(self.device)
        ev, self.events = self.events, None
        out: Dict[str, float] = {}
        for (la, a), (lb, b) in zip(ev[:-1], ev[1:]):
            half, phase = lb.rsplit(".", 1)
            if phase == "start":
                continue
            key = "%s_%s_ms" % (half.split(".")[-1], phase)
            out[key] = out.get(key, 0.0) + a.elapsed_time(b) / iterations
        return out

    def iterate(self, iterations: int = 1) -> None:
        for _ in range(iterations):
            self.iterations_done += 1
            faults.point("als.iteration", iteration=self.iterations_done, rank=self.ctx.rank)
            watchdog.heartbeat("als.iteration")
            if self._graph_ready():
                self._replay()
            else:
                self._one_iteration()

    def _one_iteration(self) -> None:
        # items given users, then users given items (MLlib order)
        self.Yb = self._half_step(self.csr_i_parts, self.X, self.Xb, self.Y, self.Yb_local,
                                  self.lay_i, "als.items", self.Yb, "Y")
        self.Xb = self._half_step(self.csr_u_parts, self.Y, self.Yb, self.X, self.Xb_local,
                                  self.lay_u, "als.users", self.Xb, "X")
        self._graph_warm = True

    # One process with nothing to exchange: an iteration is a fixed sequence of launches on
    # fixed buffers (the Gramian kernels, the solves, the bf16 copies), so after one eager
    # iteration (which creates every cached workspace) it can be captured once as a HIP graph
    # and replayed.  Off by default (ORYX_ALS_GRAPH=1 turns it on): at 25M ratings, rank 64,
    # the replay measured 1.689 ms per iteration against 1.655 for the eager launches (the
    # host stays ahead of the GPU either way, and a replay adds its own launch cost;
    # profiles/r5_graph_ab.txt).
    _GRAPHS = os.environ.get("ORYX_ALS_GRAPH", "0") == "1"

    def _graph_ready(self) -> bool:
        ctx = self.ctx
        return (self._GRAPHS and self.device.type == "cuda" and self.events is None and
                (not ctx.is_distributed) and (ctx.world_size == 1 or ctx.emulated) and
                getattr(self, "_graph_warm", False))

    def _replay(self) -> None:
        g = getattr(self, "_graph", None)
        if g is None:
            # capture on a side stream (torch.cuda.graph), after the work queued so far
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._one_iteration()
            self._graph = g
        g.replay()

    def train(self, iterations: int, checkpoint_dir: Optional[str] = None,
              checkpoint_interval: int = 0, fingerprint: str = "",
              x_init: Optional[torch.Tensor] = None,
              y_init: Optional[torch.Tensor] = None,
              x_keys: Optional[np.ndarray] = None,
              y_keys: Optional[np.ndarray] = None) -> ALSFactors:
        """Initialise (or resume from ``checkpoint_dir``) and run ``iterations`` iterations,
        checkpointing every ``checkpoint_interval``; a completed run removes its checkpoint."""
        done = 0
        t0 = time.perf_counter()
        use_ckpt = bool(checkpoint_dir) and checkpoint_interval > 0
        if use_ckpt:
            done = self.load_checkpoint(checkpoint_dir, fingerprint)
        self.resumed_from = done
        if done == 0:
            self.init_factors(x_init, y_init, x_keys, y_keys)
        self._lap("init_ms", t0)
        done = min(done, iterations)
        try:
            self._iterate_with_checkpoints(done, iterations, use_ckpt, checkpoint_dir,
                                           checkpoint_interval, fingerprint)
        except BaseException:
            # a failed run keeps its newest checkpoint: let a write under way land first
            self._finish_checkpoint()
            raise
        watchdog.get().end_heartbeats()
        dist.check_collectives(self.ctx)
        t_f = time.perf_counter()
        out = self.factors()
        self._lap("factors_ms", t_f)
        if use_ckpt:
            t_ck = time.perf_counter()
            # the run is complete: a checkpoint write not yet started is dropped, one under
            # way is finished, and the directory goes
            self._finish_checkpoint(cancel=True)
            dist.barrier(self.ctx)
            if self.ctx.is_main:
                shutil.rmtree(checkpoint_dir, ignore_errors=True)
            self._lap("checkpoint_ms", t_ck)
        return out

    def _iterate_with_checkpoints(self, done, iterations, use_ckpt, checkpoint_dir,
                                  checkpoint_interval, fingerprint) -> None:
        while done < iterations:
            step = iterations - done
            if use_ckpt:
                step = min(step, checkpoint_interval - done % checkpoint_interval)
            t_it = time.perf_counter()
            self.iterate(step)
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            self.timings.setdefault("iteration_ms", []).extend(
                [(time.perf_counter() - t_it) * 1e3 / step] * step)
            done += step
            if use_ckpt and done < iterations and done % checkpoint_interval == 0:
                t_ck = time.perf_counter()
                with tracing.range("als.checkpoint"):
                    self.save_checkpoint(checkpoint_dir, done, fingerprint, background=True)
                self._lap("checkpoint_ms", t_ck)

    def _lap(self, name: str, t0: float) -> None:
        """Adds the milliseconds since ``t0`` (device work included) to ``timings[name]``."""
        if self.device.type == "cuda":
            # this stream only (a background checkpoint copy runs on its own)
            torch.cuda.current_stream(self.device).synchronize()
        self.timings[name] = self.timings.get(name, 0.0) + (time.perf_counter() - t0) * 1e3

    def factors(self, gather: bool = True) -> ALSFactors:
        """Full fp32 factors (all-gathered from the owned shards)."""
        ctx = self.ctx
        X = dist.all_gather_rows(self.X[:self.su], self.n_users, ctx)
        Y = dist.all_gather_rows(self.Y[:self.si], self.n_items, ctx)
        X = self._original_order(X, self.n_users, self.su)[:, :self.k]
        Y = self._original_order(Y, self.n_items, self.si)[:, :self.k]
        return ALSFactors(X.contiguous(), Y.contiguous())

    @property
    def failures(self) -> int:
        return int(self.fail_count.item()) if self.fail_count is not None else 0
