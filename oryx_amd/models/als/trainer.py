"""Distributed ALS trainer on MI355X (the batch layer's hot loop).

Replaces Spark MLlib's block ALS that the reference runs at
``[mllib]/als/ALSUpdate.java:116-124``:

* ratings are partitioned twice -- by user owner (CSR for the user half-step) and by item
  owner (CSR for the item half-step) -- with one variable-size all-to-all each (the Spark
  shuffle C2); the CSRs stay resident in HBM for all iterations;
* every rank keeps a replicated bf16 copy of both factor matrices (the gather operand of the
  fused solve kernel) and an fp32 master copy of its own row shard;
* per half-step: partial Gramians of the owned fp32 shard are all-reduced (k x k, one call),
  the fused HIP kernel solves the owned rows, and the new bf16 shard is all-gathered
  (one RCCL all-gather per half-step, striped over the xGMI links);
* iteration order follows MLlib: items from users, then users from items.

With world size 1 no collectives are issued.  On CPU the exact fp32 reference solve runs.
"""

from __future__ import annotations

import logging
import math
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ...ops import als as als_ops
from ...parallel import dist
from ... import tracing

__all__ = ["ALSTrainer", "ALSFactors"]

log = logging.getLogger(__name__)


@dataclass
class ALSFactors:
    X: torch.Tensor   # fp32 [n_users, k]
    Y: torch.Tensor   # fp32 [n_items, k]


def _unit_gaussian(n: int, k: int, kp: int, gen: torch.Generator, device) -> torch.Tensor:
    v = torch.randn((n, k), generator=gen, dtype=torch.float32, device="cpu")
    v = v / v.norm(dim=1, keepdim=True).clamp_min(1e-12)
    out = torch.zeros((n, kp), dtype=torch.float32)
    out[:, :k] = v
    return out.to(device)


class ALSTrainer:
    def __init__(self, features: int, lam: float, alpha: float, implicit: bool,
                 ctx: Optional[dist.DistContext] = None, seed: int = 0):
        self.k = int(features)
        self.kp = als_ops.padded_rank(self.k)
        self.lam = float(lam)
        self.alpha = float(alpha)
        self.implicit = bool(implicit)
        self.ctx = ctx or dist.get_context()
        self.device = self.ctx.device
        self.seed = int(seed)
        self.timings: Dict[str, float] = {}
        self.fail_count = None

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
        self.u_lo, self.u_hi = dist.shard_range(self.n_users, R, W)
        self.i_lo, self.i_hi = dist.shard_range(self.n_items, R, W)
        users = users.to(dev, torch.int64)
        items = items.to(dev, torch.int64)
        ratings = ratings.to(dev, torch.float32)
        t0 = time.perf_counter()
        by_user = self._route(users, items, ratings, users // self.su)
        by_item = self._route(users, items, ratings, items // self.si)
        self.csr_u = als_ops.build_csr(by_user[0], by_user[1], by_user[2], self.u_hi - self.u_lo,
                                       self.n_items, row_offset=self.u_lo)
        self.csr_i = als_ops.build_csr(by_item[1], by_item[0], by_item[2], self.i_hi - self.i_lo,
                                       self.n_users, row_offset=self.i_lo)
        self.local_nnz = self.csr_u.nnz
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self.timings["prepare_s"] = time.perf_counter() - t0

    def _route(self, users, items, ratings, owner):
        ctx = self.ctx
        if not ctx.is_distributed:
            return users, items, ratings
        order = torch.argsort(owner, stable=True)
        counts = torch.bincount(owner, minlength=ctx.world_size).tolist()
        packed = torch.stack([users[order].to(torch.float64), items[order].to(torch.float64),
                              ratings[order].to(torch.float64)], 1)
        recv = dist.all_to_all_rows(packed, counts, ctx)
        return (recv[:, 0].to(torch.int64), recv[:, 1].to(torch.int64),
                recv[:, 2].to(torch.float32))

    # ------------------------------------------------------------------ factors
    def init_factors(self, x_init: Optional[torch.Tensor] = None,
                     y_init: Optional[torch.Tensor] = None) -> None:
        """Random unit-norm Gaussian rows (MLlib's init), or warm-start from given factors."""
        ctx, dev, k, kp = self.ctx, self.device, self.k, self.kp
        gen = torch.Generator(device="cpu")
        gen.manual_seed((self.seed * 1000003 + ctx.rank) & ((1 << 62) - 1))
        nu, ni = self.u_hi - self.u_lo, self.i_hi - self.i_lo
        self.X = torch.zeros((self.su, kp), dtype=torch.float32, device=dev)
        self.Y = torch.zeros((self.si, kp), dtype=torch.float32, device=dev)
        if x_init is not None:
            self.X[:nu, :k] = x_init[self.u_lo:self.u_hi].to(dev, torch.float32)
        else:
            self.X[:nu] = _unit_gaussian(nu, k, kp, gen, dev)
        if y_init is not None:
            self.Y[:ni, :k] = y_init[self.i_lo:self.i_hi].to(dev, torch.float32)
        else:
            self.Y[:ni] = _unit_gaussian(ni, k, kp, gen, dev)
        self.Xb_local = self.X.to(torch.bfloat16)
        self.Yb_local = self.Y.to(torch.bfloat16)
        self.Xb = dist.all_gather_rows(self.Xb_local, self.n_users, ctx).contiguous()
        self.Yb = dist.all_gather_rows(self.Yb_local, self.n_items, ctx).contiguous()
        self.fail_count = torch.zeros(1, dtype=torch.int32, device=dev)

    # ------------------------------------------------------------------ iterations
    def _half_step(self, csr, src_own_f32, src_full_bf16, dst_f32, dst_b_local, n_total_dst,
                   name):
        ctx = self.ctx
        yty = None
        if self.implicit:
            with tracing.range(name + ".gramian"):
                yty = als_ops.gramian(src_own_f32)
                dist.all_reduce_sum(yty, ctx)
        with tracing.range(name + ".solve"):
            als_ops.solve_rows(csr, src_full_bf16, yty, dst_f32, dst_b_local, self.k, self.lam,
                               self.alpha, self.implicit, fail_count=self.fail_count)
        with tracing.range(name + ".allgather"):
            full = dist.all_gather_rows(dst_b_local, n_total_dst, ctx)
        return full

    def iterate(self, iterations: int = 1) -> None:
        for _ in range(iterations):
            # items given users, then users given items (MLlib order)
            self.Yb = self._half_step(self.csr_i, self.X, self.Xb, self.Y, self.Yb_local,
                                      self.n_items, "als.items")
            self.Xb = self._half_step(self.csr_u, self.Y, self.Yb, self.X, self.Xb_local,
                                      self.n_users, "als.users")

    def train(self, iterations: int) -> ALSFactors:
        self.init_factors()
        self.iterate(iterations)
        return self.factors()

    def factors(self, gather: bool = True) -> ALSFactors:
        """Full fp32 factors (all-gathered from the owned shards)."""
        ctx = self.ctx
        X = dist.all_gather_rows(self.X, self.n_users, ctx)[:self.n_users, :self.k]
        Y = dist.all_gather_rows(self.Y, self.n_items, ctx)[:self.n_items, :self.k]
        return ALSFactors(X.contiguous(), Y.contiguous())

    @property
    def failures(self) -> int:
        return int(self.fail_count.item()) if self.fail_count is not None else 0
