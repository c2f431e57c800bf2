"""k-means device ops: nearest-center assignment, centroid accumulation, k-means|| + Lloyd.

Replaces Spark MLlib ``KMeans.train`` (invoked at ``[mllib]/kmeans/KMeansUpdate.java:116-117``;
SURVEY.md K8/K9/K11, C10/C11).  On a GPU the assignment is the fused HIP kernel
``oryx_kmeans_assign`` (bf16 MFMA distance GEMM + argmin, ``csrc/kernels/kmeans.hip``) and the
centroid sums use ``oryx_kmeans_accumulate`` (LDS-privatised column slices); across ranks the
K x d sums and K counts are all-reduced (one RCCL call per Lloyd iteration).  On CPU an exact
fp32 PyTorch path runs the same algorithm.

Precision: ``"fp32"`` (default; MLlib computes distances in double on fp32-parsed points)
uses the certified kernel ``oryx_kmeans_assign_cert``: the bf16 MFMA scan keeps each point's
three best centers and flags every point whose bf16 ranking is not provably the fp32 ranking
(rounding bounds on the bf16 operands), and ``km_rescore`` decides exactly those from the
fp32 rows -- the same argmin as an fp32 scan outside the fp32 rounding band, at close to the
bf16 kernel's cost.  ``"bf16"`` takes the bf16 argmin as is.

Algorithm (MLlib semantics): k-means|| initialisation (``initializationSteps`` rounds of
oversampling proportional to D^2 with ``l = 2k``, candidates weighted by assignment counts,
then weighted k-means++ on the candidates), or "random" (k distinct random points); Lloyd
iterations until every center moves less than ``epsilon`` or ``max_iterations``; empty
clusters keep their previous center; best of ``runs`` by cost.
"""

from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch

from .. import native
from ..parallel import dist, watchdog
from ..utils import faults

__all__ = ["assign", "accumulate", "kmeans_train", "lloyd_step", "PointSet", "KMeansResult",
           "pairwise_distances", "init_centers"]

_CHUNK = 1 << 20
# operand precision of the assignment when the caller does not name one (oryx.gpu.dtype)
DEFAULT_PRECISION = "fp32"
# cumulative (rescored top-2, full rescans) point counts of the certified kernel, per device
CERT_STATS = {}
# GPU centroid accumulation: sort-based (default) or LDS-atomic (ORYX_KMEANS_ACCUM=atomic)
_SORTED = os.environ.get("ORYX_KMEANS_ACCUM", "sorted") != "atomic"


def _pad_to(n: int, m: int) -> int:
    return ((n + m - 1) // m) * m


class DeviceCenters:
    """Centers prepared for the assignment kernel (bf16, padded, norms with +inf padding)."""

    def __init__(self, centers: torch.Tensor):
        self.k, self.d = centers.shape
        dev = centers.device
        self.d_pad = _pad_to(max(self.d, 32), 32)
        self.k_pad = _pad_to(max(self.k, 64), 64)
        cb = torch.zeros((self.k_pad, self.d_pad), dtype=torch.bfloat16, device=dev)
        cb[:self.k, :self.d] = centers
        self.cb = cb
        cn = torch.full((self.k_pad,), float("inf"), dtype=torch.float32, device=dev)
        cn[:self.k] = cb[:self.k].float().pow(2).sum(1)
        self.cnorm = cn
        self.cf = centers.to(torch.float32).contiguous()
        self._cmax = None
        self._ct2 = None

    @property
    def ct2(self) -> torch.Tensor:
        """The fp32 centers for the exact full rescan kernel, in 64-center tiles of
        dimension pairs: [ceil(k / 64)][dq / 2][64][2] with dq = d rounded up to 16 (the
        kernel's dimension slice) -- a lane's successive pair loads are 512 bytes apart (one
        base address, immediate offsets) and a wave's load covers 512 consecutive bytes.  Pad
        dimensions and pad centers are zero."""
        if self._ct2 is None:
            dq = (self.d + 15) // 16 * 16
            kc = (self.k + 63) // 64
            c = torch.zeros((kc * 64, dq), dtype=torch.float32, device=self.cf.device)
            c[:self.k, :self.d] = self.cf
            self._ct2 = c.view(kc, 64, dq // 2, 2).permute(0, 2, 1, 3).contiguous()
        return self._ct2

    @property
    def cmax(self) -> float:
        if self._cmax is None:
            self._cmax = float(self.cf.norm(dim=1).max()) if self.k else 0.0
        return self._cmax


def _kernel_ok(x: torch.Tensor) -> bool:
    return x.device.type == "cuda" and _pad_to(max(x.shape[1], 32), 32) <= 512


class PointSet:
    """A rank's points, prepared once for repeated assignment passes.

    Holds the fp32 rows (centroid sums are accumulated from these) and, when the HIP
    assignment kernel applies, a bf16 copy padded to ``d_pad`` columns plus the fp32 squared
    norms of the bf16 rows -- built once per training instead of on every Lloyd iteration
    (an N x d fp32 re-read + bf16 write that would otherwise cost as much HBM traffic as the
    assignment itself).
    """

    def __init__(self, x: torch.Tensor):
        self.x = x if x.dtype == torch.float32 and x.is_contiguous() else \
            x.to(torch.float32).contiguous()
        self.n, self.d = self.x.shape
        self.device = self.x.device
        self.xb = None
        self.xn = None
        if self.n and _kernel_ok(self.x):
            self.d_pad = _pad_to(max(self.d, 32), 32)
            self.xb = torch.zeros((self.n, self.d_pad), dtype=torch.bfloat16, device=self.device)
            self.xn = torch.empty(self.n, dtype=torch.float32, device=self.device)
            for lo in range(0, self.n, _CHUNK * 4):
                hi = min(self.n, lo + _CHUNK * 4)
                self.xb[lo:hi, :self.d] = self.x[lo:hi]
                self.xn[lo:hi] = self.xb[lo:hi].float().pow(2).sum(1)
        self._cert = None

    def cert_workspace(self):
        """(second-best index int32 [n], flags uint8 [n], full-rescan list int32 [n + 1])
        scratch of the certified kernel."""
        if self._cert is None:
            self._cert = (torch.empty(self.n, dtype=torch.int32, device=self.device),
                          torch.empty(self.n, dtype=torch.uint8, device=self.device),
                          torch.empty(self.n + 1, dtype=torch.int32, device=self.device))
        return self._cert

    @property
    def shape(self):
        return self.x.shape


def _as_points(x) -> PointSet:
    return x if isinstance(x, PointSet) else PointSet(x)


def _cert_ok(pts: "PointSet", k_pad: int) -> bool:
    return pts.d_pad in (64, 128, 256) and k_pad <= 65536


# ORYX_KMEANS_GEMM_RESCORE=1: the flag-2 points go through _rescore_flag2 (fp32 GEMM with a
# certified top-1) instead of the in-kernel full rescan.  Off by default: at K = 1000, d = 256
# it measured 12.9 ms per Lloyd step against 11.8 (the host sync, row gather, GEMM and top-k
# cost more than the rescan they replace; r3_bench_kmeans_fp32_gemm_rescore.json).
_GEMM_RESCORE = os.environ.get("ORYX_KMEANS_GEMM_RESCORE", "0") == "1"


def _rescore_flag2(x: "PointSet", dc, list2: torch.Tensor, out_a: torch.Tensor,
                   out_d: torch.Tensor) -> None:
    """The points the certified bf16 scan could not narrow to two candidates (list2: [0] =
    count, then rows): an fp32 GEMM of their rows against every center gives distances
    |x|^2 + |c|^2 - 2 x.c; a point whose GEMM best is ahead of its second best by more than
    twice the GEMM's rounding bound takes it (it is then also the exact fp32 argmin), and only
    the rest go through the exact per-dimension rescan (km_rescore_full) -- the rescan of all
    of them cost ~3 ms per Lloyd step at K = 1000, d = 256."""
    cnt = int(list2[0])
    if cnt == 0:
        return
    dev = x.device
    lib = native.require_kernels()
    if torch.backends.cuda.matmul.allow_tf32:
        # reduced-precision GEMMs void the rounding bound: every listed point is rescanned
        native.check(lib.oryx_kmeans_rescore_list(
            x.x.data_ptr(), x.x.stride(0), x.d, dc.ct2.data_ptr(), dc.k, list2.data_ptr(), cnt,
            out_a.data_ptr(), out_d.data_ptr(), native.stream_ptr(dev)),
            "oryx_kmeans_rescore_list")
        return
    rows = list2[1:1 + cnt].long()
    xf = x.x.index_select(0, rows)
    cf = dc.cf[:dc.k]
    xn = (xf * xf).sum(1)
    cn = (cf * cf).sum(1)
    d2 = torch.addmm(xn[:, None] + cn[None, :], xf, cf.t(), beta=1.0, alpha=-2.0)
    top = torch.topk(d2, min(2, dc.k), dim=1, largest=False)
    # rounding bound of the GEMM distance (and of the exact per-dimension sum), per point:
    # (d + 2) unit roundoffs of |x|^2 + |c|^2 + 2 |x| |c|, with the largest center norm
    cmax2 = cn.max()
    bound = (x.d + 2) * 2.0 ** -23 * (xn + cmax2 + 2.0 * (xn * cmax2).sqrt())
    if dc.k > 1:
        ok = (top.values[:, 1] - top.values[:, 0]) > 4.0 * bound
    else:
        ok = torch.ones(cnt, dtype=torch.bool, device=dev)
    sure = rows[ok]
    out_a[sure] = top.indices[ok, 0].to(out_a.dtype)
    out_d[sure] = top.values[ok, 0].clamp_min(0.0).to(out_d.dtype)
    rest = rows[~ok]
    if rest.numel():
        lst = torch.empty(rest.numel() + 1, dtype=torch.int32, device=dev)
        lst[0] = rest.numel()
        lst[1:] = rest.to(torch.int32)
        native.check(lib.oryx_kmeans_rescore_list(
            x.x.data_ptr(), x.x.stride(0), x.d, dc.ct2.data_ptr(), dc.k, lst.data_ptr(),
            rest.numel(), out_a.data_ptr(), out_d.data_ptr(), native.stream_ptr(dev)),
            "oryx_kmeans_rescore_list")


def assign(x, centers: torch.Tensor, exact: bool = False, out=None,
           precision: Optional[str] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(index [n], squared distance fp32 [n]) of the nearest center for each row.

    ``x``: a tensor or a prepared :class:`PointSet`.  GPU + not ``exact``: the MFMA kernels
    (indices int32, written into ``out=(idx, dist)`` when given) -- certified fp32 argmin when
    ``precision`` is "fp32" (rows the kernel re-checked carry exact fp32 distances, the others
    the bf16 estimate), bf16 argmin when "bf16".  Otherwise fp32 chunked matmul + argmin
    (indices int64).
    """
    precision = precision or DEFAULT_PRECISION
    if not exact and isinstance(x, torch.Tensor) and _kernel_ok(x) and x.shape[0]:
        x = PointSet(x)
    if isinstance(x, PointSet):
        if x.xb is not None and not exact:
            lib = native.require_kernels()
            dc = DeviceCenters(centers.float())
            n = x.n
            if out is None:
                out = (torch.empty(n, dtype=torch.int32, device=x.device),
                       torch.empty(n, dtype=torch.float32, device=x.device))
            out_a, out_d = out
            if precision == "fp32" and not _cert_ok(x, dc.k_pad):
                x = x.x          # no certified kernel for this shape: exact fp32 scan below
            elif precision == "fp32":
                idx2, flags, list2 = x.cert_workspace()
                st = CERT_STATS.get(x.device)
                if st is None:
                    st = CERT_STATS[x.device] = torch.zeros(2, dtype=torch.int64,
                                                            device=x.device)
                rc = lib.oryx_kmeans_assign_cert(
                    x.xb.data_ptr(), x.xn.data_ptr(), dc.cb.data_ptr(), n, dc.d_pad, dc.k_pad,
                    dc.cnorm.data_ptr(), x.x.data_ptr(), x.x.stride(0), x.d, dc.cf.data_ptr(),
                    dc.ct2.data_ptr(), dc.k, dc.cmax, out_a.data_ptr(), out_d.data_ptr(),
                    idx2.data_ptr(),
                    flags.data_ptr(), st.data_ptr(), list2.data_ptr(), int(_GEMM_RESCORE),
                    native.stream_ptr(x.device))
                native.check(rc, "oryx_kmeans_assign_cert")
                if _GEMM_RESCORE:
                    _rescore_flag2(x, dc, list2, out_a, out_d)
                return out_a, out_d
            else:
                rc = lib.oryx_kmeans_assign(x.xb.data_ptr(), x.xn.data_ptr(),
                                            dc.cb.data_ptr(), n, dc.d_pad, dc.k_pad,
                                            dc.cnorm.data_ptr(), out_a.data_ptr(),
                                            out_d.data_ptr(), native.stream_ptr(x.device))
                native.check(rc, "oryx_kmeans_assign")
                return out_a, out_d
        if isinstance(x, PointSet):
            x = x.x
    n = x.shape[0]
    if n == 0:
        return (torch.zeros(0, dtype=torch.int64, device=x.device),
                torch.zeros(0, dtype=torch.float32, device=x.device))
    c = centers.to(x.device, torch.float32)
    cn = c.pow(2).sum(1)
    idx = torch.empty(n, dtype=torch.int64, device=x.device)
    dd = torch.empty(n, dtype=torch.float32, device=x.device)
    for lo in range(0, n, _CHUNK):
        hi = min(n, lo + _CHUNK)
        xc = x[lo:hi].to(torch.float32)
        d2 = (xc.pow(2).sum(1, keepdim=True) + cn[None, :] - 2.0 * xc.matmul(c.t())).clamp_min_(0)
        v, i = d2.min(1)
        idx[lo:hi] = i
        dd[lo:hi] = v
    return idx, dd


def accumulate(x: torch.Tensor, idx: torch.Tensor, k: int,
               mind: Optional[torch.Tensor] = None):
    """(sums fp32 [k, d], counts int64 [k], dist stats fp64 [k, 2] = (sum d, sum d^2) or None)."""
    if isinstance(x, PointSet):
        x = x.x
    n, d = x.shape
    dev = x.device
    sums = torch.zeros((k, d), dtype=torch.float32, device=dev)
    stats = torch.zeros((k, 2), dtype=torch.float64, device=dev) if mind is not None else None
    if dev.type == "cuda" and native.kernels_available():
        lib = native.kernels()
        counts = torch.zeros(k, dtype=torch.int64, device=dev)
        xf = x if x.dtype == torch.float32 and x.is_contiguous() else \
            x.to(torch.float32).contiguous()
        ia = idx if idx.dtype == torch.int32 and idx.is_contiguous() else \
            idx.to(torch.int32).contiguous()
        md = mind.to(torch.float32).contiguous() if mind is not None else None
        mdp = md.data_ptr() if md is not None else None
        stp = stats.data_ptr() if stats is not None else None
        if _SORTED and 0 < k <= 16384 and n < (1 << 31):
            # counting sort by cluster + segmented row sums (no float atomics per element)
            ws = torch.empty(int(lib.oryx_kmeans_sorted_ws_bytes(n, k)), dtype=torch.uint8,
                             device=dev)
            rc = lib.oryx_kmeans_accumulate_sorted(xf.data_ptr(), ia.data_ptr(), mdp, n, d, d,
                                                   k, sums.data_ptr(), counts.data_ptr(), stp,
                                                   ws.data_ptr(), native.stream_ptr(dev))
            native.check(rc, "oryx_kmeans_accumulate_sorted")
            return sums, counts, stats
        rc = lib.oryx_kmeans_accumulate(xf.data_ptr(), ia.data_ptr(), mdp, n, d, d, k,
                                        sums.data_ptr(), counts.data_ptr(), stp,
                                        native.stream_ptr(dev))
        native.check(rc, "oryx_kmeans_accumulate")
        return sums, counts, stats
    idx = idx.long()
    sums.index_add_(0, idx, x.to(torch.float32))
    counts = torch.bincount(idx, minlength=k).to(torch.int64)
    if stats is not None:
        dd = mind.double().clamp_min(0).sqrt()
        stats[:, 0].index_add_(0, idx, dd)
        stats[:, 1].index_add_(0, idx, dd * dd)
    return sums, counts, stats


def pairwise_distances(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Euclidean distances [len(a), len(b)] in float64 (evaluation metrics)."""
    a = a.double()
    b = b.double()
    d2 = a.pow(2).sum(1, keepdim=True) + b.pow(2).sum(1)[None] - 2.0 * a.matmul(b.t())
    return d2.clamp_min_(0).sqrt_()


@dataclass
class KMeansResult:
    centers: torch.Tensor   # fp32 [k, d]
    counts: torch.Tensor    # int64 [k]
    cost: float
    iterations: int


def _global_count(n: int, ctx) -> int:
    if not ctx.is_distributed:
        return n
    t = torch.tensor([float(n)], dtype=torch.float64, device=ctx.device)
    dist.all_reduce_sum(t, ctx)
    return int(t.item())


def _gather_rows(rows: torch.Tensor, ctx) -> torch.Tensor:
    """All ranks' variable-size row sets concatenated (small candidate sets)."""
    if not ctx.is_distributed:
        return rows
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    sizes = [torch.zeros_like(n) for _ in range(ctx.world_size)]
    dist.all_gather_list(sizes, n, ctx)
    mx = int(max(int(s) for s in sizes))
    pad = torch.zeros((mx,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=rows.device)
    pad[:rows.shape[0]] = rows
    parts = [torch.zeros_like(pad) for _ in range(ctx.world_size)]
    dist.all_gather_list(parts, pad, ctx)
    return torch.cat([p[:int(s)] for p, s in zip(parts, sizes)])


def _kmeanspp_weighted(cands: torch.Tensor, weights: torch.Tensor, k: int,
                       gen: torch.Generator) -> torch.Tensor:
    """Weighted k-means++ on the (small) candidate set.

    Runs where the candidates live with no host round trip inside the loop: the k uniforms
    (and the fallback indices for a zero-mass step) are drawn from the host generator ``gen``
    up front, every draw is an inverse-CDF lookup on the device, and each chosen center
    updates D^2 with one GEMV (||c||^2 - 2 c.x + ||x||^2, fp64) -- the choice sequence is the
    same on CPU and GPU.  (The previous loop synchronised twice per center: 1000 centers took
    ~700 ms; this one is launch-bound at a few tens of ms.)
    """
    c = cands.double()
    dev = c.device
    w = weights.double().to(dev)
    n = c.shape[0]
    if n <= k:
        return c.float()
    u = torch.rand(k, generator=gen, dtype=torch.float64).to(dev)
    fallback = torch.randint(0, n, (k,), generator=gen).to(dev)
    cn = (c * c).sum(1)
    chosen = torch.empty(k, dtype=torch.int64, device=dev)
    if dev.type == "cuda" and native.kernels_available():
        # two small kernels per center (kmeans.hip km_pp_draw / km_pp_update: a fixed-order
        # fp64 scan, so the draws are deterministic)
        c = c.contiguous()
        ct = c.t().contiguous()
        d2 = torch.empty(n, dtype=torch.float64, device=dev)
        lib = native.require_kernels()
        native.check(lib.oryx_kmeans_pp(ct.data_ptr(), cn.contiguous().data_ptr(),
                                        w.contiguous().data_ptr(), n, c.shape[1], k,
                                        u.data_ptr(), fallback.data_ptr(), chosen.data_ptr(),
                                        d2.data_ptr(), native.stream_ptr(dev)),
                     "oryx_kmeans_pp")
        return c.index_select(0, chosen).float()

    def draw(p: torch.Tensor, s: int) -> torch.Tensor:
        cdf = torch.cumsum(p, 0)
        total = cdf[-1:]
        j = torch.searchsorted(cdf, u[s:s + 1] * total).clamp_max(n - 1)
        return torch.where(total > 0, j, fallback[s:s + 1])

    j = draw(w, 0)
    chosen[0:1] = j
    row = c.index_select(0, j)
    d2 = (cn - 2.0 * (c @ row[0]) + cn.index_select(0, j)).clamp_min(0.0)
    for s in range(1, k):
        j = draw(w * d2, s)
        chosen[s:s + 1] = j
        row = c.index_select(0, j)
        d2 = torch.minimum(d2, (cn - 2.0 * (c @ row[0]) + cn.index_select(0, j)).clamp_min(0.0))
    return c.index_select(0, chosen).float()


def _init_random(x, k, gen, ctx):
    n = x.shape[0]
    m = min(n, k)
    idx = torch.randperm(n, generator=gen)[:m].to(x.device)
    cands = _gather_rows(x[idx].float(), ctx)
    perm = torch.randperm(cands.shape[0], generator=gen)[:k]
    c = cands[perm.to(cands.device)]
    if ctx.is_distributed:
        dist.broadcast_tensor(c, ctx)
    return c


def _init_parallel(pts, k, gen, ctx, steps: int = 5, precision: Optional[str] = "bf16"):
    """k-means|| (Bahmani et al.), as MLlib's ``K_MEANS_PARALLEL``; the D^2 passes run on the
    bf16 assignment kernel by default: they only set sampling probabilities and candidate
    weights, and certifying near-ties against ~2k freshly sampled data points would re-decide
    most of them."""
    pts = _as_points(pts)
    x = pts.x
    n = x.shape[0]
    dev = x.device
    # first center: a uniformly random point (rank 0's choice broadcast)
    i0 = int(torch.randint(0, max(1, n), (1,), generator=gen))
    c0 = x[i0:i0 + 1].float() if n else torch.zeros((1, x.shape[1]), device=dev)
    if ctx.is_distributed:
        dist.broadcast_tensor(c0, ctx)
    centers = c0
    _, d2 = assign(pts, centers, precision=precision)
    d2 = d2.clone()
    # each point's nearest candidate so far, kept through the rounds: the candidate weights
    # need no final assignment pass against all ~2k * steps candidates (that pass was as much
    # distance work as all the rounds together)
    best = torch.zeros(n, dtype=torch.int64, device=dev)
    l = 2.0 * k
    # the per-point sampling uniforms come from a generator on the points' device, seeded
    # from the host generator (drawing 12.5M fp64 uniforms on the host and copying them over
    # took ~60 ms per round)
    gd = torch.Generator(device=dev)
    gd.manual_seed(int(torch.randint(0, 1 << 62, (1,), generator=gen)))
    for _ in range(steps):
        phi = d2.double().sum()
        if ctx.is_distributed:
            dist.all_reduce_sum(phi, ctx)
        if float(phi) <= 0:
            break
        p = (l * d2.double() / phi).clamp_max(1.0)
        r = torch.rand(n, generator=gd, dtype=torch.float64, device=dev)
        picked = x[(r < p)].float()
        new = _gather_rows(picked, ctx)
        if new.shape[0] == 0:
            continue
        base = centers.shape[0]
        centers = torch.cat([centers, new])
        idn, dn = assign(pts, new, precision=precision)
        closer = dn < d2
        best = torch.where(closer, idn.long() + base, best)
        d2 = torch.minimum(d2, dn)
    w = torch.bincount(best, minlength=centers.shape[0]).double()
    if ctx.is_distributed:
        dist.all_reduce_sum(w, ctx)
    chosen = _kmeanspp_weighted(centers.to(dev), w, k, gen).to(dev)
    if ctx.is_distributed:
        dist.broadcast_tensor(chosen, ctx)
    return chosen


def _farthest_points(x: torch.Tensor, d2: torch.Tensor, m: int, ctx) -> torch.Tensor:
    """The ``m`` points (over all ranks) with the largest distance to their center."""
    t = min(m, x.shape[0])
    v, i = torch.topk(d2, t) if t else (d2[:0], d2[:0].long())
    cand = torch.cat([v[:, None].float(), x[i].float()], 1)
    cand = _gather_rows(cand, ctx)
    if cand.shape[0] == 0:
        return cand[:, 1:]
    order = torch.argsort(cand[:, 0], descending=True, stable=True)[:m]
    return cand[order, 1:]


def init_centers(pts, k: int, init: str = "k-means||", seed: int = 0, run: int = 0,
                 ctx: Optional[dist.DistContext] = None, precision: Optional[str] = None):
    """The initial centers of one run (the generator seeding of :func:`kmeans_train`)."""
    pts = _as_points(pts)
    ctx = ctx or dist.DistContext(device=pts.device)
    gen = torch.Generator()
    gen.manual_seed((seed * 7919 + run * 104729 + ctx.rank) & ((1 << 62) - 1))
    if init == "random":
        return _init_random(pts.x, k, gen, ctx)
    return _init_parallel(pts, k, gen, ctx, precision=precision or "bf16")


def lloyd_step(pts: PointSet, centers: torch.Tensor, ctx, workspace=None,
               precision: Optional[str] = None):
    """One Lloyd iteration: assign (MFMA kernel), accumulate sums/counts, all-reduce them
    (one K x (d + 1) RCCL call), move the centers.  Returns (new centers, counts, assignment
    distances, number of empty clusters)."""
    kk = centers.shape[0]
    idx, d2 = assign(pts, centers, out=workspace, precision=precision)
    sums, counts, _ = accumulate(pts, idx, kk)
    if ctx.is_distributed:
        # counts ride along as an extra fp32 column (exact below 2^24 per cluster per rank;
        # summed in fp64 below)
        packed = torch.cat([sums, counts[:, None].to(torch.float32)], 1)
        if ctx.world_size * max(pts.n, 1) < (1 << 24):
            dist.all_reduce_sum(packed, ctx)
            sums, counts = packed[:, :-1], packed[:, -1].round().to(torch.int64)
        else:
            dist.all_reduce_sum(sums, ctx)
            dist.all_reduce_sum(counts, ctx)
    nonempty = counts > 0
    new = torch.where(nonempty[:, None], sums / counts.clamp_min(1)[:, None].to(torch.float32),
                      centers)
    return new, counts, d2, int((~nonempty).sum())


def _final_assign(pts: "PointSet", centers: torch.Tensor, ws, precision: Optional[str]):
    """Assignment of every point to the final centers (the model's cluster sizes) and the
    exact fp32 squared distance to its center (the run's cost).  Certified fp32 argmin on
    the MFMA kernel, then the distance to the assigned center computed directly per row (one
    read of the points) -- instead of the exact full scan of every point against every
    center, ~4x longer at 12.5M x 256 points, K = 1000."""
    precision = precision or DEFAULT_PRECISION
    if pts.xb is None or precision != "fp32" or pts.x.device.type != "cuda":
        return assign(pts, centers, exact=True)
    idx, _ = assign(pts, centers, out=ws, precision="fp32")
    x, c = pts.x, centers.float()
    d2 = torch.empty(pts.n, dtype=torch.float32, device=x.device)
    step = max(1, (1 << 28) // max(1, x.shape[1] * 4))      # ~256 MB of differences
    for lo in range(0, pts.n, step):
        hi = min(pts.n, lo + step)
        diff = x[lo:hi] - c.index_select(0, idx[lo:hi].long())
        d2[lo:hi] = diff.mul_(diff).sum(1)
    return idx.long(), d2


def kmeans_train(x, k: int, max_iterations: int, runs: int = 1,
                 init: str = "k-means||", seed: int = 0, epsilon: float = 1e-4,
                 ctx: Optional[dist.DistContext] = None,
                 precision: Optional[str] = None, reseed_empty: bool = True,
                 timings: Optional[dict] = None) -> KMeansResult:
    """Train k-means on this rank's rows ``x`` (the union over ranks is the data).

    ``timings``: when given, seconds per phase are added to it (``points`` -- the point set
    and its bf16 copy, ``init``, ``lloyd`` with ``lloyd_steps``, ``reseed``, ``final``), each
    closed by a device synchronize, so a generation can attribute its ``train`` time.

    ``reseed_empty``: a cluster left without points by a Lloyd step is moved to the point
    farthest from its center (deliberate difference, the default); False keeps its old
    center as MLlib's Lloyd loop does (``KMeans.runAlgorithm``: only clusters with points are
    updated), so an empty cluster can survive into the model with size 0."""
    dev0 = x.x.device if isinstance(x, PointSet) else x.device
    mark = [time.perf_counter()]

    def lap(name):
        if timings is None:
            return
        if dev0.type == "cuda":
            torch.cuda.synchronize(dev0)
        t = time.perf_counter()
        timings[name] = timings.get(name, 0.0) + t - mark[0]
        mark[0] = t

    pts = _as_points(x)
    x = pts.x
    ctx = ctx or dist.DistContext(device=x.device)
    best: Optional[KMeansResult] = None
    ws = None
    if pts.xb is not None:
        ws = (torch.empty(pts.n, dtype=torch.int32, device=pts.device),
              torch.empty(pts.n, dtype=torch.float32, device=pts.device))
    lap("points")
    for run in range(max(1, runs)):
        gen = torch.Generator()
        gen.manual_seed((seed * 7919 + run * 104729 + ctx.rank) & ((1 << 62) - 1))
        if init in ("random",):
            centers = _init_random(x, k, gen, ctx)
        else:
            centers = _init_parallel(pts, k, gen, ctx)
        lap("init")
        kk = centers.shape[0]
        it = 0
        for it in range(1, max_iterations + 1):
            faults.point("kmeans.iteration", iteration=it, rank=ctx.rank)
            watchdog.heartbeat("kmeans.iteration")
            new, counts, d2, n_empty = lloyd_step(pts, centers, ctx, ws, precision)
            moved = None
            if n_empty and reseed_empty:
                lap("lloyd")
                # re-seed empty clusters at the points farthest from their centers
                far = _farthest_points(x, d2, n_empty, ctx)
                if far.shape[0] == n_empty:
                    new[counts == 0] = far
                    moved = float("inf")
                lap("reseed")
            if moved is None:
                moved = (new - centers).pow(2).sum(1).max().item() if kk else 0.0
            centers = new
            if timings is not None:
                timings["lloyd_steps"] = timings.get("lloyd_steps", 0) + 1
            lap("lloyd")
            if moved <= epsilon * epsilon:
                break
        idx, d2 = _final_assign(pts, centers, ws, precision)
        cost = d2.double().sum()
        counts = torch.bincount(idx, minlength=kk).to(torch.int64)
        if ctx.is_distributed:
            dist.all_reduce_sum(cost, ctx)
            dist.all_reduce_sum(counts, ctx)
        watchdog.get().end_heartbeats()
        dist.check_collectives(ctx)
        res = KMeansResult(centers, counts, float(cost), it)
        lap("final")
        if best is None or res.cost < best.cost:
            best = res
    return best
