"""ALS device ops: CSR construction, Gramian, fused normal-equation solve.

The hot op is :func:`solve_rows` -- for each row of a CSR ratings matrix, gather the opposite
factor rows, form the per-row Gramian and solve the ALS normal equations.  On a GPU this
calls the hand-written CDNA4 kernel ``oryx_als_solve`` (``csrc/kernels/als.hip``: MFMA
segmented Gramian + in-register Cholesky); on CPU (tests, the ``local[*]`` plumbing config)
an exact fp32 PyTorch reference of the same math runs instead.

Normal equations (Spark MLlib's ALS, which the reference invokes at
``[mllib]/als/ALSUpdate.java:116-124``):

* implicit: ``(YtY + sum c1 y yT + lambda*n+ I) x = sum_{r>0} (1+c1) y``, ``c1 = alpha*|r|``
* explicit: ``(sum y yT + lambda*n I) x = sum r y``
"""

from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from .. import native

__all__ = ["CSR", "build_csr", "padded_rank", "gramian", "solve_rows", "solve_rows_reference",
           "to_bf16_padded", "to_split_bf16", "from_split_bf16", "pair_dots", "KERNEL_MAX_KP"]

KERNEL_MAX_KP = 128
_KERNEL_KPS = (16, 32, 48, 64, 80, 96, 112, 128)


def padded_rank(k: int) -> int:
    """Rank padded to the kernel's tile granularity (16; 16..64 and 80..128 are supported)."""
    kp = max(16, int(math.ceil(k / 16.0)) * 16)
    return kp


@dataclass
class CSR:
    """Row-compressed ratings: ``row_ptr`` int64 [n_rows+1], ``cols`` int32, ``vals`` fp32.

    ``order`` lists rows with at least one rating, longest first (the kernel's work queue).
    """

    row_ptr: torch.Tensor
    cols: torch.Tensor
    vals: torch.Tensor
    n_rows: int
    n_cols: int
    order: torch.Tensor
    # rows longer than the split threshold are accumulated in segments by several waves:
    # long_slot [n_work] int32 (-1 = not split), segs [n_seg, 4] int64 (row, slot, beg, end)
    long_slot: Optional[torch.Tensor] = None
    segs: Optional[torch.Tensor] = None
    n_long: int = 0
    _ws: Optional[torch.Tensor] = None
    _ws_epoch: int = 0

    @property
    def nnz(self) -> int:
        return int(self.cols.numel())

    @property
    def n_seg(self) -> int:
        return 0 if self.segs is None else int(self.segs.shape[0])

    def to(self, device) -> "CSR":
        mv = (lambda t: None if t is None else t.to(device))
        return CSR(self.row_ptr.to(device), self.cols.to(device), self.vals.to(device),
                   self.n_rows, self.n_cols, self.order.to(device), mv(self.long_slot),
                   mv(self.segs), self.n_long)

    def row_range(self, lo: int, hi: int) -> "CSR":
        """A view solving only rows [lo, hi): same arrays, its own work list and long-row
        split (the shared workspace is re-zeroed by every launch, which is stream-ordered)."""
        o = self.order.to(torch.int64)
        order = o[(o >= lo) & (o < hi)]
        counts = self.row_ptr[1:] - self.row_ptr[:-1]
        long_slot, segs, n_long = (None, None, 0)
        if self.long_slot is not None and order.numel():
            # rows split in the full CSR stay split (same threshold: the shortest split row)
            split_rows = o[:self.n_long]
            thr = int(counts[split_rows].min()) - 1
            seg = int((self.segs[:, 3] - self.segs[:, 2]).max())
            long_slot, segs, n_long = _split_long_rows(self.row_ptr, order, counts, thr, seg)
        return CSR(self.row_ptr, self.cols, self.vals, self.n_rows, self.n_cols,
                   order.to(torch.int32).contiguous(), long_slot, segs, n_long)

    def workspace(self, kp: int) -> Optional[torch.Tensor]:
        """fp32 scratch for the split rows' partial normal equations: one reduced record per
        long row, then one record per segment (``als_partial`` stores each segment's record,
        ``als_partial_reduce`` sums them per row), then one uint32 completion counter per
        long row (zeroed here; the solves count epochs on it, :meth:`next_epoch`)."""
        if self.n_seg == 0:
            return None
        need = (self.n_long + self.n_seg) * ws_stride(kp) + self.n_long
        if self._ws is None or self._ws.numel() < need or self._ws.device != self.row_ptr.device:
            self._ws = torch.zeros(need, dtype=torch.float32, device=self.row_ptr.device)
            self._ws_epoch = 0
        return self._ws

    def next_epoch(self) -> int:
        """The epoch of the next solve on this workspace (1, 2, ...; its counters never
        reset: a long row's counter reaches epoch x blocks once that solve's record is
        complete)."""
        self._ws_epoch += 1
        return self._ws_epoch


# Rows longer than the split threshold are cut into segments (one wave each, partial normal
# equations added with fp32 atomics) so one popular row does not set the kernel's tail.  The
# threshold adapts to the data: max(SPLIT_MIN, min(SPLIT_MEAN_FACTOR x mean row length,
# nnz / SPLIT_WORK_UNITS)), segments half of it -- at 1 GPU (items: mean 423 ratings) that is
# 4096/2048, which measured 13 % faster than 2048/1024 (fewer atomics); an 8-GPU rank's item
# shard (c2: 7.4k items, mean 3.5k ratings) gets 6250/3125: 1.755 ms per iteration against
# 1.864 with the mean-only rule (4x mean = 13.9k: the longest whole rows set the tail), 1.85 at
# 4096 and 1.82 at 8192 (r4_emul_c2_w8_split_*.json).  ORYX_ALS_SPLIT="thr,seg" fixes both.
SPLIT_MIN = 4096
SPLIT_MEAN_FACTOR = 4
SPLIT_WORK_UNITS = 4096
_SPLIT_ENV = os.environ.get("ORYX_ALS_SPLIT")


def split_params(nnz: int, n_nonempty: int) -> Tuple[int, int]:
    if _SPLIT_ENV:
        thr, seg = (int(v) for v in _SPLIT_ENV.split(","))
        return thr, seg
    mean = nnz / max(1, n_nonempty)
    thr = max(SPLIT_MIN, int(min(SPLIT_MEAN_FACTOR * mean, nnz / SPLIT_WORK_UNITS)))
    return thr, max(256, thr // 2)


def ws_stride(kp: int) -> int:
    """Floats per split-row workspace record: A [kp*kp], b [kp], count; 16-byte aligned."""
    return (kp * kp + kp + 1 + 3) // 4 * 4


def _split_long_rows(row_ptr: torch.Tensor, order: torch.Tensor, counts: torch.Tensor,
                     threshold: int, seg: int):
    lens = counts[order]
    n_long = int((lens > threshold).sum())   # order is longest-first: long rows lead
    if n_long == 0:
        return None, None, 0
    dev = order.device
    long_rows = order[:n_long].to(torch.int64)
    nseg = (lens[:n_long] + seg - 1) // seg
    seg_slot = torch.repeat_interleave(torch.arange(n_long, device=dev), nseg)
    first = torch.cumsum(nseg, 0) - nseg
    j = torch.arange(int(nseg.sum()), device=dev) - first[seg_slot]
    seg_row = long_rows[seg_slot]
    beg = row_ptr[seg_row] + j * seg
    end = torch.minimum(beg + seg, row_ptr[seg_row + 1])
    segs = torch.stack([seg_row, seg_slot, beg, end], 1).contiguous()
    long_slot = torch.full((order.numel(),), -1, dtype=torch.int32, device=dev)
    long_slot[:n_long] = torch.arange(n_long, dtype=torch.int32, device=dev)
    return long_slot, segs, n_long


def build_csr(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n_rows: int,
              n_cols: int, row_offset: int = 0, split_threshold: Optional[int] = None,
              split_segment: Optional[int] = None) -> CSR:
    """CSR of (row, col, val) triples (rows are global ids; ``row_offset`` makes them local).

    Triples must already be unique per (row, col).  Runs on the tensors' device.
    """
    device = rows.device
    r = rows.to(torch.int64) - row_offset
    key = r * int(n_cols) + cols.to(torch.int64)
    key_sorted, perm = torch.sort(key)
    r_sorted = torch.div(key_sorted, int(n_cols), rounding_mode="floor")
    c_sorted = (key_sorted - r_sorted * int(n_cols)).to(torch.int32)
    v_sorted = vals.to(torch.float32)[perm]
    counts = torch.bincount(r_sorted, minlength=n_rows)
    row_ptr = torch.zeros(n_rows + 1, dtype=torch.int64, device=device)
    torch.cumsum(counts, 0, out=row_ptr[1:])
    nz_rows = torch.nonzero(counts, as_tuple=False).flatten()
    order = nz_rows[torch.argsort(counts[nz_rows], descending=True, stable=True)]
    thr, seg = split_params(int(key.numel()), int(nz_rows.numel()))
    if split_threshold is not None:
        thr = split_threshold
    if split_segment is not None:
        seg = split_segment
    long_slot, segs, n_long = _split_long_rows(row_ptr, order, counts, thr, seg)
    return CSR(row_ptr, c_sorted.contiguous(), v_sorted.contiguous(), int(n_rows), int(n_cols),
               order.to(torch.int32).contiguous(), long_slot, segs, n_long)


def to_split_bf16(x: torch.Tensor) -> torch.Tensor:
    """fp32 [n, kp] -> bf16 [n, 2*kp]: ``hi = bf16(x)`` then ``lo = bf16(x - hi)``.

    The fp32-factor operand of the solve kernels (``store_xb`` / the SPLIT kernels in
    csrc/kernels/als.hip): ``hi + lo`` equals ``x`` to ~2^-17 relative, so the Gramian keeps
    close to fp32 precision while every load stays a bf16 MFMA operand.  Same bytes per row as
    fp32.
    """
    x = x.to(torch.float32)
    hi = x.to(torch.bfloat16)
    lo = (x - hi.to(torch.float32)).to(torch.bfloat16)
    return torch.cat([hi, lo], 1).contiguous()


def from_split_bf16(xs: torch.Tensor) -> torch.Tensor:
    kp = xs.shape[1] // 2
    return xs[:, :kp].to(torch.float32) + xs[:, kp:].to(torch.float32)


def to_bf16_padded(x: torch.Tensor, kp: int) -> torch.Tensor:
    if x.shape[1] == kp:
        return x.to(torch.bfloat16).contiguous()
    out = torch.zeros((x.shape[0], kp), dtype=torch.bfloat16, device=x.device)
    out[:, :x.shape[1]] = x
    return out


_GRAM_WS = {}


def gramian(x: torch.Tensor) -> torch.Tensor:
    """``XᵀX`` in fp32.

    On the GPU (width a multiple of 16, <= 128) this is the split-K fp32-MFMA kernel
    ``oryx_gramian_f32`` (csrc/kernels/gramian.hip): ~10 us for 162k x 64, where a library
    GEMM tiles the tiny 64 x 64 output over a handful of CUs.  Elsewhere a plain matmul.
    """
    x = x.to(torch.float32)
    kp = x.shape[1] if x.dim() == 2 else 0
    if (x.device.type == "cuda" and kp % 16 == 0 and 0 < kp <= 128 and x.shape[0] > 0
            and x.stride(1) == 1 and native.kernels_available()):
        lib = native.kernels()
        need = lib.oryx_gramian_ws_floats(kp)
        key = (x.device, kp)
        ws = _GRAM_WS.get(key)
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.float32, device=x.device)
            _GRAM_WS[key] = ws
        out = torch.empty((kp, kp), dtype=torch.float32, device=x.device)
        rc = lib.oryx_gramian_f32(x.data_ptr(), x.shape[0], x.stride(0), kp, out.data_ptr(),
                                  ws.data_ptr(), native.stream_ptr(x.device))
        native.check(rc, "oryx_gramian_f32")
        return out
    return x.t().matmul(x)


def tuning_kernels_available() -> bool:
    """Whether the loaded kernel library holds the superseded solve kernels (the tuning build,
    ``csrc/kernels/tuning/``); the default build has only the als_batch.hip ones."""
    return bool(native.require_kernels().oryx_als_tuning_available())


@contextlib.contextmanager
def solve_variant(v: int):
    """Temporarily select the KP <= 64 solve kernel (``ORYX_ALS_VARIANT`` values; A/B tests)."""
    lib = native.require_kernels()
    old = lib.oryx_als_get_variant()
    native.check(lib.oryx_als_set_variant(int(v)), "oryx_als_set_variant")
    try:
        yield
    finally:
        lib.oryx_als_set_variant(old)


@contextlib.contextmanager
def solve_wide_variant(v: int):
    """Temporarily select the KP > 64 / fp32-mode solve kernel (``ORYX_ALS_WIDE_VARIANT``:
    0 = als_solve_wide / als_solve_wave, 1 = als_solve_block, 2 = als_solve_batch_gl)."""
    lib = native.require_kernels()
    old = lib.oryx_als_get_wide_variant()
    native.check(lib.oryx_als_set_wide_variant(int(v)), "oryx_als_set_wide_variant")
    try:
        yield
    finally:
        lib.oryx_als_set_wide_variant(old)


def _use_kernel(device: torch.device, kp: int) -> bool:
    return device.type == "cuda" and kp in _KERNEL_KPS


# ORYX_ALS_PARTIAL_OVERLAP=1: the long rows' partial sums run on a side stream beside the
# batched solve (which takes the split rows last and waits per row).  Off by default: the
# resident solve grid holds every CU, so the partial sums only start as solve blocks retire
# and the waiting rows end up on the critical path -- rank 64 items 1.03 ms against 0.61
# serial, rank 128 fp32 5.54 against 4.04 (profiles/r5_partial_overlap_ab.txt)
_PARTIAL_OVERLAP = os.environ.get("ORYX_ALS_PARTIAL_OVERLAP", "0") == "1"


def solve_rows(csr: CSR, y_bf16: torch.Tensor, yty: Optional[torch.Tensor], x_out: torch.Tensor,
               xb_out: Optional[torch.Tensor], k: int, lam: float, alpha: float,
               implicit: bool, y_f32: Optional[torch.Tensor] = None,
               fail_count: Optional[torch.Tensor] = None, split: bool = False) -> None:
    """Solve every non-empty row of ``csr`` into ``x_out`` (fp32 [n_rows, kp]) / ``xb_out``.

    ``y_bf16``: the opposite factors, bf16 [n_cols, kp] zero-padded.  ``yty``: fp32 [kp, kp]
    Gramian of the opposite factors (implicit), ignored for explicit feedback.
    ``split``: fp32-factor mode -- ``y_bf16`` and ``xb_out`` are [n, 2*kp] hi|lo rows
    (:func:`to_split_bf16`).
    """
    kp = x_out.shape[1]
    device = y_bf16.device
    assert y_bf16.shape[1] == (2 * kp if split else kp), (y_bf16.shape, kp, split)
    if _use_kernel(device, kp):
        lib = native.require_kernels()
        if yty is None or not implicit:
            yty = torch.zeros((kp, kp), dtype=torch.float32, device=device)
        yty = yty.to(torch.float32).contiguous()
        assert x_out.dtype == torch.float32 and x_out.shape[1] == kp and x_out.is_contiguous()
        assert csr.row_ptr.dtype == torch.int64 and csr.cols.dtype == torch.int32
        assert y_bf16.dtype == torch.bfloat16 and y_bf16.is_contiguous()
        assert x_out.shape[0] >= csr.n_rows and y_bf16.shape[0] >= csr.n_cols
        if xb_out is not None:
            assert xb_out.dtype == torch.bfloat16 and xb_out.is_contiguous()
            assert xb_out.shape == (x_out.shape[0], y_bf16.shape[1])
        ws = csr.workspace(kp)
        if ws is not None:
            assert lib.oryx_als_ws_stride(kp) == ws_stride(kp)
            assert csr.long_slot.numel() == csr.order.numel() and csr.segs.shape[1] == 4
        rc = lib.oryx_als_solve(csr.row_ptr.data_ptr(), csr.order.data_ptr(),
                                csr.cols.data_ptr(), csr.vals.data_ptr(), y_bf16.data_ptr(),
                                yty.data_ptr(), x_out.data_ptr(),
                                xb_out.data_ptr() if xb_out is not None else None,
                                int(csr.order.numel()), int(k), int(kp), float(lam),
                                float(alpha), int(bool(implicit)),
                                fail_count.data_ptr() if fail_count is not None else None,
                                csr.long_slot.data_ptr() if csr.n_seg else None,
                                csr.segs.data_ptr() if csr.n_seg else None,
                                csr.n_seg, csr.n_long,
                                ws.data_ptr() if ws is not None else None,
                                int(bool(split)), int(csr.nnz),
                                csr.next_epoch() if (ws is not None and _PARTIAL_OVERLAP) else 0,
                                native.stream_ptr(device))
        native.check(rc, "oryx_als_solve")
        return
    # exact reference path (CPU, or ranks beyond the kernel's range)
    if y_f32 is not None:
        src = y_f32
    else:
        src = from_split_bf16(y_bf16) if split else y_bf16.to(torch.float32)
    sol = solve_rows_reference(csr, src, yty, k, lam, alpha, implicit)
    rows = csr.order.to(torch.int64)
    x_out[rows] = sol[rows].to(x_out.dtype)
    if xb_out is not None:
        xb_out[rows] = to_split_bf16(sol[rows]) if split else sol[rows].to(torch.bfloat16)


def solve_rows_reference(csr: CSR, y: torch.Tensor, yty: Optional[torch.Tensor], k: int,
                         lam: float, alpha: float, implicit: bool,
                         chunk_rows: int = 8192, bf16_operands: bool = False) -> torch.Tensor:
    """PyTorch reference of the kernel's math in fp32 (or fp64 when ``y`` is float64);
    returns [n_rows, kp] (zeros for empty rows).

    ``bf16_operands``: model the bf16 factor mode's MFMA operands exactly -- the Gramian
    terms are ``bf16(c_i * y_i) * y_i`` (``y`` itself should already be bf16-rounded).
    """
    device = y.device
    kp = y.shape[1]
    dt = torch.float64 if y.dtype == torch.float64 else torch.float32
    y = y.to(dt)
    out = torch.zeros((csr.n_rows, kp), dtype=dt, device=device)
    if csr.nnz == 0:
        return out
    row_ptr = csr.row_ptr
    counts = (row_ptr[1:] - row_ptr[:-1])
    row_of = torch.repeat_interleave(torch.arange(csr.n_rows, device=device), counts)
    r = csr.vals.to(dt)
    if implicit:
        wa = alpha * r.abs()
        wb = torch.where(r > 0, 1.0 + wa, torch.zeros_like(r))
        cnt = (r > 0).to(dt)
    else:
        wa = torch.ones_like(r)
        wb = r
        cnt = torch.ones_like(r)
    pad_diag = torch.zeros(kp, device=device, dtype=dt)
    pad_diag[k:] = 1.0
    for lo in range(0, csr.n_rows, chunk_rows):
        hi = min(csr.n_rows, lo + chunk_rows)
        s, e = int(row_ptr[lo]), int(row_ptr[hi])
        if s == e:
            continue
        ro = row_of[s:e] - lo
        yy = y[csr.cols[s:e].to(torch.int64)]
        n = hi - lo
        A = torch.zeros((n, kp, kp), device=device, dtype=dt)
        cy = wa[s:e, None] * yy
        if bf16_operands:
            cy = cy.to(torch.float32).to(torch.bfloat16).to(dt)
        A.index_add_(0, ro, cy[:, :, None] * yy[:, None, :])
        b = torch.zeros((n, kp), device=device, dtype=dt)
        b.index_add_(0, ro, wb[s:e, None] * yy)
        c = torch.zeros(n, device=device, dtype=dt)
        c.index_add_(0, ro, cnt[s:e])
        if implicit and yty is not None:
            A = A + yty.to(dt)[None]
        diag = lam * c[:, None] * torch.cat([torch.ones(k, device=device, dtype=dt),
                                             torch.zeros(kp - k, device=device, dtype=dt)])[None]
        A = A + torch.diag_embed(diag + pad_diag[None])
        nonempty = counts[lo:hi] > 0
        if nonempty.any():
            idx = torch.nonzero(nonempty).flatten()
            L, info = torch.linalg.cholesky_ex(A[idx])
            if bool((info != 0).any()):
                sol = torch.linalg.lstsq(A[idx], b[idx].unsqueeze(-1)).solution.squeeze(-1)
            else:
                sol = torch.cholesky_solve(b[idx].unsqueeze(-1), L).squeeze(-1)
            out[lo + idx] = sol
    return out


def pair_dots(x: torch.Tensor, y: torch.Tensor, us: torch.Tensor, items: torch.Tensor
              ) -> torch.Tensor:
    """``dot(x[us[j]], y[items[j]])`` for each pair (evaluation predictions)."""
    if x.device.type == "cuda" and x.shape[1] % 16 == 0 and x.dtype == torch.float32 \
            and y.dtype == torch.float32 and native.kernels_available():
        lib = native.kernels()
        out = torch.empty(us.numel(), dtype=torch.float32, device=x.device)
        u32 = us.to(torch.int32).contiguous()
        i32 = items.to(torch.int32).contiguous()
        xc, yc = x.contiguous(), y.contiguous()     # alive until the launch
        rc = lib.oryx_pair_dots(xc.data_ptr(), yc.data_ptr(),
                                u32.data_ptr(), i32.data_ptr(), int(us.numel()), int(x.shape[1]),
                                out.data_ptr(), native.stream_ptr(x.device))
        native.check(rc, "oryx_pair_dots")
        return out
    return (x[us.to(torch.int64)] * y[items.to(torch.int64)]).sum(1)


def target_qui(implicit: bool, value: torch.Tensor, current: torch.Tensor) -> torch.Tensor:
    """Vectorised ``ALSUtils.computeTargetQui`` (``[app-common]/als/ALSUtils.java:37-59``).

    NaN marks "no change".  Computed in float64 like the reference.
    """
    value = value.to(torch.float64)
    current = current.to(torch.float64)
    if not implicit:
        return value.clone()
    nan = torch.full_like(value, float("nan"))
    pos = (value > 0) & (current < 1.0)
    neg = (value < 0) & (current > 0.0)
    pos_t = current + (value / (1.0 + value)) * (1.0 - current.clamp_min(0.0))
    neg_t = current + (value / (value - 1.0)) * (-current.clamp_max(1.0))
    return torch.where(pos, pos_t, torch.where(neg, neg_t, nan))


def fold_in(solver_inv: torch.Tensor, values: torch.Tensor, xu: torch.Tensor,
            xu_present: torch.Tensor, yi: torch.Tensor, implicit: bool):
    """Batched ``ALSUtils.computeUpdatedXu`` (``[app-common]/als/ALSUtils.java:74-106``).

    For B events at once: ``Qui = xu.yi`` (0.5 "don't know" target base when xu is absent),
    ``dXu = inv(YtY) (dQui * yi)`` as one [B,k]x[k,k] GEMM, ``newXu = xu + dXu``.
    Returns (new vectors fp32 [B,k], valid mask [B]); invalid rows had no target.
    """
    xu64 = xu.to(torch.float64)
    yi64 = yi.to(torch.float64)
    # the reference computes dot() with float products accumulated in double
    qui = (xu.to(torch.float32) * yi.to(torch.float32)).to(torch.float64).sum(1)
    qui = torch.where(xu_present, qui, torch.zeros_like(qui))
    base = torch.where(xu_present, qui, torch.full_like(qui, 0.5))
    tgt = target_qui(implicit, values, base)
    valid = ~torch.isnan(tgt)
    dq = torch.where(valid, tgt - qui, torch.zeros_like(tgt))
    # Java's dQuiYi[i] *= dQui: float times double, evaluated and rounded once in double
    rhs = (yi.to(torch.float32).to(torch.float64) * dq[:, None]).to(torch.float32).to(
        torch.float64)
    dx = rhs.matmul(solver_inv.to(torch.float64).t())
    dx32 = dx.to(torch.float32)
    new = torch.where(xu_present[:, None], (xu.to(torch.float32) + dx32), dx32)
    return new, valid
