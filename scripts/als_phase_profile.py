#!/usr/bin/env python3
"""Per-phase cycle breakdown of the ALS wave kernel (rank 64) on the bench's data shape.

Runs ``oryx_als_solve_profile64`` (als_solve_wave<64, PROF=true>: s_memtime stamps per row)
on the user and item CSRs of bench.py's synthetic problem and prints, per half-step, the
average shader-clock cycles per row spent in each phase.  GPU only.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BATCH_PHASES = ["batch setup", "gather+mfma (all rows of the batch)", "normal equations",
                "LDL^T 16x16 blocks", "K + trailing MFMA + rhs", "back substitution + store"]
# ORYX_PROF_K=128 [ORYX_PROF_PRECISION=fp32]: the rank-128 LDS-DMA batched kernel
# (als_solve_batch_gl<128, split, PROF>) instead of the rank-64 register kernel
K = int(os.environ.get("ORYX_PROF_K", "64"))
PRECISION = os.environ.get("ORYX_PROF_PRECISION", "bf16")
if os.environ.get("ORYX_ALS_VARIANT", "3") == "1":   # als_solve_wave (register Cholesky)
    PHASES = ["gather+mfma", "scatter/ws", "load A+YtY", "cholesky", "forward", "back+store"]
else:                                               # als_solve_panel (default)
    PHASES = ["gather+mfma+b", "-", "panel to/from LDS (+YtY, diag)",
              "panel elimination + forward", "trailing MFMA update", "back+store"]


def main():
    import bench
    from oryx_amd import native
    from oryx_amd.models.als.trainer import ALSTrainer
    from oryx_amd.ops import als as als_ops
    from oryx_amd.parallel import dist

    dev = torch.device("cuda", 0)
    ctx = dist.DistContext(device=dev)
    users, items, strength = bench._gen_ratings(162_541, 59_047, 25_000_000, 0, 1234, dev)
    tr = ALSTrainer(K, lam=0.001, alpha=1.0, implicit=True, ctx=ctx, seed=1, precision=PRECISION)
    tr.prepare(users, items, strength, 162_541, 59_047)
    tr.init_factors()
    lib = native.require_kernels()
    out = {}
    if lib.oryx_als_get_variant() == 5:
        # als_solve_batch<64, PROF>: the real half-step (split long rows included); cycles of
        # one wave (= one SIMD) per batch of 4 rows
        for name, csr, src_b, src_f, dst, dstb in (
                ("items", tr.csr_i, tr.Xb, tr.X, tr.Y, tr.Yb_local),
                ("users", tr.csr_u, tr.Yb, tr.Y, tr.X, tr.Xb_local)):
            yty = als_ops.gramian(src_f)
            prof = torch.zeros(10, dtype=torch.int64, device=dev)
            lib.oryx_als_batch_profile(prof.data_ptr())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            als_ops.solve_rows(csr, src_b, yty, dst, dstb, K, 0.001, 1.0, True,
                               split=tr.split)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            lib.oryx_als_batch_profile(None)
            p = prof.cpu().tolist()
            nb = max(1, p[6])
            out[name] = {"rows": int(csr.order.numel()), "batches": p[6], "nnz": csr.nnz,
                         "ms": ms, "cycles_per_batch": {k: p[i] / nb
                                                        for i, k in enumerate(BATCH_PHASES)}}
            if K > 64:   # the LDS-DMA kernel also splits its gather phase
                out[name]["gather_dma_wait_cycles_per_batch"] = p[7] / nb
                out[name]["gather_dma_issue_cycles_per_batch"] = p[8] / nb
        out["k"], out["precision"] = K, PRECISION
        print(json.dumps(out, indent=1))
        return
    for name, csr, src_b, src_f, dst in (("items", tr.csr_i, tr.Xb, tr.X, tr.Y),
                                         ("users", tr.csr_u, tr.Yb, tr.Y, tr.X)):
        yty = als_ops.gramian(src_f)
        prof = torch.zeros(6, dtype=torch.int64, device=dev)
        # unsplit: every row on one wave, so phase 0 includes the long rows' tails
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = lib.oryx_als_solve_profile64(csr.row_ptr.data_ptr(), csr.order.data_ptr(),
                                          csr.cols.data_ptr(), csr.vals.data_ptr(),
                                          src_b.data_ptr(), yty.data_ptr(), dst.data_ptr(),
                                          int(csr.order.numel()), 64, 0.001, 1.0, 1,
                                          int(os.environ.get("ORYX_ALS_VARIANT", "1")),
                                          prof.data_ptr(), native.stream_ptr(dev))
        native.check(rc, "profile")
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        n = int(csr.order.numel())
        p = prof.cpu().tolist()
        out[name] = {"rows": n, "nnz": csr.nnz, "ms": ms,
                     "cycles_per_row": {k: p[i] / n for i, k in enumerate(PHASES)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
