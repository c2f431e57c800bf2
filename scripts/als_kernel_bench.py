#!/usr/bin/env python3
"""Per-half-step timing of the ALS solve kernel on bench.py's synthetic problem (1 GPU).

Prints JSON: milliseconds per call (median of ``--reps``) of the item and user solves
(``als_ops.solve_rows``: als_partial + the solve kernel) and of the Gramians, measured with
HIP events around each launch.  ``ORYX_ALS_VARIANT=1`` selects the register-Cholesky kernel.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank-k", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--precision", choices=["bf16", "fp32"], default="bf16")
    args = ap.parse_args()
    import bench
    from oryx_amd.models.als.trainer import ALSTrainer
    from oryx_amd.ops import als as als_ops
    from oryx_amd.parallel import dist

    dev = torch.device("cuda", 0)
    ctx = dist.DistContext(device=dev)
    users, items, strength = bench._gen_ratings(162_541, 59_047, 25_000_000, 0, 1234, dev)
    tr = ALSTrainer(args.rank_k, lam=0.001, alpha=1.0, implicit=True, ctx=ctx, seed=1,
                    precision=args.precision)
    tr.prepare(users, items, strength, 162_541, 59_047)
    tr.init_factors()
    tr.iterate(1)

    def timed(fn):
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return statistics.median(ts)

    out = {"k": args.rank_k, "precision": args.precision,
           "variant": os.environ.get("ORYX_ALS_VARIANT", "5"),
           "wide_variant": os.environ.get("ORYX_ALS_WIDE_VARIANT", "2")}
    yty_x = als_ops.gramian(tr.X)
    yty_y = als_ops.gramian(tr.Y)
    out["gramian_users_ms"] = timed(lambda: als_ops.gramian(tr.X))
    out["gramian_items_ms"] = timed(lambda: als_ops.gramian(tr.Y))
    out["solve_items_ms"] = timed(lambda: als_ops.solve_rows(
        tr.csr_i, tr.Xb, yty_x, tr.Y, tr.Yb_local, tr.k, tr.lam, tr.alpha, True,
        fail_count=tr.fail_count, split=tr.split))
    out["solve_users_ms"] = timed(lambda: als_ops.solve_rows(
        tr.csr_u, tr.Yb, yty_y, tr.X, tr.Xb_local, tr.k, tr.lam, tr.alpha, True,
        fail_count=tr.fail_count, split=tr.split))
    out["items_long_rows"] = tr.csr_i.n_long
    out["items_segments"] = tr.csr_i.n_seg
    out["iteration_ms"] = timed(lambda: tr.iterate(1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
