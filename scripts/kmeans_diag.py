#!/usr/bin/env python3
"""k-means init / empty-cluster diagnostic on the bench_kmeans data (one GPU): k-means|| init
time, then Lloyd steps reporting empty clusters, and for every empty center its distance to
the nearest other center and to the nearest point (JSON lines)."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=12_500_000)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--init-precision", default="bf16")
    args = ap.parse_args()
    from oryx_amd.ops import kmeans as km
    from oryx_amd.parallel import dist
    dev = torch.device("cuda")
    n, d, k = args.points, args.dim, args.k
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed)
    true_c = torch.randn((k, d), generator=g, device=dev) * 4.0
    g.manual_seed(args.seed * 7919 + 1)
    x = torch.empty((n, d), dtype=torch.float32, device=dev)
    for lo in range(0, n, 1 << 20):
        hi = min(n, lo + (1 << 20))
        lab = torch.randint(0, k, (hi - lo,), generator=g, device=dev)
        x[lo:hi] = true_c[lab] + torch.randn((hi - lo, d), generator=g, device=dev)
    pts = km.PointSet(x)
    ctx = dist.DistContext(device=dev)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        centers = km.init_centers(pts, k, "k-means||", seed=args.seed, ctx=ctx,
                                  precision=args.init_precision)
        torch.cuda.synchronize()
        init_ms = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"init_ms": init_ms, "rep": rep}), flush=True)
    cd = torch.cdist(centers, centers)
    cd.fill_diagonal_(float("inf"))
    print(json.dumps({"min_center_gap": float(cd.min()),
                      "duplicate_pairs": int((cd < 1e-3).sum()) // 2}), flush=True)
    for it in range(args.steps):
        new, counts, d2, ne = km.lloyd_step(pts, centers, ctx, None, "fp32")
        rec = {"step": it, "empty": ne}
        if ne:
            e = torch.nonzero(counts == 0).flatten()
            dd = torch.cdist(centers[e], centers)
            dd[torch.arange(len(e)), e] = float("inf")
            near_pt = torch.cdist(centers[e], x[:2_000_000]).min(1).values
            rec.update({"empty_ids": e[:10].tolist(),
                        "gap_to_other_center": dd.min(1).values[:10].tolist(),
                        "nearest_point_dist_2M": near_pt[:10].tolist()})
        print(json.dumps(rec), flush=True)
        centers = new
    return 0


if __name__ == "__main__":
    sys.exit(main())
