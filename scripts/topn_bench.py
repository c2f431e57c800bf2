#!/usr/bin/env python3
"""Serving scan microbenchmark (no HTTP): ``ALSServingModel.top_n`` and ``ItemIndex.scan`` on
an ``--items`` x ``--features`` model, per request shape, plus the HBM the model holds.

``python scripts/topn_bench.py --items 20000000 --features 250 [--sample-rate 1.0]``
Prints one JSON line.  Factors are random Gaussians generated on the GPU (the host copy the
feature store keeps is filled from them in chunks).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _timed(fn, reps):
    import torch
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts)), float(np.min(ts))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=20_000_000)
    ap.add_argument("--features", type=int, default=250)
    ap.add_argument("--sample-rate", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from oryx_amd.models.als.serving import ALSServingModel
    from oryx_amd.ops import topn
    dev = torch.device("cuda")
    n, k = args.items, args.features
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    t0 = time.perf_counter()
    m = ALSServingModel(k, True, args.sample_rate, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    chunk = 1 << 21
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        part = torch.randn((hi - lo, k), generator=g, device=dev).cpu().numpy()
        m.Y.set_vectors(["I%d" % i for i in range(lo, hi)], part)
        print(json.dumps({"loaded": hi}), flush=True)
    load_s = time.perf_counter() - t0
    tq = torch.randn((16, k), generator=g, device=dev).cpu().numpy()
    t0 = time.perf_counter()
    m.top_n(tq[0], 10)
    first_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    hbm = (torch.cuda.memory_allocated() - base) / 2**30
    idx = m.index
    lsh_on = m.lsh.get_max_bits_differing() < m.lsh.get_num_hashes()

    def q(j, hm, cos=False):
        c = m.lsh.get_candidate_indices(tq[j]) if lsh_on else None
        return topn.TopNQuery(tq[j], hm, cos, c, None)

    out = {"items": n, "features": k, "sample_rate": args.sample_rate,
           "model_hbm_gib": hbm, "store_mirror_gib":
           float(m.Y._dev.numel() * 4) / 2**30, "index_borrowed": bool(idx.borrowed),
           "load_s": load_s, "first_query_s": first_s}
    shapes = {
        "scan_1q_top10": lambda: idx.scan([q(0, 10)]),
        "scan_1q_top10_cosine": lambda: idx.scan([q(0, 10, True)]),
        "scan_16q_top10": lambda: idx.scan([q(j, 10) for j in range(16)]),
        "scan_1q_top100": lambda: idx.scan([q(0, 100)]),
        "scan_1q_top500": lambda: idx.scan([q(0, 500)]),
        "scan_1q_top2000": lambda: idx.scan([q(0, 2000)]),
        "top_n_1q_top10": lambda: m.top_n(tq[1], 10),
        "all_scores_1q": lambda: idx.all_scores(tq[0], False),
    }
    for name, fn in shapes.items():
        fn()
        med, best = _timed(fn, args.reps)
        out[name + "_ms"] = med
        out[name + "_min_ms"] = best
        print(json.dumps({name: med}), flush=True)
    bytes_read = n * idx.kp * 4 * (args.sample_rate if lsh_on else 1.0)
    out["scan_1q_top10_effective_gbps"] = bytes_read / (out["scan_1q_top10_min_ms"] * 1e-3) / 1e9
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
