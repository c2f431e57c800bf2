#!/usr/bin/env python3
"""k-means batch-layer benchmark on MI355X (BASELINE.json config "k-means k=1000 d=256 on
100M points, 8xMI355X (MFMA distance + centroid all-reduce)").

``python bench_kmeans.py --gpus N --steps K --warmup W`` (N > 1: one rank per GPU under
``torch.distributed.run``; without an external launcher the script starts them itself).  A
*step* is one Lloyd iteration of the batch layer's k-means trainer
(``oryx_amd.ops.kmeans.lloyd_step``, the loop MLlib runs for the reference at
``[mllib]/kmeans/KMeansUpdate.java:116-117``): the fused MFMA distance + argmin kernel over
every point against all K centers (``--precision fp32``, the default since the BASELINE config
names no reduced dtype: the certified kernel whose ambiguous points are re-decided in fp32,
i.e. the fp32 argmin; ``bf16``: the plain bf16 argmin), the fp32 centroid accumulation
kernel, ONE RCCL all-reduce of the K x (d + 1) sums/counts, and the center move.

Weak scaling: every rank owns 100M / 8 = 12.5M points (the 8-GPU config's per-GPU share), so
N = 8 is exactly the BASELINE config.  Data: a synthetic Gaussian mixture (1000 true centers,
d = 256, fp32 resident in HBM); centers start from k-means|| (the app's default init, timed
separately as ``init_ms``; ``--init sample`` starts from a random sample instead).  The reference publishes no batch-layer numbers, so
``vs_baseline`` is null.  Prints ONE JSON line (rank 0): ``value`` = points processed per
second over all ranks; ``tflops`` = the distance-GEMM work rate (2 * n * K * d per point set).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def _speed_latency(centers, counts, true_c, events: int, dev) -> dict:
    """The k-means speed layer on the trained model: ``events`` new points (CSV lines from
    the same mixture) per micro-batch, build + append of the cluster updates."""
    import shutil
    import tempfile
    import numpy as np
    from oryx_amd.api import Dataset
    from oryx_amd.layers.speed import measure_intervals
    from oryx_amd.models.kmeans.common import ClusterInfo
    from oryx_amd.models.kmeans.speed import KMeansSpeedModel, KMeansSpeedModelManager
    from oryx_amd.textlines import TextLines
    from oryx_amd.transport.producer import LogTopicProducer
    from oryx_amd.utils import config as cfg
    k, d = centers.shape
    conf = cfg.overlay_on({
        "oryx.input-schema.feature-names": "[%s]" % ",".join('"f%d"' % j for j in range(d)),
        "oryx.input-schema.categorical-features": "[]"}, cfg.get_default())
    mgr = KMeansSpeedModelManager(conf)
    c_h = centers.double().cpu().numpy()
    n_h = counts.cpu().numpy()
    mgr.model = KMeansSpeedModel([ClusterInfo(j, c_h[j], max(1, int(n_h[j])))
                                  for j in range(k)], dev)
    g = np.random.default_rng(11)
    tc = true_c.cpu().numpy()
    pts = tc[g.integers(0, k, events)] + g.standard_normal((events, d))
    lines = [",".join("%.6f" % v for v in row) for row in pts]
    ds = Dataset.from_values(TextLines.from_strings(lines))
    logdir = tempfile.mkdtemp(prefix="oryx_bench_kmeans_speed_")
    producer = LogTopicProducer("log:" + logdir, "OryxUpdate", async_=False,
                                max_message=1 << 30)
    try:
        return measure_intervals(mgr, ds, producer, reps=12, warmup=2)
    finally:
        producer.close()
        shutil.rmtree(logdir, ignore_errors=True)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--points-per-gpu", type=int, default=12_500_000)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--init", choices=["k-means||", "sample"], default="k-means||")
    ap.add_argument("--speed-events", type=int, default=10_000,
                    help="speed-layer micro-batch size timed against the trained centers "
                         "(0: skip)")
    args = ap.parse_args(argv)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oryx_amd.parallel import launch
    rc = launch.relaunch_if_needed(os.path.abspath(__file__), argv, args.gpus)
    if rc is not None:
        return rc
    from oryx_amd.parallel import dist
    from oryx_amd.ops import kmeans as km

    ctx = dist.init_from_env(device=args.device)
    dev = ctx.device
    W = ctx.world_size
    n, d, k = args.points_per_gpu, args.dim, args.k

    g = torch.Generator(device=dev)
    g.manual_seed(args.seed)            # the same true centers on every rank
    true_c = torch.randn((k, d), generator=g, device=dev) * 4.0
    g.manual_seed(args.seed * 7919 + ctx.rank + 1)
    x = torch.empty((n, d), dtype=torch.float32, device=dev)
    chunk = 1 << 20
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        lab = torch.randint(0, k, (hi - lo,), generator=g, device=dev)
        x[lo:hi] = true_c[lab] + torch.randn((hi - lo, d), generator=g, device=dev)
    pts = km.PointSet(x)
    init_ms = None
    if args.init == "sample":
        # initial centers: a random sample of rank 0's points, broadcast
        idx = torch.randperm(n, generator=g, device=dev)[:k]
        centers = x[idx].clone()
        if ctx.is_distributed:
            torch.distributed.broadcast(centers, src=0)
    else:
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dist.barrier(ctx)
        t_init = time.perf_counter()
        centers = km.init_centers(pts, k, "k-means||", seed=args.seed, ctx=ctx)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        init_ms = (time.perf_counter() - t_init) * 1e3
    ws = None
    if pts.xb is not None:
        ws = (torch.empty(n, dtype=torch.int32, device=dev),
              torch.empty(n, dtype=torch.float32, device=dev))

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dist.barrier(ctx)

    empties = 0
    for _ in range(args.warmup):
        centers, counts, _, ne = km.lloyd_step(pts, centers, ctx, ws, args.precision)
    sync()
    km.CERT_STATS.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        centers, counts, _, ne = km.lloyd_step(pts, centers, ctx, ws, args.precision)
        empties += ne
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if ctx.is_distributed:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    total_points = n * W * args.steps
    ms = elapsed / args.steps * 1e3
    total_counts = int(counts.sum().item())
    st = km.CERT_STATS.get(dev)
    rescored = None if st is None else [v / args.steps for v in st.tolist()]
    info = dist.run_info(ctx)
    speed = None
    if ctx.is_main and args.speed_events > 0:
        speed = _speed_latency(centers, counts, true_c, args.speed_events, dev)
    if ctx.is_main:
        print(json.dumps({
            "world_size": info["world_size"], "backend": info["backend"],
            "rank_devices": [r.get("current_device", r["device"]) for r in info["ranks"]],
            "metric": "k-means Lloyd-iteration points/sec (batch layer), 1/2/4/8 MI355X",
            "value": total_points / elapsed, "unit": "points/s", "n_gpus": W,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.precision,
            "dtype_detail": ("fp32 argmin: bf16 MFMA scan certified by rounding bounds, "
                             "ambiguous points re-decided from fp32 rows" if args.precision ==
                             "fp32" else "bf16 MFMA distances") + ", fp32 sums",
            "data": "synthetic Gaussian mixture (1000 true centers), %s init" % args.init,
            "config": {"model": "k-means k=%d d=%d" % (k, d), "global_batch": n * W,
                       "seq_len": None, "parallelism": "dp%d (point shards, RCCL all-reduce "
                       "of K x (d+1) sums/counts)" % W, "points_per_gpu": n,
                       "step": "1 Lloyd iteration (assign + accumulate + all-reduce + move)"},
            "tflops": 2.0 * n * W * k * d / (ms * 1e-3) / 1e12,
            "counted_points": total_counts, "empty_clusters_seen": empties,
            "init_ms": init_ms, "rescored_points_per_step": rescored,
            "speed_layer_update_ms": speed["median_ms"] if speed else None,
            "speed_layer_update_p90_ms": speed["p90_ms"] if speed else None,
            "speed_layer_phase_ms": speed.get("phase_ms") if speed else None,
            "speed_layer_reps": speed["reps"] if speed else None,
            "speed_layer_events": args.speed_events,
            "speed_layer_messages": speed["messages"] if speed else None,
            "speed_layer_path": "KMeansSpeedModelManager.build_updates against the trained "
                                "centers + the UP messages' append to an update log, end to "
                                "end (layers/speed.measure_intervals)",
        }), flush=True)
    if ctx.is_distributed:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
