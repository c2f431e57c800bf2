#!/usr/bin/env python3
"""Random-decision-forest benchmark on MI355X (BASELINE.json config "Random-decision-forest
50Mx100 features + Kafka speed-layer incremental updates, 8xMI355X").

``python bench_rdf.py --gpus N --steps K --warmup W`` (N > 1: one rank per GPU under
``torch.distributed.run``).  A *step* trains one whole forest with the batch layer's trainer
(``oryx_amd.ops.rdf.train_forest``; the reference runs MLlib ``RandomForest.trainClassifier``
at ``[mllib]/rdf/RDFUpdate.java:143-165``): reference defaults num-trees = 20, max-depth = 8,
max-split-candidates = 100, impurity = entropy, "auto" feature subsets (sqrt(100) = 10 per
node), Poisson bootstrap -- every level of all 20 trees is one HIP histogram pass (LDS-
privatised at the top levels), one RCCL all-reduce of the level histograms, the split
search, and one HIP routing pass.

Weak scaling: every rank owns 50M / 8 = 6.25M examples x 100 numeric features (the 8-GPU
config's per-GPU share), binned once to uint8 before timing (as the batch layer does once
per generation).  Labels: 2 classes from a noisy linear rule over 8 of the features.
The speed-layer half of the metric: the real ``RDFSpeedModelManager.build_updates`` on a
``--speed-events`` micro-batch of text input lines against the trained forest (PMML round
trip included), reported as ``speed_layer_update_ms``.  Prints ONE JSON line (rank 0);
``value`` = training examples per second over all ranks (examples x 1 forest / step time).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch


def _speed_latency(trained, data, schema_cfg, events: int, P: int, dev) -> float:
    from oryx_amd.api import Dataset, KeyMessage
    from oryx_amd.models.rdf import pmml as rdf_pmml
    from oryx_amd.models.rdf.batch import _to_spec
    from oryx_amd.models.rdf.speed import RDFSpeedModelManager
    from oryx_amd.models.schema import CategoricalValueEncodings, InputSchema
    from oryx_amd.utils import pmml as pmmlu

    schema = InputSchema(schema_cfg)
    enc = CategoricalValueEncodings({P: ["0", "1"]})
    roots = [_to_spec(r, data, schema, True) for r in trained.roots]
    imp = trained.predictor_counts / max(1.0, trained.predictor_counts.sum())
    doc = rdf_pmml.forest_to_pmml(roots, schema, enc, imp, 8, 100, "entropy")
    mgr = RDFSpeedModelManager(schema_cfg)
    mgr.device = dev
    mgr.consume([KeyMessage("MODEL", pmmlu.to_string(doc))])
    rng = np.random.default_rng(7)
    xs = rng.standard_normal((events, P))
    lines = [",".join("%.6f" % v for v in row) + "," + str(int(row[0] > 0)) for row in xs]
    from oryx_amd.layers.speed import measure_intervals
    from oryx_amd.textlines import TextLines
    from oryx_amd.transport.producer import LogTopicProducer
    import shutil
    import tempfile
    ds = Dataset.from_values(TextLines.from_strings(lines))
    logdir = tempfile.mkdtemp(prefix="oryx_bench_rdf_speed_")
    producer = LogTopicProducer("log:" + logdir, "OryxUpdate", async_=False,
                                max_message=1 << 30)
    try:
        # build + append of the UP messages, median / p90 of 12 after 2 warm-ups
        r = measure_intervals(mgr, ds, producer, reps=12, warmup=2)
    finally:
        producer.close()
        shutil.rmtree(logdir, ignore_errors=True)
    assert r["messages"], "speed layer produced no updates"
    return r


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--examples-per-gpu", type=int, default=6_250_000)
    ap.add_argument("--features", type=int, default=100)
    ap.add_argument("--trees", type=int, default=20)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--bins", type=int, default=100)
    ap.add_argument("--speed-events", type=int, default=10_000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--device", default="auto")
    args = ap.parse_args(argv)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oryx_amd.parallel import launch
    rc = launch.relaunch_if_needed(os.path.abspath(__file__), argv, args.gpus)
    if rc is not None:
        return rc
    from oryx_amd.parallel import dist
    from oryx_amd.ops import rdf as rdf_ops
    from oryx_amd.utils import config as cfg

    ctx = dist.init_from_env(device=args.device)
    dev = ctx.device
    W = ctx.world_size
    n, P = args.examples_per_gpu, args.features

    g = torch.Generator(device=dev)
    g.manual_seed(args.seed * 7919 + ctx.rank + 1)
    X = torch.randn((n, P), generator=g, device=dev)
    wv = torch.zeros(P, device=dev)
    wv[:8] = torch.tensor([1.0, -0.8, 0.6, 0.5, -0.4, 0.3, 0.25, -0.2], device=dev)
    y = ((X @ wv + 0.3 * torch.randn(n, generator=g, device=dev)) > 0).to(torch.int32)
    # identical bins on every rank: thresholds from rank 0's sample, broadcast implicitly by
    # using the same seeded sample source (the first 200k rows of a shared-seed generator)
    gs = torch.Generator(device=dev)
    gs.manual_seed(args.seed)
    thr_src = torch.randn((200_000, P), generator=gs, device=dev)
    data = rdf_ops.bin_features(X, [False] * P, [0] * P, args.bins, dev, seed=args.seed,
                                threshold_source=thr_src)
    del X

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dist.barrier(ctx)

    trained = None
    for i in range(args.warmup):
        trained = rdf_ops.train_forest(data, y, 2, args.trees, args.depth, "entropy",
                                       seed=args.seed + i, ctx=ctx)
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        trained = rdf_ops.train_forest(data, y, 2, args.trees, args.depth, "entropy",
                                       seed=args.seed + 100 + i, ctx=ctx)
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if ctx.is_distributed:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3

    def count_nodes(nd):
        return 1 + (count_nodes(nd.left) + count_nodes(nd.right) if nd.feature >= 0 else 0)

    speed_ms = None
    info = dist.run_info(ctx)
    if ctx.is_main:
        names = ",".join('"%d"' % i for i in range(P + 1))
        schema_cfg = cfg.overlay_on({
            "oryx.input-schema.feature-names": "[%s]" % names,
            "oryx.input-schema.categorical-features": '["%d"]' % P,
            "oryx.input-schema.target-feature": '"%d"' % P}, cfg.get_default())
        speed = None
        if args.speed_events > 0:
            speed = _speed_latency(trained, data, schema_cfg, args.speed_events, P, dev)
            speed_ms = speed["median_ms"]
        print(json.dumps({
            "metric": "RDF batch-layer training examples/sec + speed-layer update latency, "
                      "1/2/4/8 MI355X",
            "value": n * W * args.steps / elapsed, "unit": "examples/s", "n_gpus": W,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32 histograms (uint8 bins)",
            "data": "synthetic Gaussian features, 2 classes from a noisy linear rule",
            "config": {"model": "RDF classification trees=%d depth=%d bins=%d entropy" % (
                args.trees, args.depth, args.bins), "global_batch": n * W, "seq_len": None,
                "parallelism": "dp%d (example shards, RCCL all-reduce of level histograms)" % W,
                "examples_per_gpu": n, "features": P,
                "step": "1 full forest (all levels of all trees)"},
            "world_size": info["world_size"], "backend": info["backend"],
            "rank_devices": [r.get("current_device", r["device"]) for r in info["ranks"]],
            "nodes": sum(count_nodes(r) for r in trained.roots),
            "speed_layer_update_ms": speed_ms, "speed_layer_events": args.speed_events,
            "speed_layer_update_p90_ms": speed["p90_ms"] if speed else None,
            "speed_layer_phase_ms": speed.get("phase_ms") if speed else None,
            "speed_layer_reps": speed["reps"] if speed else None,
            "speed_layer_messages": speed["messages"] if speed else None,
            "speed_layer_path": "RDFSpeedModelManager.build_updates + the UP messages' append "
                                "to an update log, end to end (layers/speed.measure_intervals)",
        }), flush=True)
    if ctx.is_distributed:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
