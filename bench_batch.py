#!/usr/bin/env python3
"""End-to-end batch-layer benchmark: input log -> published ALS ``MODEL`` + ``UP`` rows.

Where ``bench.py`` times the trainer's iterations on device-generated data, this times the
whole generation the reference's batch layer runs (``[lambda]/batch/BatchUpdateFunction.java:
86-155`` -> ``[mllib]/als/ALSUpdate.java:100-230``): ``--ratings`` synthetic
``user,item,strength,timestamp`` lines are appended to the input log, then ONE
``BatchLayer.run_interval`` drains them, parses (native), aggregates per (user, item) in time
order, builds the CSRs, trains ALS on the GPU, writes ``X/`` / ``Y/`` and the PMML, saves the
interval's data, publishes ``MODEL`` and every ``UP`` row.  Phase seconds come from the
layer / ``ALSUpdate`` timers.

``python bench_batch.py --ratings 25000000 --gpus 1``; ``--gpus N`` runs N ranks (sharded
generations: each rank reads its share of the input partitions).  Prints one JSON line
(rank 0): ``value`` = ratings per second from log to published model.
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def _cprofile_top(prof, n: int = 30):
    """The n functions with the most cumulative and the most own time."""
    import pstats
    st = pstats.Stats(prof)
    rows = []
    for (fn, line, name), (cc, nc, tt, ct, _) in st.stats.items():
        rows.append((ct, tt, nc, "%s:%d(%s)" % (os.path.relpath(fn, ROOT)
                                                  if fn.startswith(ROOT) else fn, line, name)))
    def fmt(rs):
        return [{"cum_s": round(r[0], 4), "own_s": round(r[1], 4), "calls": r[2], "fn": r[3]}
                for r in rs]
    return {"by_cumulative": fmt(sorted(rows, reverse=True)[:n]),
            "by_own": fmt(sorted(rows, key=lambda r: -r[1])[:n])}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--ratings", type=int, default=25_000_000)
    ap.add_argument("--users", type=int, default=162_541)
    ap.add_argument("--items", type=int, default=59_047)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--iterations", type=int, default=10)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--dir", default=None, help="work dir (default: a fresh temp dir)")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--generations", type=int, default=1,
                    help="generations to run (1 GPU): generation g > 1 appends --next-ratings "
                         "new ratings and trains on them plus all earlier ones (the past part "
                         "files -- the resident parsed history's steady state)")
    ap.add_argument("--next-ratings", type=int, default=1_000_000)
    ap.add_argument("--no-warm-up", action="store_true",
                    help="skip the batch layer's start-up warm-up (first-call costs then land "
                         "in the first generation)")
    ap.add_argument("--cprofile", action="store_true",
                    help="profile the first generation's host side (cProfile): the top "
                         "functions by cumulative time go into the record")
    ap.add_argument("--test-fraction", type=float, default=None,
                    help="oryx.ml.eval.test-fraction (the reference default is 0.1: the newest "
                         "tenth of the interval's data is held out and evaluated); default 0.0 "
                         "for ALS, 0.1 for k-means and RDF")
    ap.add_argument("--app", default="als", choices=["als", "kmeans", "rdf"],
                    help="als (default), kmeans (BASELINE config #4's per-GPU share: "
                         "--points 12.5M x --dims 256, k 1000) or rdf (config #5's per-GPU "
                         "share: --points 6.25M x --dims 100 predictors)")
    ap.add_argument("--points", type=int, default=None)
    ap.add_argument("--dims", type=int, default=None)
    ap.add_argument("--k", type=int, default=1000, help="k-means clusters")
    ap.add_argument("--trees", type=int, default=20, help="RDF trees")
    ap.add_argument("--depth", type=int, default=8, help="RDF max depth")
    ap.add_argument("--chunk", type=int, default=1 << 20, help="generated rows per append")
    args = ap.parse_args(argv)
    if args.test_fraction is None:
        args.test_fraction = 0.0 if args.app == "als" else 0.1
    if args.app == "kmeans":
        args.points = args.points or 12_500_000
        args.dims = args.dims or 256
    elif args.app == "rdf":
        args.points = args.points or 6_250_000
        args.dims = args.dims or 100

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oryx_amd.parallel import launch
    rc = launch.relaunch_if_needed(os.path.abspath(__file__), argv, args.gpus)
    if rc is not None:
        return rc
    import numpy as np
    import torch
    from oryx_amd.layers.batch import BatchLayer
    from oryx_amd.parallel import dist
    from oryx_amd.transport import log as tlog
    from oryx_amd.utils import config as cfg

    ctx = dist.init_from_env(device=args.device)
    work = args.dir
    if work is None:
        work = dist.broadcast_object(tempfile.mkdtemp(prefix="oryx_bench_batch_")
                                     if ctx.is_main else None, ctx)
    base = {
        "oryx.input-topic.broker": "log:" + work + "/log",
        "oryx.update-topic.broker": "log:" + work + "/log",
        "oryx.input-topic.partitions": args.partitions,
        "oryx.input-topic.message.max-size": 1 << 30,
        "oryx.update-topic.message.max-size": 1 << 30,
        "oryx.batch.storage.data-dir": work + "/data",
        "oryx.batch.storage.model-dir": work + "/model",
        "oryx.ml.eval.candidates": 1,
        "oryx.ml.eval.test-fraction": args.test_fraction,
        "oryx.gpu.device": args.device,
        "oryx.gpu.dtype": args.dtype,
    }
    if args.app == "als":
        base.update({
            "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.als.ALSUpdate",
            "oryx.als.hyperparams.features": args.features,
            "oryx.als.iterations": args.iterations,
            "oryx.als.implicit": "true"})
    elif args.app == "kmeans":
        base.update({
            "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.kmeans.KMeansUpdate",
            "oryx.input-schema.num-features": args.dims,
            "oryx.input-schema.categorical-features": "[]",
            "oryx.kmeans.hyperparams.k": args.k,
            "oryx.kmeans.iterations": args.iterations,
            "oryx.kmeans.runs": 1,
            "oryx.kmeans.evaluation-strategy": "SILHOUETTE",
            "oryx.gpu.dtype": "fp32"})
    else:
        base.update({
            "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.rdf.RDFUpdate",
            "oryx.input-schema.num-features": args.dims + 1,
            "oryx.input-schema.target-feature": '"%d"' % args.dims,
            "oryx.input-schema.categorical-features": '["%d"]' % args.dims,
            "oryx.rdf.num-trees": args.trees,
            "oryx.rdf.hyperparams.max-depth": args.depth,
            "oryx.rdf.hyperparams.max-split-candidates": 32,
            "oryx.rdf.hyperparams.impurity": "gini"})
    conf = cfg.overlay_on(base, cfg.get_default())
    layer = BatchLayer(conf)
    t_ingest = 0.0
    if ctx.is_main:
        layer._context = layer.layer_context()
        layer._update = layer.load_update_instance()
        layer.build_input_consumer()
        # what BatchLayer.start does before its first interval (outside the timed generation,
        # reported as startup_warm_up_s)
        if not args.no_warm_up:
            layer.warm_up()
        rng = np.random.default_rng(7)
        now = int(time.time() * 1000)

        def append_features(n_total, now):
            """k-means / RDF input generated on the device and formatted there as CSV lines
            (values on a 0.01 grid): chunks appended round-robin over the partitions."""
            from oryx_amd.ops import textfmt
            from oryx_amd.api import MessageBlock
            dev = ctx.device
            g = torch.Generator(device=dev)
            g.manual_seed(7)
            topic = tlog.Topic(work + "/log", "OryxInput")
            if args.app == "kmeans":
                centers = torch.randn(args.k, args.dims, generator=g, device=dev) * 10
            for j, lo in enumerate(range(0, n_total, args.chunk)):
                m = min(args.chunk, n_total - lo)
                if args.app == "kmeans":
                    c = torch.randint(0, args.k, (m,), generator=g, device=dev)
                    x = centers[c] + torch.randn(m, args.dims, generator=g, device=dev)
                else:
                    f = torch.randn(m, args.dims, generator=g, device=dev)
                    y = ((f[:, 0] + f[:, 1] * f[:, 2] + 0.3 * f[:, 3]) > 0).float()
                    x = torch.cat([f, y[:, None]], 1)
                x = torch.round(x * 100) / 100
                if dev.type == "cuda":
                    rows = textfmt.format_csv(x)
                    blk = MessageBlock(rows.blob, rows.ends - 1)
                    topic.append_block(blk, partition=j % args.partitions,
                                       timestamp_ms=now)
                else:
                    xs = x.cpu().numpy()
                    lines = [",".join("%g" % v for v in row) for row in xs]
                    topic.append_values(lines, partition=j % args.partitions,
                                        timestamp_ms=now)
            topic.close()

        def append(n_total, now):
            if args.app != "als":
                return append_features(n_total, now)
            topic = tlog.Topic(work + "/log", "OryxInput")
            chunk = 1 << 20
            for lo in range(0, n_total, chunk):
                n = min(chunk, n_total - lo)
                u = (args.users * rng.random(n) ** 1.3).astype(np.int64)
                it = (args.items * rng.random(n) ** 2.5).astype(np.int64)
                s = rng.integers(1, 11, n) * 0.5
                ts = now - rng.integers(0, 86_400_000, n)
                lines = ["%d,%d,%.1f,%d" % row for row in zip(u.tolist(), it.tolist(),
                                                             s.tolist(), ts.tolist())]
                topic.append_batch([(None, l) for l in lines])
            topic.close()

        t0 = time.perf_counter()
        n_records = args.ratings if args.app == "als" else args.points
        append(n_records, now)
        t_ingest = time.perf_counter() - t0
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier(ctx)
        # cyclic-GC passes inside the generation (a gen-2 pass stops the interpreter for as
        # long as its walk over every tracked object takes)
        import gc
        gc_ms = {"n": 0, "total_ms": 0.0, "max_ms": 0.0}
        gc_t = [None]

        def _gc_cb(phase, info):
            if phase == "start":
                gc_t[0] = time.perf_counter()
            elif gc_t[0] is not None:
                dt = (time.perf_counter() - gc_t[0]) * 1e3
                gc_ms["n"] += 1
                gc_ms["total_ms"] += dt
                gc_ms["max_ms"] = max(gc_ms["max_ms"], dt)
        gc.callbacks.append(_gc_cb)
        prof = None
        if args.cprofile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        if torch.cuda.is_available():
            torch.cuda.reset_peak_memory_stats()
        t0 = time.perf_counter()
        layer.run_interval(now)
        t_gen = time.perf_counter() - t0
        gc.callbacks.remove(_gc_cb)
        # the first generation's peak device memory (the caching allocator's view)
        peak_hbm = torch.cuda.max_memory_allocated() / 2**30 if torch.cuda.is_available() \
            else None
        if prof is not None:
            prof.disable()
            cprof_top = _cprofile_top(prof)
        sharded_path = layer._sharded()
        # the first generation's phases (phase_seconds accumulates over generations)
        first_phases = dict(getattr(layer._update, "phase_seconds", {}))
        first_train = dict(getattr(layer._update, "train_phases", {}) or {})
        first_lay = dict(layer.last_phases)
        h1 = getattr(layer._update, "history", None)
        first_hist = json.loads(json.dumps(h1.stats)) if h1 is not None else None
        later = []
        for g in range(1, max(1, args.generations) if ctx.world_size == 1 else 1):
            before = dict(layer._update.phase_seconds)
            before_t = dict(getattr(layer._update, "train_phases", {}) or {})
            now += 60_000
            append(args.next_ratings, now)
            t0 = time.perf_counter()
            layer.run_interval(now)
            dt = time.perf_counter() - t0
            after = layer._update.phase_seconds
            hist = getattr(layer._update, "history", None)
            later.append({"generation": g + 1, "generation_s": dt,
                          "ratings": args.ratings + g * args.next_ratings,
                          "phase_s": {k: after[k] - before.get(k, 0.0) for k in after},
                          "layer_phase_s": dict(layer.last_phases),
                          "train_phase_s": {k: v - before_t.get(k, 0.0) for k, v in
                                            (getattr(layer._update, "train_phases", {})
                                             or {}).items()},
                          "history": dict(hist.stats) if hist is not None else None})
        layer.close()
    else:
        dist.barrier(ctx)
        t0 = time.perf_counter()
        layer.run_follower()
        t_gen = time.perf_counter() - t0
        peak_hbm = None
        sharded_path = layer._sharded()
        first_phases = dict(getattr(layer._update, "phase_seconds", {}))
        first_train = dict(getattr(layer._update, "train_phases", {}) or {})
        first_lay = dict(layer.last_phases)
        first_hist = None
    phases = first_phases
    if not ctx.is_main:
        later = []
    phases.update({"layer_" + k: v for k, v in first_lay.items()})
    # the layer's own phases plus the update's (whose sum is the layer's "update" phase)
    lay = first_lay
    inner = sum(v for k, v in phases.items()
                if not k.startswith(("layer_", "pub_")) and
                k not in ("publish_y", "publish_x", "write_factors_total"))
    # (save_data_total runs beside the update: only its exposed part, save_data, counts)
    attributed = inner + sum(v for k, v in lay.items() if k not in ("update", "save_data_total"))
    if ctx.is_main:
        # count what was published
        ut = tlog.Topic(work + "/log", "OryxUpdate")
        ends = ut.end_offsets()
        ut.close()
        n_records = args.ratings if args.app == "als" else args.points
        metric = {"als": "ALS batch generation ratings/sec (input log -> published MODEL + UP "
                         "rows)",
                  "kmeans": "k-means batch generation points/sec (input log -> parse -> "
                            "k-means -> evaluation -> published MODEL)",
                  "rdf": "RDF batch generation examples/sec (input log -> parse -> forest -> "
                         "evaluation -> published MODEL)"}[args.app]
        unit = {"als": "ratings/s", "kmeans": "points/s", "rdf": "examples/s"}[args.app]
        rec = {
            "metric": metric, "app": args.app,
            "value": n_records / t_gen, "unit": unit, "higher_is_better": True,
            "n_gpus": ctx.world_size, "generation_s": t_gen, "log_append_s": t_ingest,
            "phase_s": phases,
            "train_phase_s": first_train,
            "startup_warm_up_s": layer.warm_up_s,
            "peak_hbm_gib_first_generation": peak_hbm,
            "gc_in_generation": gc_ms if ctx.is_main else None,
            "cprofile_top": cprof_top if args.cprofile and ctx.is_main else None,
            "update_messages": int(sum(ends)),
            "attributed_s": attributed, "unattributed_s": t_gen - attributed,
            "history_first": first_hist,
            "later_generations": later,
            "config": ({"ratings": args.ratings, "users": args.users, "items": args.items,
                        "features": args.features} if args.app == "als" else
                       {"points": args.points, "dims": args.dims,
                        "k": args.k if args.app == "kmeans" else None,
                        "trees": args.trees if args.app == "rdf" else None,
                        "depth": args.depth if args.app == "rdf" else None}) | {
                       "iterations": args.iterations,
                       "dtype": args.dtype if args.app == "als" else "fp32",
                       "partitions": args.partitions,
                       "test_fraction": args.test_fraction,
                       "sharded": bool(sharded_path),
                       "forced_collectives": bool(ctx.forced)},
            "data": ("synthetic power-law users x items, strengths 0.5..5, last-day timestamps"
                     if args.app == "als" else
                     "synthetic Gaussian blobs around k random centers, values on a 0.01 grid"
                     if args.app == "kmeans" else
                     "synthetic Gaussian predictors, binary target from a fixed rule"),
        }
        print(json.dumps(rec), flush=True)
        if args.dir is None:
            shutil.rmtree(work, ignore_errors=True)
    if ctx.is_distributed:
        dist.barrier(ctx)
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
