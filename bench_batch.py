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
    ap.add_argument("--test-fraction", type=float, default=0.0,
                    help="oryx.ml.eval.test-fraction (the reference default is 0.1: the newest "
                         "tenth of the interval's data is held out and AUC is evaluated)")
    args = ap.parse_args(argv)

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
    conf = cfg.overlay_on({
        "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.als.ALSUpdate",
        "oryx.input-topic.broker": "log:" + work + "/log",
        "oryx.update-topic.broker": "log:" + work + "/log",
        "oryx.input-topic.partitions": args.partitions,
        "oryx.update-topic.message.max-size": 1 << 30,
        "oryx.batch.storage.data-dir": work + "/data",
        "oryx.batch.storage.model-dir": work + "/model",
        "oryx.als.hyperparams.features": args.features,
        "oryx.als.iterations": args.iterations,
        "oryx.als.implicit": "true",
        "oryx.ml.eval.candidates": 1,
        "oryx.ml.eval.test-fraction": args.test_fraction,
        "oryx.gpu.device": args.device,
        "oryx.gpu.dtype": args.dtype,
    }, cfg.get_default())
    layer = BatchLayer(conf)
    t_ingest = 0.0
    if ctx.is_main:
        layer._context = layer.layer_context()
        layer._update = layer.load_update_instance()
        layer.build_input_consumer()
        rng = np.random.default_rng(7)
        now = int(time.time() * 1000)

        def append(n_total, now):
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
        append(args.ratings, now)
        t_ingest = time.perf_counter() - t0
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier(ctx)
        t0 = time.perf_counter()
        layer.run_interval(now)
        t_gen = time.perf_counter() - t0
        sharded_path = layer._sharded()
        later = []
        for g in range(1, max(1, args.generations) if ctx.world_size == 1 else 1):
            before = dict(layer._update.phase_seconds)
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
                          "history": dict(hist.stats) if hist is not None else None})
        layer.close()
    else:
        dist.barrier(ctx)
        t0 = time.perf_counter()
        layer.run_follower()
        t_gen = time.perf_counter() - t0
        sharded_path = layer._sharded()
    upd = layer._update
    phases = dict(getattr(upd, "phase_seconds", {}))
    if not ctx.is_main:
        later = []
    phases.update({"layer_" + k: v for k, v in layer.last_phases.items()})
    # the layer's own phases plus the update's (whose sum is the layer's "update" phase)
    lay = layer.last_phases
    inner = sum(v for k, v in phases.items()
                if not k.startswith("layer_") and k not in ("publish_y", "publish_x"))
    attributed = inner + sum(v for k, v in lay.items() if k != "update")
    if ctx.is_main:
        # count what was published
        ut = tlog.Topic(work + "/log", "OryxUpdate")
        ends = ut.end_offsets()
        ut.close()
        rec = {
            "metric": "ALS batch generation ratings/sec (input log -> published MODEL + UP rows)",
            "value": args.ratings / t_gen, "unit": "ratings/s", "higher_is_better": True,
            "n_gpus": ctx.world_size, "generation_s": t_gen, "log_append_s": t_ingest,
            "phase_s": phases, "update_messages": int(sum(ends)),
            "attributed_s": attributed, "unattributed_s": t_gen - attributed,
            "later_generations": later,
            "config": {"ratings": args.ratings, "users": args.users, "items": args.items,
                       "features": args.features, "iterations": args.iterations,
                       "dtype": args.dtype, "partitions": args.partitions,
                       "test_fraction": args.test_fraction,
                       "sharded": bool(sharded_path),
                       "forced_collectives": bool(ctx.forced)},
            "data": "synthetic power-law users x items, strengths 0.5..5, last-day timestamps",
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
