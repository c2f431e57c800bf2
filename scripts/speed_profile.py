#!/usr/bin/env python3
"""Host-side profile of one ALS speed-layer micro-batch (the ``bench.py`` speed phase):
``ALSSpeedModelManager.build_updates`` + the UP block append, repeated, with per-call timings
of the parse / aggregation pieces and a cProfile of the whole loop (top entries by own time).

``python scripts/speed_profile.py [--events 10000] [--reps 20] [--k 64]``; prints JSON lines.
"""

from __future__ import annotations

import argparse
import cProfile
import io
import json
import os
import pstats
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--users", type=int, default=162541)
    ap.add_argument("--items", type=int, default=59047)
    ap.add_argument("--chunks", type=int, default=4)
    args = ap.parse_args()
    import torch
    from oryx_amd import ingest
    from oryx_amd.api import Dataset
    from oryx_amd.layers.speed import publish_blocks
    from oryx_amd.models.als.batch import aggregate_scores
    from oryx_amd.models.als.speed import ALSSpeedModel, ALSSpeedModelManager
    from oryx_amd.transport.producer import LogTopicProducer
    from oryx_amd.utils import config as cfg

    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    g = np.random.default_rng(5)
    k = args.k
    model = ALSSpeedModel(k, True, dev)
    model.X.set_vectors(["U%d" % j for j in range(args.users)],
                        (g.standard_normal((args.users, k)) * 0.1).astype(np.float32))
    model.Y.set_vectors(["I%d" % j for j in range(args.items)],
                        (g.standard_normal((args.items, k)) * 0.1).astype(np.float32))
    mgr = ALSSpeedModelManager(cfg.get_default())
    mgr.model = model
    B = args.events
    now = int(time.time() * 1000)
    lines = ["U%d,I%d,%.2f,%d" % (a, b, v, now) for a, b, v in
             zip(g.integers(0, args.users, B).tolist(), g.integers(0, args.items, B).tolist(),
                 (g.random(B) * 4 + 0.5).tolist())]
    ds = Dataset.from_values(lines)

    # the pieces of parse_aggregate on their own
    piece = {"values": [], "parse": [], "aggregate": []}
    d1, d2 = ingest.IdDict(), ingest.IdDict()
    for _ in range(args.reps):
        t0 = time.perf_counter()
        vals = ds.values()
        t1 = time.perf_counter()
        u, i, s, ts = ingest.parse_ratings(vals, d1.clear(), d2.clear(), default_ts=0)
        t2 = time.perf_counter()
        aggregate_scores(u, i, s, ts, True)
        t3 = time.perf_counter()
        piece["values"].append((t1 - t0) * 1e3)
        piece["parse"].append((t2 - t1) * 1e3)
        piece["aggregate"].append((t3 - t2) * 1e3)
    print(json.dumps({"pieces_median_ms": {kk: float(np.median(v)) for kk, v in piece.items()}}),
          flush=True)

    logdir = tempfile.mkdtemp(prefix="oryx_speed_prof_")
    producer = LogTopicProducer("log:" + logdir, "OryxUpdate", async_=False,
                                max_message=1 << 30)
    times, phases = [], []
    prof = cProfile.Profile()
    try:
        for rep in range(args.reps + 2):
            model.X.version += 1
            if dev.type == "cuda":
                torch.cuda.synchronize()
            if rep == 2:
                prof.enable()
            t1 = time.perf_counter()
            pub: dict = {}
            publish_blocks(producer, mgr.build_update_blocks(ds, chunks=args.chunks), pub)
            t3 = time.perf_counter()
            if rep >= 2:
                times.append((t3 - t1) * 1e3)
                ph = dict(mgr.last_phase_ms)
                ph.update(pub)
                phases.append(ph)
        prof.disable()
    finally:
        producer.close()
        shutil.rmtree(logdir, ignore_errors=True)
    out = io.StringIO()
    pstats.Stats(prof, stream=out).sort_stats("tottime").print_stats(25)
    print(json.dumps({"median_ms": float(np.median(times)),
                      "p90_ms": float(np.percentile(times, 90)),
                      "phases_median_ms": {kk: float(np.median([p.get(kk, 0.0) for p in phases]))
                                           for kk in phases[0]}}),
          flush=True)
    print(out.getvalue())
    return 0


if __name__ == "__main__":
    sys.exit(main())
