#!/usr/bin/env python3
"""Serving-layer benchmark: ``/recommend`` throughput and latency (BASELINE.md's published metric).

Mirrors the reference's ``LoadBenchmark`` / ``LoadTestALSModelFactory``
(``[serving-app]/src/test/.../als/LoadBenchmark.java``, ``model/LoadTestALSModelFactory.java``):
an ALS serving model of ``--items`` random Gaussian item vectors and ``--users`` users with
Poisson(20) known items each, served over HTTP; ``--workers`` concurrent clients each issue
``GET /recommend/U<random>`` (Accept: application/json, known items excluded) and the harness
reports requests/s and mean latency.  Clients are separate processes (no GIL sharing with the
server).  Published reference numbers (32-core Xeon, JDK 8, performance.md:112-128) are printed
alongside for the matching (features, items, sample-rate) row.

Usage: ``python bench_serving.py --items 1000000 --features 50 --sample-rate 0.3``
Prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# performance.md:112-128 -- (features, items M, sample rate) -> (qps, latency ms)
PUBLISHED = {
    (50, 1, 0.3): (437, 7), (250, 1, 0.3): (151, 13), (50, 5, 0.3): (84, 24),
    (250, 5, 0.3): (36, 56), (50, 20, 0.3): (14, 69), (250, 20, 0.3): (6, 162),
    (50, 1, 1.0): (74, 27), (250, 1, 1.0): (23, 44), (50, 5, 1.0): (13, 80),
    (250, 5, 1.0): (5, 191), (50, 20, 1.0): (4, 282), (250, 20, 1.0): (1, 708),
}

CLIENT = r"""
import http.client, json, random, sys, time
port, users, n, seed = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
rnd = random.Random(seed)
conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
lat = []
errors = 0
t0 = time.perf_counter()
for _ in range(n):
    path = "/recommend/U%d" % rnd.randrange(users)
    t = time.perf_counter()
    conn.request("GET", path, headers={"Accept": "application/json"})
    r = conn.getresponse()
    body = r.read()
    lat.append((time.perf_counter() - t) * 1e3)
    if r.status != 200:
        errors += 1
print(json.dumps({"n": n, "wall": time.perf_counter() - t0, "lat": lat, "errors": errors}))
"""


def build_model(items: int, users: int, features: int, sample_rate: float, seed: int):
    import torch
    from oryx_amd.models.als.serving import ALSServingModel
    rng = np.random.default_rng(seed)
    model = ALSServingModel(features, True, sample_rate)
    chunk = 1 << 20
    for lo in range(0, items, chunk):
        hi = min(items, lo + chunk)
        model.Y.set_vectors(["I%d" % i for i in range(lo, hi)],
                            rng.standard_normal((hi - lo, features), dtype=np.float32))
    for lo in range(0, users, chunk):
        hi = min(users, lo + chunk)
        model.X.set_vectors(["U%d" % i for i in range(lo, hi)],
                            rng.standard_normal((hi - lo, features), dtype=np.float32))
    counts = rng.poisson(20, users)
    known = rng.integers(0, items, int(counts.sum()))
    pos = 0
    for u in range(users):
        c = int(counts[u])
        model.add_known_items("U%d" % u, ["I%d" % i for i in known[pos:pos + c].tolist()])
        pos += c
    model.Y.device_view()          # push the matrix to HBM before timing
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return model


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--users", type=int, default=100_000)
    ap.add_argument("--features", type=int, default=50)
    ap.add_argument("--sample-rate", type=float, default=0.3)
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--requests", type=int, default=500, help="per worker")
    ap.add_argument("--warmup", type=int, default=50, help="per worker, untimed")
    ap.add_argument("--seed", type=int, default=7)
    args = ap.parse_args(argv)

    from oryx_amd.api import AbstractServingModelManager
    from oryx_amd.serving.layer import ServingLayer
    from oryx_amd.utils import config as cfg

    t0 = time.perf_counter()
    model = build_model(args.items, args.users, args.features, args.sample_rate, args.seed)
    build_s = time.perf_counter() - t0

    class _Manager(AbstractServingModelManager):
        def consume(self, updates, context=None):
            for _ in updates:
                pass

        def get_model(self):
            return model

    conf = cfg.overlay_on({
        "oryx.serving.api.port": 0,
        "oryx.serving.api.read-only": "true",
        "oryx.serving.no-init-topics": "true",
        "oryx.serving.application-resources": '"com.cloudera.oryx.app.serving,'
                                              'com.cloudera.oryx.app.serving.als"',
    }, cfg.get_default())
    layer = ServingLayer(conf, manager=_Manager(conf), host="127.0.0.1").start()
    port = layer.actual_port

    def run(n):
        procs = [subprocess.Popen([sys.executable, "-c", CLIENT, str(port), str(args.users),
                                   str(n), str(args.seed * 100 + w)],
                                  stdout=subprocess.PIPE, text=True)
                 for w in range(args.workers)]
        t = time.perf_counter()
        outs = [json.loads(p.communicate()[0]) for p in procs]
        return outs, time.perf_counter() - t

    try:
        run(args.warmup)
        outs, wall = run(args.requests)
    finally:
        layer.close()
    lat = np.concatenate([o["lat"] for o in outs])
    total = sum(o["n"] for o in outs)
    errors = sum(o["errors"] for o in outs)
    # wall clock of the slowest client (process start-up excluded)
    client_wall = max(o["wall"] for o in outs)
    qps = total / client_wall
    key = (args.features, int(round(args.items / 1e6)), args.sample_rate)
    pub = PUBLISHED.get(key)
    rec = {
        "metric": "/recommend throughput (LoadBenchmark equivalent)",
        "value": qps, "unit": "req/s", "higher_is_better": True,
        "mean_latency_ms": float(lat.mean()), "p50_ms": float(np.percentile(lat, 50)),
        "p99_ms": float(np.percentile(lat, 99)),
        "items": args.items, "users": args.users, "features": args.features,
        "sample_rate": args.sample_rate, "workers": args.workers, "requests": total,
        "errors": errors, "model_build_s": build_s,
        "published_reference": {"qps": pub[0], "latency_ms": pub[1],
                                "hardware": "32-core Xeon 2.3GHz Haswell, JDK 8"} if pub else None,
        "vs_reference_qps": (qps / pub[0]) if pub else None,
        "data": "synthetic random Gaussian factors, Poisson(20) known items per user",
    }
    print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
