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
query = sys.argv[5] if len(sys.argv) > 5 else ""
cafile = sys.argv[6] if len(sys.argv) > 6 else ""
rnd = random.Random(seed)
if cafile:
    import ssl
    # one keep-alive TLS connection per client (as the reference's load test): one handshake
    conn = http.client.HTTPSConnection("127.0.0.1", port, timeout=60,
                                       context=ssl.create_default_context(cafile=cafile))
else:
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
lat = []
errors = 0
t0 = time.perf_counter()
for _ in range(n):
    path = "/recommend/U%d%s" % (rnd.randrange(users), query)
    t = time.perf_counter()
    conn.request("GET", path, headers={"Accept": "application/json"})
    r = conn.getresponse()
    body = r.read()
    lat.append((time.perf_counter() - t) * 1e3)
    if r.status != 200:
        errors += 1
print(json.dumps({"n": n, "wall": time.perf_counter() - t0, "lat": lat, "errors": errors}))
"""


def make_data(items: int, users: int, features: int, seed: int):
    """Item / user factor matrices, ids and Poisson(20) known items (LoadTestALSModelFactory)."""
    rng = np.random.default_rng(seed)
    # generated in chunks with a progress line each (20M x 250 takes minutes: a silent run
    # that long looks hung to a supervisor)
    Y = np.empty((items, features), dtype=np.float32)
    step = 1 << 21
    for lo in range(0, items, step):
        Y[lo:lo + step] = rng.standard_normal((min(step, items - lo), features),
                                              dtype=np.float32)
        print("make_data: %d / %d item rows" % (min(items, lo + step), items), file=sys.stderr,
              flush=True)
    X = rng.standard_normal((users, features), dtype=np.float32)
    item_ids = ["I%d" % i for i in range(items)]
    user_ids = ["U%d" % i for i in range(users)]
    counts = rng.poisson(20, users)
    known = rng.integers(0, items, int(counts.sum()))
    return Y, X, item_ids, user_ids, counts, known


def build_model(data, features: int, sample_rate: float, max_batch: int = 16,
                rescorer: bool = False):
    import torch
    from oryx_amd.models.als.serving import ALSServingModel
    provider = None
    if rescorer:
        # the example provider (models/als/rescorer.py): drops every item whose numeric ID is
        # a multiple of 10 and scales the other scores (device form: a cached row mask)
        from oryx_amd.models.als.rescorer import ItemFilterRescorerProvider
        os.environ["ORYX_EXAMPLE_RESCORER_EXCLUDE_MOD"] = "10"
        provider = ItemFilterRescorerProvider()
    Y, X, item_ids, user_ids, counts, known = data
    model = ALSServingModel(features, True, sample_rate, provider, max_batch=max_batch)
    chunk = 1 << 21
    for lo in range(0, len(item_ids), chunk):
        model.Y.set_vectors(item_ids[lo:lo + chunk], Y[lo:lo + chunk])
    for lo in range(0, len(user_ids), chunk):
        model.X.set_vectors(user_ids[lo:lo + chunk], X[lo:lo + chunk])
    print("build_model: factors loaded", file=sys.stderr, flush=True)
    pos = 0
    for u, c in enumerate(counts.tolist()):
        model.add_known_items(user_ids[u], [item_ids[i] for i in known[pos:pos + c].tolist()])
        pos += c
        if u % 100000 == 0:
            print("build_model: known items %d / %d users" % (u, len(counts)), file=sys.stderr,
                  flush=True)
    model.Y.device_view()          # push the matrix to HBM before timing
    if model.index is not None:
        model.index.refresh()      # and build the bucket-sorted scan index
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return model


def _self_signed(dirname: str):
    """(cert, key) PEM files of a throwaway self-signed certificate for 127.0.0.1."""
    cert, key = os.path.join(dirname, "cert.pem"), os.path.join(dirname, "key.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                    "-out", cert, "-days", "2", "-subj", "/CN=127.0.0.1",
                    "-addext", "subjectAltName=IP:127.0.0.1"], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return cert, key


def serve_and_measure(model, users: int, workers: int, requests: int, warmup: int,
                      seed: int, query: str = "", tls: bool = False):
    from oryx_amd.api import AbstractServingModelManager
    from oryx_amd.serving.layer import ServingLayer
    from oryx_amd.utils import config as cfg

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
        # ORYX_BENCH_PYTHON_HTTP=1: the Python http.server front end (A/B)
        "oryx.serving.api.native-http":
            "false" if os.environ.get("ORYX_BENCH_PYTHON_HTTP") == "1" else "true",
        "oryx.serving.api.handler-threads": int(os.environ.get("ORYX_BENCH_HTTP_THREADS", "16")),
    }, cfg.get_default())
    cafile = ""
    if tls:
        # HTTPS on the native front end (OpenSSL inside csrc/runtime/oryx_http.cpp)
        import tempfile
        cert, key = _self_signed(tempfile.mkdtemp(prefix="oryx_bench_tls_"))
        conf = cfg.overlay_on({"oryx.serving.api.secure-port": 0,
                               "oryx.serving.api.keystore-file": '"%s"' % cert,
                               "oryx.serving.api.key-file": '"%s"' % key}, conf)
        cafile = cert
    layer = ServingLayer(conf, manager=_Manager(conf), host="127.0.0.1").start()
    port = layer.actual_port

    def run(n):
        procs = [subprocess.Popen([sys.executable, "-c", CLIENT, str(port), str(users),
                                   str(n), str(seed * 100 + w), query, cafile],
                                  stdout=subprocess.PIPE, text=True)
                 for w in range(workers)]
        outs = [json.loads(p.communicate()[0]) for p in procs]
        return outs

    try:
        run(warmup)
        outs = run(requests)
    finally:
        layer.close()
    lat = np.concatenate([o["lat"] for o in outs])
    total = sum(o["n"] for o in outs)
    errors = sum(o["errors"] for o in outs)
    # wall clock of the slowest client (process start-up excluded)
    client_wall = max(o["wall"] for o in outs)
    return total / client_wall, lat, total, errors


def record(model, args_like, qps, lat, total, errors, build_s, workers, sample_rate, items,
           features):
    key = (features, int(round(items / 1e6)), sample_rate)
    pub = PUBLISHED.get(key)
    b = model.batcher
    return {
        "metric": "/recommend throughput (LoadBenchmark equivalent)",
        "value": qps, "unit": "req/s", "higher_is_better": True,
        "mean_latency_ms": float(lat.mean()), "p50_ms": float(np.percentile(lat, 50)),
        "p99_ms": float(np.percentile(lat, 99)),
        "items": items, "users": args_like.users, "features": features,
        "sample_rate": sample_rate, "workers": workers, "requests": total,
        "errors": errors, "model_build_s": build_s,
        "scan": "fused HIP top-N (topn.hip)" if b is not None else "torch",
        "mean_batch": (b.requests / b.batches) if b is not None and b.batches else None,
        "published_reference": {"qps": pub[0], "latency_ms": pub[1],
                                "hardware": "32-core Xeon 2.3GHz Haswell, JDK 8"} if pub else None,
        "vs_reference_qps": (qps / pub[0]) if pub else None,
        "vs_reference_latency": (pub[1] / float(lat.mean())) if pub else None,
        "data": "synthetic random Gaussian factors, Poisson(20) known items per user",
    }


def time_to_ready(items: int, users: int, features: int, seed: int) -> dict:
    """Model load through the update topic: MODEL (PMML with XIDs / YIDs) then every Y and
    X row as an ``UP`` message (what the batch layer publishes), consumed by a serving layer
    from the log; seconds until the model reports fraction-loaded 1 and every row is present.
    Also the HBM the loaded model holds (device mirror + scan index)."""
    import shutil
    import tempfile
    import torch
    from oryx_amd import ingest
    from oryx_amd.models.als import serving as als_serving
    from oryx_amd.serving import layer as serving_layer
    from oryx_amd.serving.layer import ServingLayer
    from oryx_amd.transport import log as tlog
    from oryx_amd.utils import config as cfg, pmml as pmmlu
    work = tempfile.mkdtemp(prefix="oryx_ttr_", dir=os.environ.get("ORYX_TTR_DIR"))
    try:
        Y, X, item_ids, user_ids, counts, known = make_data(items, users, features, seed)
        root = os.path.join(work, "log")
        t_gen = time.perf_counter()
        tlog.maybe_create_topic(root, "OryxUpdate", 1, max_message=1 << 30)
        topic = tlog.Topic(root, "OryxUpdate")
        doc = pmmlu.build_skeleton_pmml()
        doc.add_extension("X", "X/")
        doc.add_extension("Y", "Y/")
        doc.add_extension("features", features)
        doc.add_extension("lambda", 0.001)
        doc.add_extension("implicit", True)
        doc.add_extension("alpha", 1.0)
        doc.add_extension_content("XIDs", user_ids)
        doc.add_extension_content("YIDs", item_ids)
        topic.append_batch([("MODEL", pmmlu.to_string(doc))])
        # the batch layer's publish path: rows formatted and assembled natively, appended
        # as blocks
        chunk = 1 << 20
        for lo in range(0, items, chunk):
            hi = min(items, lo + chunk)
            topic.append_block(ingest.assemble_row_messages(
                "Y", item_ids[lo:hi], ingest.format_float_rows_blob(Y[lo:hi])), key="UP")
            print("time_to_ready: log %d / %d item rows" % (hi, items), file=sys.stderr,
                  flush=True)
        pos = np.r_[0, np.cumsum(counts)]
        names = ingest.IdDict()
        names.encode(["I%d" % i for i in range(items)])
        for lo in range(0, users, chunk):
            hi = min(users, lo + chunk)
            uu = np.repeat(np.arange(hi - lo), counts[lo:hi])
            kt = ingest.known_items_text(names, uu, known[pos[lo]:pos[hi]], hi - lo)
            topic.append_block(ingest.assemble_row_messages(
                "X", user_ids[lo:hi], ingest.format_float_rows_blob(X[lo:hi]), kt,
                np.arange(hi - lo)), key="UP")
        topic.close()
        gen_s = time.perf_counter() - t_gen
        log_bytes = sum(os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(root)
                        for f in fs)
        conf = cfg.overlay_on({
            "oryx.serving.api.port": 0,
            "oryx.serving.api.read-only": "true",
            "oryx.transport.log-dir": '"%s"' % root,
            "oryx.update-topic.message.max-size": 1 << 30,
            "oryx.serving.model-manager-class":
                "com.cloudera.oryx.app.serving.als.model.ALSServingModelManager",
            "oryx.serving.application-resources":
                '"com.cloudera.oryx.app.serving,com.cloudera.oryx.app.serving.als"',
        }, cfg.get_default())
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            base = torch.cuda.memory_allocated()
        t0 = time.perf_counter()
        layer = ServingLayer(conf, host="127.0.0.1").start()
        try:
            mgr = layer.manager
            while True:
                m = mgr.get_model()
                if m is not None and m.get_fraction_loaded() >= 1.0 and \
                        m.get_num_items() == items and m.get_num_users() == users:
                    break
                if time.perf_counter() - t0 > 3000:
                    raise TimeoutError("model not loaded")
                if int((time.perf_counter() - t0) * 50) % 500 == 0:
                    print("time_to_ready: loading, %.0f s" % (time.perf_counter() - t0),
                          file=sys.stderr, flush=True)
                time.sleep(0.02)
            ready_s = time.perf_counter() - t0
            # first query also pushes the matrix to HBM and builds the scan index
            t1 = time.perf_counter()
            m.top_n(Y[0], 10)
            first_query_s = time.perf_counter() - t1
            hbm = (torch.cuda.memory_allocated() - base) / 2**30 \
                if torch.cuda.is_available() else None
        finally:
            layer.close()
        return {"metric": "ALS serving model time-to-ready from the update topic",
                "items": items, "users": users, "features": features,
                "update_log_gb": log_bytes / 1e9, "log_build_s": gen_s, "ready_s": ready_s,
                "rows_per_s": (items + users) / ready_s,
                "first_query_s": first_query_s, "model_hbm_gib": hbm,
                "drain": dict(als_serving.DRAIN_STATS),
                "take": dict(serving_layer.TAKE_STATS, **ingest.PARSE_STATS),
                "data": "synthetic Gaussian factors, Poisson(20) known items per user"}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--users", type=int, default=500_000)
    ap.add_argument("--features", type=int, default=50)
    ap.add_argument("--sample-rate", type=float, default=0.3)
    ap.add_argument("--workers", default="2", help="comma list of concurrent clients")
    ap.add_argument("--requests", type=int, default=500, help="per worker")
    ap.add_argument("--warmup", type=int, default=50, help="per worker, untimed")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--sweep", action="store_true",
                    help="every published row: features 50/250 x items 1/5/20M x sample rate "
                         "0.3/1.0 at each --workers count (one JSON line each)")
    ap.add_argument("--sweep-features", default="50,250",
                    help="--sweep: the feature counts to cover (comma list)")
    ap.add_argument("--sweep-items", default="1000000,5000000,20000000",
                    help="--sweep: the item counts to cover (comma list)")
    ap.add_argument("--max-batch", type=int, default=16)
    ap.add_argument("--time-to-ready", action="store_true",
                    help="measure the model load through the update topic instead")
    ap.add_argument("--rescorer", action="store_true",
                    help="requests carry rescorerParams for the example ItemFilterRescorer "
                         "provider (every candidate filtered / rescored, on the device)")
    ap.add_argument("--tls", choices=("off", "on", "both"), default="off",
                    help="HTTPS on the native front end (self-signed certificate); both: an "
                         "HTTP and an HTTPS run per worker count, with their req/s ratio")
    args = ap.parse_args(argv)
    if args.time_to_ready:
        print(json.dumps(time_to_ready(args.items, args.users, args.features, args.seed)),
              flush=True)
        return 0
    workers = [int(w) for w in str(args.workers).split(",")]
    if args.sweep:
        grid = [(int(f), int(m)) for f in args.sweep_features.split(",")
                for m in args.sweep_items.split(",")]
        rates = (0.3, 1.0)
    else:
        grid = [(args.features, args.items)]
        rates = (args.sample_rate,)
    for features, items in grid:
        data = make_data(items, args.users, features, args.seed)
        for rate in rates:
            t0 = time.perf_counter()
            model = build_model(data, features, rate, args.max_batch, args.rescorer)
            build_s = time.perf_counter() - t0
            modes = {"off": (False,), "on": (True,), "both": (False, True)}[args.tls]
            for w in workers:
                http_qps = None
                for tls in modes:
                    if model.batcher is not None:
                        model.batcher.batches = model.batcher.requests = 0
                    qps, lat, total, errors = serve_and_measure(
                        model, args.users, w, args.requests, args.warmup, args.seed,
                        "?rescorerParams=factor:1.5" if args.rescorer else "", tls=tls)
                    rec = record(model, args, qps, lat, total, errors, build_s, w, rate,
                                 items, features)
                    rec["rescorer"] = bool(args.rescorer)
                    rec["front_end"] = "python http.server" if \
                        os.environ.get("ORYX_BENCH_PYTHON_HTTP") == "1" else \
                        "native (oryx_http.cpp), %s handler threads" % \
                        os.environ.get("ORYX_BENCH_HTTP_THREADS", "16")
                    rec["tls"] = tls
                    if tls and http_qps:
                        rec["https_over_http_qps"] = qps / http_qps
                    if not tls:
                        http_qps = qps
                    print(json.dumps(rec), flush=True)
            if model.batcher is not None:
                model.batcher.close()
            del model
        del data
    return 0


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    sys.stderr.flush()
    # no interpreter finalisation: a daemon thread (HTTP handlers, the top-N batcher) that
    # returns from a GIL-free native call while the interpreter shuts down is ended with a
    # forced unwind, which aborts the process after the records are already written
    os._exit(rc)
