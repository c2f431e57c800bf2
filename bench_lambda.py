#!/usr/bin/env python3
"""Whole lambda loop latency: ``POST /ingest`` -> speed layer ``UP`` -> visible in ``/recommend``.

The path the reference runs through Kafka and Spark Streaming
(``[serving-app]/als/Ingest.java:59-80`` -> input topic -> ``[lambda]/speed/SpeedLayerUpdate.java:
51-64`` -> update topic -> the serving model manager's consumer): a serving layer (HTTP) and a
speed layer share the input and update logs; an ALS model of ``--items`` x ``--features``
item vectors and ``--users`` users is loaded through the update topic (MODEL + UP rows, as the
batch layer publishes it).  Each trial reads ``/recommend/<user>``, POSTs one new rating of
that user to ``/ingest``, and polls ``/recommend/<user>`` until the response changes (the
speed layer's fold-in moved the user's vector).  The speed layer runs its micro-batches
back to back every ``--interval-ms`` (the reference's streaming interval is a
configuration choice -- 10 s by default -- and adds its own wait on top).

``python bench_lambda.py [--trials 50] [--interval-ms 10]``; prints one JSON line with the
p50 / p90 / max ingest-to-visible latency in ms.
"""

from __future__ import annotations

import argparse
import http.client
import json
import os
import shutil
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--users", type=int, default=50_000)
    ap.add_argument("--features", type=int, default=50)
    ap.add_argument("--trials", type=int, default=50)
    ap.add_argument("--interval-ms", type=float, default=10.0)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--seed", type=int, default=3)
    args = ap.parse_args(argv)
    from oryx_amd import ingest
    from oryx_amd.layers.speed import SpeedLayer
    from oryx_amd.serving.layer import ServingLayer
    from oryx_amd.transport import log as tlog
    from oryx_amd.utils import config as cfg, pmml as pmmlu

    work = tempfile.mkdtemp(prefix="oryx_lambda_")
    root = os.path.join(work, "log")
    g = np.random.default_rng(args.seed)
    k = args.features
    try:
        tlog.maybe_create_topic(root, "OryxInput", 1)
        tlog.maybe_create_topic(root, "OryxUpdate", 1, max_message=1 << 30)
        # the model, as the batch layer publishes it
        Y = (g.standard_normal((args.items, k)) * 0.3).astype(np.float32)
        X = (g.standard_normal((args.users, k)) * 0.3).astype(np.float32)
        item_ids = ["I%d" % i for i in range(args.items)]
        user_ids = ["U%d" % i for i in range(args.users)]
        topic = tlog.Topic(root, "OryxUpdate")
        doc = pmmlu.build_skeleton_pmml()
        for key, val in (("X", "X/"), ("Y", "Y/"), ("features", k), ("lambda", 0.001),
                         ("implicit", True), ("alpha", 1.0)):
            doc.add_extension(key, val)
        doc.add_extension_content("XIDs", user_ids)
        doc.add_extension_content("YIDs", item_ids)
        topic.append_batch([("MODEL", pmmlu.to_string(doc))])
        topic.append_block(ingest.assemble_row_messages(
            "Y", item_ids, ingest.format_float_rows_blob(Y)), key="UP")
        topic.append_block(ingest.assemble_row_messages(
            "X", user_ids, ingest.format_float_rows_blob(X)), key="UP")
        topic.close()
        conf = cfg.overlay_on({
            "oryx.id": '"lambda-bench"',
            "oryx.transport.log-dir": '"%s"' % root,
            "oryx.update-topic.message.max-size": 1 << 30,
            "oryx.serving.api.port": 0,
            "oryx.speed.model-manager-class":
                "com.cloudera.oryx.app.speed.als.ALSSpeedModelManager",
            "oryx.serving.model-manager-class":
                "com.cloudera.oryx.app.serving.als.model.ALSServingModelManager",
            "oryx.serving.application-resources":
                '"com.cloudera.oryx.app.serving,com.cloudera.oryx.app.serving.als"',
            "oryx.gpu.device": '"%s"' % args.device,
        }, cfg.get_default())
        serving = ServingLayer(conf, host="127.0.0.1").start()
        speed = SpeedLayer(conf).start(start_timer=False)
        stop = threading.Event()
        try:
            t0 = time.time()
            while time.time() - t0 < 600:
                sm = speed.manager.model
                vm = serving.manager.get_model()
                if sm is not None and vm is not None and sm.get_fraction_loaded() >= 1.0 and \
                        vm.get_fraction_loaded() >= 1.0 and vm.get_num_users() == args.users \
                        and sm.X.size() == args.users:
                    break
                time.sleep(0.05)
            load_s = time.time() - t0

            def micro_batches():
                while not stop.is_set():
                    t = time.perf_counter()
                    speed.run_interval()
                    left = args.interval_ms / 1e3 - (time.perf_counter() - t)
                    if left > 0:
                        stop.wait(left)
            runner = threading.Thread(target=micro_batches, name="speed-batches", daemon=True)
            runner.start()
            conn = http.client.HTTPConnection("127.0.0.1", serving.actual_port, timeout=30)

            def get(path):
                conn.request("GET", path, headers={"Accept": "application/json"})
                r = conn.getresponse()
                return r.status, r.read()

            def post(path, body):
                conn.request("POST", path, body=body, headers={"Content-Type": "text/plain"})
                r = conn.getresponse()
                r.read()
                return r.status

            lat = []
            timeouts = 0
            for trial in range(args.trials + 3):
                u = "U%d" % int(g.integers(args.users))
                i = "I%d" % int(g.integers(args.items))
                st, before = get("/recommend/%s?howMany=10" % u)
                assert st == 200, st
                t_send = time.perf_counter()
                assert post("/ingest", ("%s,%s,5\n" % (u, i)).encode()) in (200, 204)
                seen = None
                while time.perf_counter() - t_send < 10.0:
                    st, now = get("/recommend/%s?howMany=10" % u)
                    if now != before:
                        seen = time.perf_counter()
                        break
                if seen is None:
                    timeouts += 1
                elif trial >= 3:
                    lat.append((seen - t_send) * 1e3)
            conn.close()
        finally:
            stop.set()
            speed.close()
            serving.close()
        lat_a = np.asarray(lat)
        print(json.dumps({
            "metric": "ingest -> visible latency (POST /ingest -> speed UP -> /recommend "
                      "changes)",
            "p50_ms": float(np.percentile(lat_a, 50)) if len(lat) else None,
            "p90_ms": float(np.percentile(lat_a, 90)) if len(lat) else None,
            "max_ms": float(lat_a.max()) if len(lat) else None,
            "trials": len(lat), "timeouts": timeouts, "interval_ms": args.interval_ms,
            "items": args.items, "users": args.users, "features": k,
            "model_load_s": load_s,
            "path": "HTTP POST /ingest -> input log (async producer) -> speed layer micro-batch "
                    "(parse, fold-in, UP append) -> update log -> serving consumer -> HTTP GET "
                    "/recommend",
        }), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
