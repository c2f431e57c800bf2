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

            # the update log, read from its end before each trial: the speed layer's UP
            # for the trial's user tells a published update (then: is it in the serving
            # model yet?) from a micro-batch that produced none for the user (a no-op
            # fold-in: the implicit target moved nothing, e.g. Xu.Yi already >= 1)
            upd_topic = tlog.Topic(root, "OryxUpdate")
            in_topic = tlog.Topic(root, "OryxInput")
            lat, up_lat, vis_lat = [], [], []
            timeouts = noops = unchanged_lists = 0
            for trial in range(args.trials + 3):
                u = "U%d" % int(g.integers(args.users))
                i = "I%d" % int(g.integers(args.items))
                st, before = get("/recommend/%s?howMany=10" % u)
                assert st == 200, st
                reader = upd_topic.reader(0, upd_topic.end_offset(0))
                in_end = in_topic.end_offset(0)
                t_send = time.perf_counter()
                assert post("/ingest", ("%s,%s,5\n" % (u, i)).encode()) in (200, 204)
                seen = t_up = t_vis = None
                up_vec = None
                runs_at_input = None
                while time.perf_counter() - t_send < 10.0:
                    if runs_at_input is None and in_topic.end_offset(0) > in_end:
                        runs_at_input = speed.intervals_run   # the rating is in the input log
                    if up_vec is None:
                        for _, _, key, msg in reader.poll(4096, 0):
                            if key == "UP" and msg.startswith('["X","%s",' % u):
                                up_vec = np.asarray(json.loads(msg)[2], dtype=np.float32)
                                t_up = time.perf_counter()
                    if up_vec is not None and t_vis is None:
                        cur = serving.manager.get_model().get_user_vector(u)
                        if cur is not None and np.array_equal(np.asarray(cur, np.float32),
                                                              up_vec):
                            t_vis = time.perf_counter()
                    if seen is None:
                        st, now = get("/recommend/%s?howMany=10" % u)
                        if now != before:
                            seen = time.perf_counter()
                    if seen is not None and t_vis is not None:
                        break
                    # two intervals past the one that drained the rating and still no UP
                    # for the user: the fold-in was a no-op
                    if up_vec is None and runs_at_input is not None and \
                            speed.intervals_run >= runs_at_input + 2:
                        for _, _, key, msg in reader.poll(4096, 0):
                            if key == "UP" and msg.startswith('["X","%s",' % u):
                                up_vec = np.asarray(json.loads(msg)[2], dtype=np.float32)
                                t_up = time.perf_counter()
                        if up_vec is None:
                            break
                    time.sleep(0.0005)
                reader.close()
                if up_vec is None:
                    noops += runs_at_input is not None
                    timeouts += runs_at_input is None
                    continue
                if trial < 3:
                    continue
                up_lat.append((t_up - t_send) * 1e3)
                if t_vis is not None:
                    vis_lat.append((t_vis - t_send) * 1e3)
                else:
                    timeouts += 1                 # published but never applied: lost
                if seen is not None:
                    lat.append((seen - t_send) * 1e3)
                else:
                    unchanged_lists += 1          # applied, but the top 10 did not change
            upd_topic.close()
            in_topic.close()
            conn.close()
        finally:
            stop.set()
            speed.close()
            serving.close()
        vis_a = np.asarray(vis_lat)
        up_a = np.asarray(up_lat)
        lat_a = np.asarray(lat)
        pct = lambda a, q: float(np.percentile(a, q)) if len(a) else None
        print(json.dumps({
            "metric": "ingest -> visible latency (POST /ingest -> speed UP -> the serving "
                      "model holds the user's new vector)",
            "p50_ms": pct(vis_a, 50), "p90_ms": pct(vis_a, 90),
            "max_ms": float(vis_a.max()) if len(vis_a) else None,
            "ingest_to_up_in_log_p50_ms": pct(up_a, 50), "ingest_to_up_in_log_p90_ms":
                pct(up_a, 90),
            "recommend_changed_p50_ms": pct(lat_a, 50), "recommend_changed_p90_ms":
                pct(lat_a, 90),
            "trials": len(vis_lat), "noop_foldins": noops, "lost_or_timeouts": timeouts,
            "applied_but_top10_unchanged": unchanged_lists, "interval_ms": args.interval_ms,
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
