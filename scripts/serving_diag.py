#!/usr/bin/env python3
"""Where a /recommend request's time goes in a model loaded from the update log
(bench_traffic's setup): model.top_n directly, then over HTTP back-to-back and with gaps."""
import http.client
import json
import os
import shutil
import sys
import tempfile
import time
import cProfile
import pstats
import io

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if os.environ.get("DIAG_SWITCH"):
        sys.setswitchinterval(float(os.environ["DIAG_SWITCH"]))
    import bench_serving
    import bench_traffic
    from oryx_amd.serving.layer import ServingLayer
    from oryx_amd.utils import config as cfg
    items, users, k = 1_000_000, 200_000, 50
    work = tempfile.mkdtemp(prefix="oryx_diag_")
    root = os.path.join(work, "log")
    data = bench_serving.make_data(items, users, k, 7)
    Y = data[0]
    bench_traffic.write_model_log(root, data, k)
    extra = {}
    if os.environ.get("DIAG_ID"):
        extra["oryx.id"] = '"traffic-bench"'
    if os.environ.get("DIAG_SPEEDCLS"):
        extra["oryx.speed.model-manager-class"] = \
            "com.cloudera.oryx.app.speed.als.ALSSpeedModelManager"
    conf = cfg.overlay_on(dict(extra, **{
        "oryx.transport.log-dir": '"%s"' % root,
        "oryx.update-topic.message.max-size": 1 << 30,
        "oryx.serving.api.port": 0,
        "oryx.als.sample-rate": 0.3,
        "oryx.serving.model-manager-class":
            "com.cloudera.oryx.app.serving.als.model.ALSServingModelManager",
        "oryx.serving.application-resources":
            '"com.cloudera.oryx.app.serving,com.cloudera.oryx.app.serving.als"',
    }), cfg.get_default())
    layer = ServingLayer(conf, host="127.0.0.1").start()
    while True:
        m = layer.manager.get_model()
        if m is not None and m.get_fraction_loaded() >= 1.0 and m.get_num_items() == items \
                and m.get_num_users() == users:
            break
        time.sleep(0.05)
    lsh = getattr(m, "lsh", None)
    out = {"lsh_hashes": len(lsh.hash_vectors) if lsh is not None else None}
    m.top_n(Y[0], 10)
    if os.environ.get("DIAG_NOWARM"):
        import argparse
        args = argparse.Namespace(workers=4, interval_ms=2.0, users=users, items=items,
                                  duration_s=8.0)
        print(json.dumps({"nowarm_idle4": bench_traffic.run_phase(
            layer.actual_port, args, {"recommend": 1.0}, 3)}), flush=True)
    t = time.perf_counter()
    for j in range(200):
        m.top_n(Y[j], 10)
    out["top_n_ms"] = (time.perf_counter() - t) * 1e3 / 200
    conn = http.client.HTTPConnection("127.0.0.1", layer.actual_port, timeout=30)
    def get(p):
        conn.request("GET", p, headers={"Accept": "application/json"})
        r = conn.getresponse()
        r.read()
    for j in range(20):
        get("/recommend/U%d" % j)
    t = time.perf_counter()
    for j in range(200):
        get("/recommend/U%d" % j)
    out["http_b2b_ms"] = (time.perf_counter() - t) * 1e3 / 200
    lat = []
    for j in range(100):
        t = time.perf_counter()
        get("/recommend/U%d" % (j + 300))
        lat.append((time.perf_counter() - t) * 1e3)
        time.sleep(0.008)
    out["http_gap8ms_ms"] = float(np.mean(lat))
    # bench_traffic's idle phase: 4 client processes, exponential gaps (mean 8 ms each)
    import argparse
    b0 = (m.batcher.batches, m.batcher.requests, m.batcher.inline) if m.batcher else None
    args = argparse.Namespace(workers=4, interval_ms=2.0, users=users, items=items,
                              duration_s=8.0)
    res = bench_traffic.run_phase(layer.actual_port, args, {"recommend": 1.0}, 3)
    out["idle4"] = res
    if b0 is not None:
        out["batcher"] = {"batches": m.batcher.batches - b0[0],
                          "requests": m.batcher.requests - b0[1],
                          "inline": m.batcher.inline - b0[2]}
    # the same with 1 client at the same per-client gap
    args.workers = 1
    args.interval_ms = 8.0
    out["idle1"] = bench_traffic.run_phase(layer.actual_port, args, {"recommend": 1.0}, 4)
    # the /recommend resource in this thread (no HTTP): where its time goes
    from oryx_amd.serving import http as ohttp
    router = layer._server.router
    def disp(u):
        req = ohttp.Request("GET", "/recommend/U%d" % u, {}, {"accept": "application/json"},
                            b"", layer.context)
        return router.dispatch(req)
    for j in range(20):
        disp(j)
    t = time.perf_counter()
    for j in range(200):
        disp(1000 + j)
    out["dispatch_ms"] = (time.perf_counter() - t) * 1e3 / 200
    pr = cProfile.Profile()
    pr.enable()
    for j in range(100):
        disp(2000 + j)
    pr.disable()
    sio = io.StringIO()
    pstats.Stats(pr, stream=sio).sort_stats("cumulative").print_stats(30)
    out["dispatch_profile"] = sio.getvalue()[:5000]
    if m.batcher is not None:
        out["batcher_state"] = {"contended": m.batcher._contended, "busy": m.batcher._busy,
                                "last_scan_ms": m.batcher._last_scan_s * 1e3,
                                "wait_s": m.batcher.wait_s}
    print(json.dumps(out), flush=True)
    layer.close()
    shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
    sys.stdout.flush()
    os._exit(0)
