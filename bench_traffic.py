#!/usr/bin/env python3
"""Serving under a mixed read / write load with the speed layer live (the reference's
``TrafficUtil``, ``app/oryx-app-serving/src/test/java/com/cloudera/oryx/app/traffic/
TrafficUtil.java:64-163``, with its ALS endpoint mix ``.../traffic/als/ALSEndpoint.java:44-66``:
``/pref`` 0.5, ``/recommend`` 0.3, ``/similarity`` 0.2).

An ALS model of ``--items`` x ``--features`` item vectors and ``--users`` users (Poisson(20)
known items each) is published into the update log as the batch layer does (MODEL + UP rows);
a serving layer (read-write, native HTTP) and a speed layer (ALS fold-in) load it from there.
``--workers`` client processes then issue requests with exponentially distributed gaps (each
client's mean gap is ``workers x --interval-ms``, as TrafficUtil's per-client interval), for
``--duration-s`` seconds per phase:

* idle: ``/recommend`` only, nothing written (the baseline latency);
* mix: the endpoint mix, while the speed layer runs a micro-batch every
  ``--speed-interval-ms``: every ``/pref`` goes POST -> input log -> fold-in -> ``UP`` rows
  for the user and the item -> the serving consumer -> the item index (moved items re-bucketed
  in place, ops/topn.py).

Prints one JSON line: per phase and endpoint the count, mean, stdev, p50 and p99 ms, errors;
the speed intervals run and UP rows published during the mix; the item index's re-sorts and
incremental refreshes during the mix (per speed interval), its delta-segment and dead rows.

``python bench_traffic.py --items 1000000 --features 50 --sample-rate 0.3``
"""

from __future__ import annotations

import argparse
import gc
import json
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CLIENT = r"""
import http.client, json, random, sys, time
port, users, items, dur, gap_ms, seed = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]),
                                         float(sys.argv[4]), float(sys.argv[5]), int(sys.argv[6]))
mix = json.loads(sys.argv[7])
names = list(mix)
weights = [mix[n] for n in names]
rnd = random.Random(seed)
conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
lat = {n: [] for n in names}
err = {n: 0 for n in names}
slow = []      # (wall-clock start, ms, endpoint) of requests over 25 ms
t_end = time.perf_counter() + dur
while time.perf_counter() < t_end:
    ep = rnd.choices(names, weights)[0]
    u = "U%d" % rnd.randrange(users)
    i = "I%d" % rnd.randrange(items)
    t = time.perf_counter()
    tw = time.time()
    try:
        if ep == "pref":
            conn.request("POST", "/pref/%s/%s" % (u, i), body=str(rnd.randint(1, 5)).encode(),
                         headers={"Content-Type": "text/plain"})
        elif ep == "recommend":
            conn.request("GET", "/recommend/" + u, headers={"Accept": "application/json"})
        else:
            conn.request("GET", "/similarity/" + i, headers={"Accept": "application/json"})
        r = conn.getresponse()
        r.read()
        ok = r.status < 400
    except Exception:
        ok = False
        conn.close()
        conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    el = (time.perf_counter() - t) * 1e3
    lat[ep].append(el)
    err[ep] += 0 if ok else 1
    if el > 25.0:
        slow.append((tw, el, ep))
    if gap_ms > 0:
        want = rnd.expovariate(1.0 / gap_ms)
        if el < want:
            time.sleep((want - el) / 1e3)
print(json.dumps({"lat": lat, "err": err, "slow": slow}))
"""


def write_model_log(root, data, features):
    """MODEL + UP rows into the update topic at ``root`` (the batch layer's publish)."""
    from oryx_amd import ingest
    from oryx_amd.transport import log as tlog
    from oryx_amd.utils import pmml as pmmlu
    Y, X, item_ids, user_ids, counts, known = data
    items, users = len(item_ids), len(user_ids)
    tlog.maybe_create_topic(root, "OryxInput", 1)
    tlog.maybe_create_topic(root, "OryxUpdate", 1, max_message=1 << 30)
    topic = tlog.Topic(root, "OryxUpdate")
    doc = pmmlu.build_skeleton_pmml()
    for key, val in (("X", "X/"), ("Y", "Y/"), ("features", features), ("lambda", 0.001),
                     ("implicit", True), ("alpha", 1.0)):
        doc.add_extension(key, val)
    doc.add_extension_content("XIDs", user_ids)
    doc.add_extension_content("YIDs", item_ids)
    topic.append_batch([("MODEL", pmmlu.to_string(doc))])
    chunk = 1 << 20
    for lo in range(0, items, chunk):
        hi = min(items, lo + chunk)
        topic.append_block(ingest.assemble_row_messages(
            "Y", item_ids[lo:hi], ingest.format_float_rows_blob(Y[lo:hi])), key="UP")
        print("bench_traffic: log %d / %d item rows" % (hi, items), file=sys.stderr,
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


SPEED_CHILD = r"""
import json, os, sys, threading, time
sys.path.insert(0, sys.argv[1])
from oryx_amd.layers.speed import SpeedLayer
from oryx_amd.utils import config as cfg
conf = cfg.deserialize(open(sys.argv[2]).read())
users, interval_ms = int(sys.argv[3]), float(sys.argv[4])
speed = SpeedLayer(conf).start(start_timer=False)
t0 = time.time()
while True:
    sm = speed.manager.model
    if sm is not None and sm.get_fraction_loaded() >= 1.0 and sm.X.size() == users:
        break
    time.sleep(0.05)
# the manager warms a completely loaded model on its consumer thread (row maps, device
# mirrors, Gramians: ALSSpeedModel.warm); wait for it like a deployment's first interval would
t1 = time.time()
mgr = speed.manager
while mgr.warm_s is None:
    time.sleep(0.05)
print(json.dumps({"loaded_s": t1 - t0, "warm_s": time.time() - t1,
                  "manager_warm_s": mgr.warm_s}), flush=True)
assert sys.stdin.readline().strip() == "go"
stop = threading.Event()
durs = []
phases = []
def run():
    while not stop.is_set():
        t = time.perf_counter()
        speed.run_interval()
        dt = time.perf_counter() - t
        durs.append(dt * 1e3)
        phases.append(dict(getattr(mgr, "last_phase_ms", {}) or {}))
        if interval_ms / 1e3 > dt:
            stop.wait(interval_ms / 1e3 - dt)
th = threading.Thread(target=run, daemon=True)
th.start()
sys.stdin.readline()
stop.set()
th.join(120)
print(json.dumps({"intervals": speed.intervals_run, "up_rows": speed.updates_sent,
                  "interval_ms": durs, "interval_phase_ms": phases}), flush=True)
speed.close()
os._exit(0)
"""


class _GcPauses:
    """Times the serving interpreter's cyclic-GC passes (a gen-2 pass over a big heap stops
    every handler thread)."""

    def __init__(self):
        self.t = None
        self.ms = {0: [], 1: [], 2: []}
        gc.callbacks.append(self._cb)

    def _cb(self, phase, info):
        if phase == "start":
            self.t = time.perf_counter()
        elif self.t is not None:
            self.ms[info["generation"]].append((time.perf_counter() - self.t) * 1e3)

    def take(self):
        out = {"gen%d" % g: {"n": len(v), "max_ms": max(v) if v else 0.0,
                             "total_ms": sum(v)} for g, v in self.ms.items()}
        self.ms = {0: [], 1: [], 2: []}
        return out


def _stats(v):
    a = np.asarray(v, dtype=np.float64)
    if not len(a):
        return {"n": 0}
    return {"n": int(len(a)), "mean_ms": float(a.mean()), "stdev_ms": float(a.std()),
            "p50_ms": float(np.percentile(a, 50)), "p99_ms": float(np.percentile(a, 99)),
            "max_ms": float(a.max())}


def _index_counters(model):
    idx = getattr(model, "index", None)
    if idx is None:
        return {}
    shards = getattr(idx, "shards", None) or [idx]
    return {"rebuilds": sum(s.rebuilds for s in shards),
            "incremental": sum(getattr(s, "incremental", 0) for s in shards),
            "delta_added": sum(getattr(s, "delta_added", 0) for s in shards),
            "dead": sum(getattr(s, "n_dead", 0) for s in shards),
            "delta_rows": sum(getattr(s, "n", 0) - getattr(s, "n_main", 0) for s in shards)}


def _server_side(serving):
    """(endpoint -> (seconds sum, count)) of the serving layer's request histograms."""
    out = {}
    for (name, labels), h in list(serving.metrics._hist.items()):
        if name == "oryx_http_request_seconds":
            out[dict(labels).get("endpoint")] = (h.sum, h.n)
    return out


def _server_delta(a, b):
    return {ep: {"server_mean_ms": 1e3 * (b[ep][0] - a.get(ep, (0, 0))[0]) /
                 max(1, b[ep][1] - a.get(ep, (0, 0))[1]),
                 "server_n": b[ep][1] - a.get(ep, (0, 0))[1]} for ep in b}


class _Sampler:
    """Poor man's profiler: samples every thread's Python stack every 2 ms (--sample)."""

    def __init__(self):
        import collections
        self.counts = collections.Counter()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        me = threading.get_ident()
        names = {}
        while not self._stop.is_set():
            for th in threading.enumerate():
                names[th.ident] = th.name
            for tid, fr in sys._current_frames().items():
                if tid == me:
                    continue
                stack = []
                f = fr
                while f is not None and len(stack) < 4:
                    stack.append("%s:%d" % (f.f_code.co_name, f.f_lineno))
                    f = f.f_back
                self.counts[(names.get(tid, "?")[:20], " < ".join(stack))] += 1
            time.sleep(0.002)

    def start(self):
        self._t.start()
        return self

    def stop(self, top=25):
        self._stop.set()
        self._t.join()
        return [(n, st, c) for (n, st), c in self.counts.most_common(top)]


def run_phase(port, args, mix, seed):
    gap = args.workers * args.interval_ms
    t_start = time.time()
    procs = [subprocess.Popen([sys.executable, "-c", CLIENT, str(port), str(args.users),
                               str(args.items), str(args.duration_s), str(gap),
                               str(seed * 1000 + w), json.dumps(mix)],
                              stdout=subprocess.PIPE, text=True)
             for w in range(args.workers)]
    outs = [json.loads(p.communicate()[0]) for p in procs]
    lat = {ep: sum((o["lat"][ep] for o in outs), []) for ep in mix}
    err = {ep: sum(o["err"][ep] for o in outs) for ep in mix}
    res = {ep: dict(_stats(lat[ep]), errors=err[ep]) for ep in mix}
    slow = sorted((tuple(x) for o in outs for x in o.get("slow", [])), key=lambda x: -x[1])
    res["_slow"] = slow[:40]
    res["_t_start"] = t_start
    return res


class _StallWatch:
    """A thread that sleeps 1 ms at a time in the serving process and records every wake-up
    that came more than 15 ms late (wall-clock time, ms): a pause of the whole interpreter --
    a GIL held by a long native call, a GC pass -- shows up here, and the record lines it up
    with the slow requests and the UP applications."""

    def __init__(self, dump_path=None):
        self.stalls = []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name="stall-watch")
        # faulthandler's watchdog is a C thread: armed for 20 ms on every wake-up, it dumps
        # every Python thread's stack WITHOUT the GIL when a wake-up is that late -- the stack
        # of whoever holds the interpreter during the stall
        self._dump = open(dump_path, "w") if dump_path else None

    def _run(self):
        import faulthandler
        last = time.perf_counter()
        while not self._stop.is_set():
            if self._dump is not None:
                faulthandler.dump_traceback_later(0.02, repeat=False, file=self._dump)
            time.sleep(0.001)
            if self._dump is not None:
                faulthandler.cancel_dump_traceback_later()
            now = time.perf_counter()
            if now - last > 0.015:
                self.stalls.append((time.time() - (now - last), (now - last) * 1e3))
            last = now

    def start(self):
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        self._t.join()
        if self._dump is not None:
            self._dump.close()
        return self.stalls


def _attribute_slow(slow, stalls, applies, t_start, index_events=(), scans=()):
    """Per slow request (start, ms, endpoint): when it started (seconds into the phase), and
    the serving-process stalls, UP applications, index refreshes / bf16 conversions and slow
    scan batches whose time overlaps it."""
    out = []

    def over(ev, t0, t1):
        return ev[0] < t1 and ev[0] + ev[1] / 1e3 > t0
    for t0, ms, ep in slow:
        t1 = t0 + ms / 1e3
        st = [round(d, 1) for (s0, d) in stalls if s0 < t1 and s0 + d / 1e3 > t0]
        ap = [(round(d, 1), n) for (s0, d, n) in applies if s0 < t1 and s0 + d / 1e3 > t0]
        ix = [(round(e[1], 1), e[2], e[3]) + tuple(e[4:]) for e in index_events
              if over(e, t0, t1)]
        sc = [(round(e[0] - t_start, 3), round(e[1], 1), e[2]) for e in scans if over(e, t0, t1)]
        out.append({"ms": round(ms, 1), "endpoint": ep, "at_s": round(t0 - t_start, 3),
                    "stalls_ms": st, "up_apply": ap, "index": ix, "scan_batches": sc})
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--users", type=int, default=200_000)
    ap.add_argument("--features", type=int, default=50)
    ap.add_argument("--sample-rate", type=float, default=0.3)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--interval-ms", type=float, default=2.0,
                    help="TrafficUtil's requestIntervalMS: mean gap between requests over all "
                         "clients (each client: workers x this)")
    ap.add_argument("--duration-s", type=float, default=20.0, help="per phase")
    ap.add_argument("--speed-interval-ms", type=float, default=1000.0)
    ap.add_argument("--mix", default="pref=0.5,recommend=0.3,similarity=0.2")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--settle-s", type=float, default=5.0,
                    help="after the load: requests for this long before timing (warm-up)")
    ap.add_argument("--sample", action="store_true",
                    help="sample the server's Python stacks during the idle phase")
    ap.add_argument("--no-speed", action="store_true",
                    help="no speed layer in the process (A/B: the idle phase without it)")
    args = ap.parse_args(argv)
    import bench_serving
    import torch
    from oryx_amd.serving.layer import ServingLayer
    from oryx_amd.utils import config as cfg

    mix = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in args.mix.split(",")}
    work = tempfile.mkdtemp(prefix="oryx_traffic_", dir=os.environ.get("ORYX_TTR_DIR"))
    root = os.path.join(work, "log")
    rec = {"metric": "serving latency under the TrafficUtil mix with the speed layer live",
           "items": args.items, "users": args.users, "features": args.features,
           "sample_rate": args.sample_rate, "workers": args.workers,
           "interval_ms": args.interval_ms, "speed_interval_ms": args.speed_interval_ms,
           "duration_s": args.duration_s, "mix": mix}
    try:
        t0 = time.perf_counter()
        data = bench_serving.make_data(args.items, args.users, args.features, args.seed)
        write_model_log(root, data, args.features)
        del data
        rec["log_build_s"] = time.perf_counter() - t0
        conf = cfg.overlay_on({
            "oryx.id": '"traffic-bench"',
            "oryx.transport.log-dir": '"%s"' % root,
            "oryx.update-topic.message.max-size": 1 << 30,
            "oryx.serving.api.port": 0,
            "oryx.als.sample-rate": args.sample_rate,
            "oryx.speed.model-manager-class":
                "com.cloudera.oryx.app.speed.als.ALSSpeedModelManager",
            "oryx.serving.model-manager-class":
                "com.cloudera.oryx.app.serving.als.model.ALSServingModelManager",
            "oryx.serving.application-resources":
                '"com.cloudera.oryx.app.serving,com.cloudera.oryx.app.serving.als"',
        }, cfg.get_default())
        t0 = time.perf_counter()
        serving = ServingLayer(conf, host="127.0.0.1").start()
        # the speed layer in its own process, as deployed (oryx-run.sh speed): it shares the
        # GPU with the serving layer, not its interpreter
        speed = None
        if not args.no_speed:
            conf_path = os.path.join(work, "speed.conf")
            with open(conf_path, "w") as fh:
                fh.write(cfg.serialize(conf))
            speed = subprocess.Popen([sys.executable, "-c", SPEED_CHILD, ROOT, conf_path,
                                      str(args.users), str(args.speed_interval_ms)],
                                     stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        try:
            while True:
                vm = serving.manager.get_model()
                if vm is not None and vm.get_fraction_loaded() >= 1.0 and \
                        vm.get_num_users() == args.users and vm.get_num_items() == args.items:
                    break
                if time.perf_counter() - t0 > 3000:
                    raise TimeoutError("model not loaded")
                if int((time.perf_counter() - t0) * 50) % 500 == 0:
                    print("bench_traffic: loading, %.0f s" % (time.perf_counter() - t0),
                          file=sys.stderr, flush=True)
                time.sleep(0.02)
            rec["load_s"] = time.perf_counter() - t0
            t_w = time.perf_counter()
            while getattr(serving.manager, "warm_s", 0.0) is None and \
                    time.perf_counter() - t_w < 60:
                time.sleep(0.02)
            rec["serving_warm_s"] = getattr(serving.manager, "warm_s", None)
            if speed is not None:
                ld = json.loads(speed.stdout.readline())
                rec["speed_load_s"], rec["speed_warm_s"] = ld["loaded_s"], ld["warm_s"]
                rec["speed_manager_warm_s"] = ld.get("manager_warm_s")
            vm = serving.manager.get_model()
            vm.top_n(np.zeros(args.features, np.float32), 10)   # device mirror + index
            port = serving.actual_port
            # warm-up: the same traffic, untimed
            if args.settle_s > 0:
                import argparse as _ap
                run_phase(port, _ap.Namespace(**dict(vars(args), duration_s=args.settle_s)),
                          {"recommend": 1.0}, args.seed + 17)
            # ---- idle baseline: /recommend only, nothing written
            print("bench_traffic: idle phase", file=sys.stderr, flush=True)
            gcp = _GcPauses()
            s0 = _server_side(serving)
            smp = _Sampler().start() if args.sample else None
            rec["idle"] = run_phase(port, args, {"recommend": 1.0}, args.seed)
            rec["idle"].pop("_slow", None)
            rec["idle"].pop("_t_start", None)
            if smp is not None:
                rec["idle_stack_samples"] = smp.stop()
            rec["idle_server"] = _server_delta(s0, _server_side(serving))
            rec["idle_gc"] = gcp.take()
            if speed is None:
                return 0 if print(json.dumps(rec), flush=True) is None else 0
            # ---- the mix with the speed layer live
            c0 = _index_counters(vm)
            speed.stdin.write("go\n")
            speed.stdin.flush()
            print("bench_traffic: mix phase", file=sys.stderr, flush=True)
            s0 = _server_side(serving)
            dump = os.path.join(work, "stall_stacks.txt")
            sw = _StallWatch(dump).start()
            rec["mix_phase"] = run_phase(port, args, mix, args.seed + 1)
            stalls = sw.stop()
            slow = rec["mix_phase"].pop("_slow", [])
            t_mix = rec["mix_phase"].pop("_t_start")
            mgr = serving.manager
            # (UP applications of the mix phase only: the model load's are long and earlier)
            applies = [a for a in getattr(mgr, "apply_log", []) if a[0] >= t_mix]
            rec["mix_attribution"] = {
                "stalls": [(round(t - t_mix, 3), round(d, 1))
                           for t, d in sorted(stalls, key=lambda x: -x[1])[:20]],
                "up_apply_ms": _stats([d for _, d, _ in applies]) if applies else None,
                "slow_requests": _attribute_slow(
                    slow, stalls, applies, t_mix,
                    list(getattr(getattr(vm, "index", None), "event_log", [])),
                    list(getattr(getattr(vm, "batcher", None), "slow_log", []))),
                # the interpreter's stacks during each stall (faulthandler, see _StallWatch)
                "stall_stacks": open(dump).read()[:20000] if os.path.exists(dump) else None}
            rec["mix_server"] = _server_delta(s0, _server_side(serving))
            rec["mix_gc"] = gcp.take()
            speed.stdin.write("stop\n")
            speed.stdin.flush()
            sp = json.loads(speed.stdout.readline())
            # let the last UP rows reach the serving model, then count what the index did
            time.sleep(1.0)
            vm.top_n(np.zeros(args.features, np.float32), 10)
            c1 = _index_counters(vm)
            runs = sp["intervals"]
            rec["speed"] = {"intervals": runs, "up_rows": sp["up_rows"],
                            "interval_ms": _stats(sp["interval_ms"]),
                            "process": "separate (as deployed)",
                            # every interval: its duration and the manager's phases
                            "per_interval": [dict(ms=d, phases=p) for d, p in
                                             zip(sp["interval_ms"],
                                                 sp.get("interval_phase_ms", []))]}
            rec["index"] = {k: c1.get(k, 0) - c0.get(k, 0) for k in ("rebuilds", "incremental",
                                                                    "delta_added")}
            rec["index"].update(delta_rows_now=c1.get("delta_rows"), dead_now=c1.get("dead"))
            rec["index"]["rebuilds_per_interval"] = rec["index"]["rebuilds"] / max(runs, 1)
            idle99 = rec["idle"]["recommend"].get("p99_ms")
            mix99 = rec["mix_phase"].get("recommend", {}).get("p99_ms")
            rec["recommend_p99_mix_over_idle"] = (mix99 / idle99) if idle99 and mix99 else None
        finally:
            if speed is not None and speed.poll() is None:
                speed.kill()
                speed.wait(30)
            serving.close()
        if torch.cuda.is_available():
            rec["device"] = torch.cuda.get_device_name(0)
        print(json.dumps(rec), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)
    return 0


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)
