"""Speed-layer latency while the batch layer trains on the same GPU.

The speed layer's micro-batch update (``ALSSpeedModelManager.build_update_blocks`` + the UP
block's append to an update log, exactly bench.py's speed measurement: 10k events against a
c2-sized rank-64 model) is timed idle, then again while another process runs ALS training
iterations on the same GPU (``bench.py --speed-events 0`` with a long timed loop; the speed
measurement starts once that loop has).  Prints one JSON line: idle and loaded median / p90,
their ratio, and the trainer's ms per iteration under the speed layer's load.

``python scripts/speed_under_load.py [--events 10000] [--reps 14] [--train-steps 5000]``
"""

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=14)
    ap.add_argument("--train-steps", type=int, default=5000)
    ap.add_argument("--users", type=int, default=162541)
    ap.add_argument("--items", type=int, default=59047)
    ap.add_argument("--k", type=int, default=64)
    args = ap.parse_args()

    import numpy as np
    import torch
    from oryx_amd.api import Dataset
    from oryx_amd.layers.speed import publish_blocks
    from oryx_amd.models.als.speed import ALSSpeedModel, ALSSpeedModelManager
    from oryx_amd.textlines import TextLines
    from oryx_amd.transport.producer import LogTopicProducer
    from oryx_amd.utils import config as cfg

    dev = torch.device("cuda", 0)
    g = np.random.default_rng(5)
    X = (g.standard_normal((args.users, args.k)) * 0.1).astype(np.float32)
    Y = (g.standard_normal((args.items, args.k)) * 0.1).astype(np.float32)
    mgr = ALSSpeedModelManager(cfg.get_default())
    model = ALSSpeedModel(args.k, True, dev)
    model.X.set_vectors(["U%d" % j for j in range(len(X))], X)
    model.Y.set_vectors(["I%d" % j for j in range(len(Y))], Y)
    mgr.model = model
    B = args.events
    now = int(time.time() * 1000)
    lines = ["U%d,I%d,%.2f,%d" % (a, b, v, now) for a, b, v in
             zip(g.integers(0, len(X), B).tolist(), g.integers(0, len(Y), B).tolist(),
                 (g.random(B) * 4 + 0.5).tolist())]
    ds = Dataset.from_values(TextLines.from_strings(lines))
    logdir = tempfile.mkdtemp(prefix="oryx_speed_load_")
    producer = LogTopicProducer("log:" + logdir, "OryxUpdate", async_=False,
                                max_message=1 << 30)

    def measure(reps):
        times, phases = [], []
        for rep in range(reps):
            model.X.version += 1          # the factors changed: inverses recomputed
            time.sleep(0.05)              # micro-batches arrive one per interval
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            pub = {}
            publish_blocks(producer, mgr.build_update_blocks(ds), pub)
            t2 = time.perf_counter()
            if rep >= 2:
                times.append((t2 - t1) * 1e3)
                ph = dict(mgr.last_phase_ms)
                ph["publish_write"] = pub.get("write_ms", 0.0)
                phases.append(ph)
        med = {k: float(np.median([p.get(k, 0.0) for p in phases])) for k in phases[0]}
        return float(np.median(times)), float(np.percentile(times, 90)), med, times

    try:
        idle50, idle90, idle_ph, idle_t = measure(args.reps)
        mark = os.path.join(logdir, "timed")
        env = dict(os.environ, ORYX_BENCH_TIMED_MARK=mark)
        child = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--steps",
                                  str(args.train_steps), "--warmup", "3", "--speed-events", "0"],
                                 env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                 text=True)
        t_wait = time.time()
        while not os.path.exists(mark):
            if child.poll() is not None:
                raise RuntimeError("trainer exited before its timed loop")
            if time.time() - t_wait > 240:
                child.kill()
                raise RuntimeError("trainer did not start")
            time.sleep(0.02)
        t_loaded0 = time.time()
        load50, load90, load_ph, load_t = measure(args.reps)
        t_loaded1 = time.time()
        out, _ = child.communicate(timeout=600)
        train = json.loads(out.strip().splitlines()[-1])
        # the trainer must still have been running when the loaded measurement ended
        overlap = train["ms_per_step"] * args.train_steps / 1e3 > (t_loaded1 - t_loaded0)
        print(json.dumps({
            "metric": "speed-layer update latency, idle vs during batch-layer ALS training "
                      "on the same GPU",
            "events": B, "k": args.k, "users": args.users, "items": args.items,
            "idle_ms": idle50, "idle_p90_ms": idle90,
            "loaded_ms": load50, "loaded_p90_ms": load90,
            "loaded_over_idle": load50 / idle50,
            "idle_phase_ms": idle_ph, "loaded_phase_ms": load_ph,
            "idle_times_ms": idle_t, "loaded_times_ms": load_t,
            "trainer_ms_per_step_under_load": train["ms_per_step"],
            "trainer_steps": args.train_steps, "loaded_window_s": t_loaded1 - t_loaded0,
            "trainer_covered_window": bool(overlap),
        }), flush=True)
    finally:
        producer.close()
        shutil.rmtree(logdir, ignore_errors=True)


if __name__ == "__main__":
    main()
