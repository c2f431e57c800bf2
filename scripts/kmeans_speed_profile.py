"""Phase profile of the k-means speed layer's micro-batch (KMeansSpeedModelManager
.build_updates on the GPU path) at the bench_kmeans.py shape: k = 1000 centers x 256 dims,
10k new points per micro-batch.  Prints the manager's per-phase medians, the device parse's own
laps (features._device_block) and a cProfile of one micro-batch (top 30 by cumulative time).

    python scripts/kmeans_speed_profile.py [--events 10000] [--k 1000] [--dim 256]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--reps", type=int, default=12)
    args = ap.parse_args()
    import numpy as np
    import torch
    from oryx_amd.api import Dataset
    from oryx_amd.models import features as feat
    from oryx_amd.models.kmeans.common import ClusterInfo
    from oryx_amd.models.kmeans.speed import KMeansSpeedModel, KMeansSpeedModelManager
    from oryx_amd.models.schema import InputSchema
    from oryx_amd.textlines import TextLines
    from oryx_amd.utils import config as cfg
    dev = torch.device("cuda:0")
    k, d = args.k, args.dim
    conf = cfg.overlay_on({
        "oryx.input-schema.feature-names": "[%s]" % ",".join('"f%d"' % j for j in range(d)),
        "oryx.input-schema.categorical-features": "[]"}, cfg.get_default())
    g = np.random.default_rng(11)
    centers = g.standard_normal((k, d)) * 4
    mgr = KMeansSpeedModelManager(conf)
    mgr.model = KMeansSpeedModel([ClusterInfo(j, centers[j], 10) for j in range(k)], dev)
    pts = centers[g.integers(0, k, args.events)] + g.standard_normal((args.events, d))
    lines = [",".join("%.6f" % v for v in row) for row in pts]
    ds = Dataset.from_values(TextLines.from_strings(lines))
    phases, times = [], []
    for rep in range(args.reps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = mgr.build_updates(ds)
        times.append((time.perf_counter() - t0) * 1e3)
        phases.append(dict(mgr.last_phase_ms))
    times, phases = times[2:], phases[2:]
    res = {"events": args.events, "k": k, "dim": d, "messages": len(out),
           "build_ms_median": float(np.median(times)),
           "phase_ms": {key: float(np.median([p[key] for p in phases])) for key in phases[0]}}
    # the device parse's laps
    schema = InputSchema(conf)
    hist = feat.FeatureHistory(dev, keep=False)
    laps = []
    for rep in range(6):
        hist.stats.pop("device_parse_s", None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        blk = hist.parse(ds.values(), schema, torch.float64)
        x = blk.predictors(schema)
        torch.cuda.synchronize()
        lp = {key: v * 1e3 for key, v in hist.stats.get("device_parse_s", {}).items()}
        lp["total"] = (time.perf_counter() - t0) * 1e3
        laps.append(lp)
    laps = laps[2:]
    res["parse_laps_ms"] = {key: float(np.median([l.get(key, 0.0) for l in laps]))
                            for key in laps[0]}
    pr = cProfile.Profile()
    pr.enable()
    mgr.build_updates(ds)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(30)
    res["cprofile_top"] = s.getvalue().splitlines()[:60]
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
