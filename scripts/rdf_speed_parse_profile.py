"""Where the RDF speed layer's device parse of a 10k-line micro-batch (100 numeric features +
a categorical target, ~700 B per line) spends its time: the device parse's own laps
(features._device_block) and a cProfile of features.parse_features (top 30 by cumulative time).

    python scripts/rdf_speed_parse_profile.py [--events 10000] [--features 100]
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
    ap.add_argument("--features", type=int, default=100)
    args = ap.parse_args()
    import numpy as np
    import torch
    from oryx_amd.models import features as feat
    from oryx_amd.models.schema import InputSchema
    from oryx_amd.textlines import TextLines
    from oryx_amd.utils import config as cfg
    P = args.features
    conf = cfg.overlay_on({
        "oryx.input-schema.feature-names": "[%s]" % ",".join('"%d"' % j for j in range(P + 1)),
        "oryx.input-schema.categorical-features": '["%d"]' % P,
        "oryx.input-schema.target-feature": '"%d"' % P}, cfg.get_default())
    schema = InputSchema(conf)
    g = np.random.default_rng(5)
    xs = g.standard_normal((args.events, P))
    lines = [",".join("%.6f" % v for v in row) + "," + str(int(row[0] > 0)) for row in xs]
    tl = TextLines.from_strings(lines)
    dev = torch.device("cuda:0")
    laps, totals = [], []
    for rep in range(8):
        hist = feat.FeatureHistory(dev, keep=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        blk = hist.parse(tl, schema, torch.float64)
        torch.cuda.synchronize()
        totals.append((time.perf_counter() - t0) * 1e3)
        laps.append({k: v * 1e3 for k, v in hist.stats.get("device_parse_s", {}).items()})
    res = {"events": args.events, "features": P, "bytes": int(tl.nbytes()),
           "parse_ms_median": float(np.median(totals[2:])),
           "laps_ms": {k: float(np.median([l.get(k, 0.0) for l in laps[2:]])) for k in laps[-1]}}
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        feat.parse_features(tl, schema, dev, torch.float64)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    res["cprofile_5_parses_by_tottime"] = s.getvalue().splitlines()[:50]
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
