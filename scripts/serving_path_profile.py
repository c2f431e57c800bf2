"""Where a /recommend request's time goes without HTTP: the recommend resource called in a
loop on one thread (model lookups, LSH candidates, known-item exclusion, the top-N scan,
result formatting), timed, then under cProfile (top functions by cumulative time).

``python scripts/serving_path_profile.py [--items 1000000] [--features 50] [--rate 0.3]``
"""

import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench_serving  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--users", type=int, default=500_000)
    ap.add_argument("--features", type=int, default=50)
    ap.add_argument("--rate", type=float, default=0.3)
    ap.add_argument("--n", type=int, default=2000)
    args = ap.parse_args()
    import numpy as np
    from oryx_amd.models.als import resources
    from oryx_amd.serving import http as ohttp
    data = bench_serving.make_data(args.items, args.users, args.features, 7)
    model = bench_serving.build_model(data, args.features, args.rate)

    from oryx_amd.serving import resources as sres
    from oryx_amd.utils import config as cfg

    class _Mgr:
        def get_model(self):
            return model

        def get_config(self):
            return cfg.get_default()

    ctx = {sres.MODEL_MANAGER_KEY: _Mgr()}
    rnd = np.random.default_rng(1)
    users = ["U%d" % u for u in rnd.integers(0, args.users, args.n)]

    def one(u):
        req = ohttp.Request("GET", "/recommend/" + u, {}, {}, b"", ctx)
        return resources.recommend(req, u)

    for u in users[:100]:
        one(u)
    t0 = time.perf_counter()
    for u in users:
        one(u)
    per = (time.perf_counter() - t0) / len(users) * 1e3
    pr = cProfile.Profile()
    pr.enable()
    for u in users[:500]:
        one(u)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(35)
    print(json.dumps({"items": args.items, "features": args.features, "rate": args.rate,
                      "ms_per_request_no_http": per}), flush=True)
    print(s.getvalue())


if __name__ == "__main__":
    main()
