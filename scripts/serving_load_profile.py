"""Where serving model load (bench_serving.py --time-to-ready) spends its time: wall time of
the update iterator's frame poll, the native UP parse, the ID / known-item code step and the
apply to the model store, summed over the load.  Usage:
    python scripts/serving_load_profile.py ITEMS USERS [FEATURES]"""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench_serving  # noqa: E402
from oryx_amd import ingest  # noqa: E402
from oryx_amd.models.als import serving as als_serving  # noqa: E402
from oryx_amd.transport import log as tlog  # noqa: E402

T = {}


def _wrap(obj, name, key):
    f = getattr(obj, name)

    def w(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[key] = T.get(key, 0.0) + time.perf_counter() - t
    setattr(obj, name, w)


def main():
    items, users = int(sys.argv[1]), int(sys.argv[2])
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 250
    _wrap(ingest, "parse_up_records", "parse_total_s")
    _wrap(ingest, "_up_ids_codes", "ids_known_codes_s")
    _wrap(als_serving, "apply_up_parsed", "apply_s")
    _wrap(tlog.PartitionReader, "poll_frames", "poll_frames_s")
    r = bench_serving.time_to_ready(items, users, k, 7)
    out = {key: r[key] for key in ("items", "users", "features", "update_log_gb", "ready_s",
                                   "rows_per_s")}
    out.update({key: round(v, 3) for key, v in sorted(T.items())})
    out["native_parse_s"] = round(T.get("parse_total_s", 0) - T.get("ids_known_codes_s", 0), 3)
    out["cpus"] = len(os.sched_getaffinity(0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
