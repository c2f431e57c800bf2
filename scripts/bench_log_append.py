#!/usr/bin/env python3
"""Update-log append cost of one speed-layer micro-batch's UP block (~14 MB, 20k messages):
the pwrite path, the mapped path with and without the preallocated / pre-faulted tail,
back to back and with an idle gap between appends (a speed layer appends once per
interval).  One JSON line per variant (medians of 10 appends after 2 warm-ups).

``python scripts/bench_log_append.py [--dir D]``; variants run as child processes because the
knobs (ORYX_LOG_MMAP_MIN, ORYX_LOG_PREALLOC) are read once per process."""

import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(gap: float, where: str) -> None:
    sys.path.insert(0, ROOT)
    import numpy as np
    from oryx_amd.api import MessageBlock
    from oryx_amd.transport.producer import LogTopicProducer
    g = np.random.default_rng(0)
    row = ",".join("%.7g" % x for x in g.normal(size=64))
    msgs = ['["X","U%d",[%s],["I%d"]]' % (j, row, j) for j in range(20000)]
    buf = ("\n".join(msgs) + "\n").encode()
    ends = np.cumsum([len(m) + 1 for m in msgs]) - 1
    blk = MessageBlock(np.frombuffer(buf, dtype=np.uint8).copy(), ends.astype(np.int64))
    logdir = tempfile.mkdtemp(dir=where)
    p = LogTopicProducer("log:" + logdir, "OryxUpdate", async_=False, max_message=1 << 30)
    times = []
    try:
        for r in range(12):
            time.sleep(gap)
            t0 = time.perf_counter()
            p.send_block("UP", blk)
            times.append((time.perf_counter() - t0) * 1e3)
    finally:
        p.close()
        shutil.rmtree(logdir, ignore_errors=True)
    t = sorted(times[2:])
    print(json.dumps({"mb": len(buf) / 1e6, "median_ms": t[len(t) // 2], "min_ms": t[0],
                      "max_ms": t[-1]}))


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(float(sys.argv[2]), sys.argv[3])
        return 0
    where = sys.argv[2] if len(sys.argv) > 2 and sys.argv[1] == "--dir" else \
        tempfile.gettempdir()
    variants = [("pwrite", {"ORYX_LOG_MMAP_MIN": "0"}),
                ("mapped_no_prealloc", {"ORYX_LOG_PREALLOC": "0"}),
                ("mapped_prealloc", {})]
    for name, env in variants:
        for gap in (0.0, 0.05):
            e = dict(os.environ, **env)
            out = subprocess.run([sys.executable, __file__, "--child", str(gap), where],
                                 env=e, capture_output=True, text=True, timeout=300)
            rec = json.loads(out.stdout.strip().splitlines()[-1]) if out.returncode == 0 \
                else {"error": out.stderr[-500:]}
            rec.update({"variant": name, "gap_s": gap, "dir": where})
            print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
