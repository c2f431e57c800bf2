"""Part-file write throughput on the box's temp filesystem: one 8 GB file with one write()
vs the same bytes as 2 / 4 / 8 files written concurrently.  One JSON line.

Usage: python scripts/write_probe.py [GB]
"""

import json
import os
import shutil
import sys
import tempfile
import threading
import time

import numpy as np

GB = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0


def main():
    n = int(GB * (1 << 30))
    buf = np.empty(n, dtype=np.uint8)
    buf[::4096] = 49
    d = tempfile.mkdtemp()
    out = {"gb": GB, "dir": d, "fs": None}
    try:
        out["fs"] = os.popen("df -T %s | tail -1" % d).read().split()[1]
    except Exception:
        pass
    for parts in (1, 2, 4, 8, 1):
        edges = [n * j // parts for j in range(parts + 1)]

        def w(j):
            with open(os.path.join(d, "part-%05d.txt" % j), "wb") as f:
                f.write(memoryview(buf[edges[j]:edges[j + 1]]))

        t = time.perf_counter()
        ts = [threading.Thread(target=w, args=(j,)) for j in range(parts)]
        for x in ts:
            x.start()
        for x in ts:
            x.join()
        dt = time.perf_counter() - t
        out.setdefault("s", []).append([parts, round(dt, 3), round(GB / dt, 2)])
        for f in os.listdir(d):
            os.remove(os.path.join(d, f))
    shutil.rmtree(d, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
