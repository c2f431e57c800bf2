"""Host -> device copy of a large pageable text buffer (the device CSV parse's input,
models/features.py h2d): plain copy_ vs the pinned, natively staged pipeline.  One JSON line.

Usage: python scripts/h2d_probe.py [GB]
"""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oryx_amd import hostbuf, native
from oryx_amd.models.features import h2d


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    n = int(gb * (1 << 30))
    native.runtime()
    buf = hostbuf.empty(n)
    buf[::4096] = 7
    buf[-1] = 3
    dst = torch.empty(n + 32, dtype=torch.uint8, device="cuda")
    out = {"gb": gb}
    for staged in (False, True, False, True):
        torch.cuda.synchronize()
        t = time.perf_counter()
        h2d(buf, 0, n, dst, staged=staged)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        key = "staged" if staged else "pageable"
        out.setdefault(key + "_s", []).append(round(dt, 4))
        assert int(dst[n - 1]) == 3 and int(dst[4096 * 5]) == 7
    out["pageable_gbps"] = round(gb * 1.0737 / min(out["pageable_s"]), 2)
    out["staged_gbps"] = round(gb * 1.0737 / min(out["staged_s"]), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
