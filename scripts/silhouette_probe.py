"""Time the silhouette kernels on the k-means evaluation's shape (100k sample cap, d = 256,
k = 1000 clusters of skewed sizes).  One JSON line.

Usage: python scripts/silhouette_probe.py
"""

import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oryx_amd.models.kmeans import evaluation as ev  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(3)
    s, d, k = 100_000, 256, 1000
    x = torch.randn((s, d), device="cuda", dtype=torch.float64, generator=g)
    w = torch.from_numpy(np.random.default_rng(1).zipf(1.5, k).clip(1, 5000).astype(np.float64))
    idx = torch.multinomial(w, s, replacement=True).to("cuda")
    out = {"s": s, "d": d, "k": k, "rs64": os.environ.get("ORYX_KM_SIL_RS", "22 (default)")}
    # the MFMA kernel (default) and the VALU kernel it replaced, same sample
    for name, mfma in (("mfma", True), ("valu", False)):
        ev._SIL_MFMA = mfma
        ms = []
        for _ in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            v = ev._silhouette_kernel(x, idx, k)
            torch.cuda.synchronize()
            ms.append(round((time.perf_counter() - t) * 1e3, 2))
        out[name] = {"ms": ms, "best_ms": min(ms), "value": v}
    out["value_rel_diff"] = abs(out["mfma"]["value"] - out["valu"]["value"]) / \
        abs(out["valu"]["value"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
