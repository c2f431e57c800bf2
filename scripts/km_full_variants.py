"""A/B timing of the exact full-rescan kernel variants (km_rescore_full instantiations picked
by ORYX_KM_FULL_VARIANT): n_list points against K centers at d, checked against a torch fp32
argmin.  Usage: python scripts/km_full_variants.py [variant]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oryx_amd import native  # noqa: E402
from oryx_amd.ops.kmeans import DeviceCenters  # noqa: E402


def main():
    lib = native.require_kernels()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    n, npts, k, d = 1_000_000, 37_392, 1000, 256
    X = torch.randn((n, d), device=dev, generator=g)
    C = torch.randn((k, d), device=dev, generator=g)
    dc = DeviceCenters(C)
    rows = torch.randperm(n, device=dev, generator=g)[:npts].to(torch.int32)
    lst = torch.cat([torch.tensor([npts], dtype=torch.int32, device=dev), rows])
    assign = torch.full((n,), -1, dtype=torch.int32, device=dev)
    mind = torch.zeros(n, dtype=torch.float32, device=dev)
    st = native.stream_ptr(dev)

    def run():
        native.check(lib.oryx_kmeans_rescore_list(X.data_ptr(), X.stride(0), d,
                                                  dc.ct2.data_ptr(), k, lst.data_ptr(), npts,
                                                  assign.data_ptr(), mind.data_ptr(), st),
                     "rescore_list")
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    xr = X[rows.long()]
    ref = torch.cdist(xr, C).argmin(1)
    got = assign[rows.long()].long()
    agree = float((ref == got).float().mean())
    print(json.dumps({"variant": os.environ.get("ORYX_KM_FULL_VARIANT", "0"), "ms": ms,
                      "points": npts, "k": k, "d": d, "argmin_agree_vs_cdist": agree,
                      "gflops": 3.0 * npts * k * d / ms / 1e6}), flush=True)


if __name__ == "__main__":
    main()
