"""Host-side (Python) profile of one RDF forest at the bench shape: where the wall time
between GPU kernels goes.  Prints the wall time and the top functions by cumulative time."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oryx_amd.ops import rdf as rdf_ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n, P = int(os.environ.get("N", 6_250_000)), 100
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    X = torch.randn((n, P), generator=g, device=dev)
    y = (X[:, 0] - 0.8 * X[:, 1] > 0).to(torch.int32)
    data = rdf_ops.bin_features(X, [False] * P, [0] * P, 100, dev, seed=1,
                                threshold_source=X[:200_000])
    del X
    rdf_ops.train_forest(data, y, 2, 20, 8, "entropy", seed=1)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    rdf_ops.train_forest(data, y, 2, 20, 8, "entropy", seed=2)
    torch.cuda.synchronize()
    pr.disable()
    print("forest ms %.1f" % ((time.perf_counter() - t0) * 1e3))
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
