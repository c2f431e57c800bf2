"""The RCCL code paths on one GPU: ALS, k-means and RDF trained with every collective issued
(``ORYX_FORCE_COLLECTIVES=1``: a world of one on the ``nccl`` backend) give the same results as
the collective-free single-process run.

At world size one every all-reduce / all-gather / all-to-all is an identity, so the results
must agree bit for bit (k-means centers to fp32 rounding: its k-means++ draws use a device
scan whose last bits vary run to run); a difference means a collective path reorders, drops
or re-lays-out data.  The ALS run with an explicit 3-range factor exchange checks the chunk-major gathered
layout and its remapped column ids; its padded shard changes the Gramian's fp32 summation
order, so it is compared in the fp32 factor mode to a 1e-4 bound instead of bit for bit.  Runs in a child process, because the process
group is process-global.
"""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys, json
import numpy as np, torch
sys.path.insert(0, ROOT)
from oryx_amd.parallel import dist
from oryx_amd.models.als.trainer import ALSTrainer
from oryx_amd.ops import kmeans as km, rdf as rdf_ops

dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")


def als(ctx, chunks=None, precision="bf16"):
    g = torch.Generator().manual_seed(5)
    key = torch.unique(torch.randint(0, 3000 * 800, (60000,), generator=g))
    u, i = key // 800, key % 800
    r = torch.randint(1, 6, (key.numel(),), generator=g).float()
    tr = ALSTrainer(24, lam=0.05, alpha=1.0, implicit=True, ctx=ctx, seed=3,
                    gather_chunks=chunks, precision=precision)
    tr.prepare(u, i, r, 3000, 800)
    tr.init_factors()
    tr.iterate(3)
    f = tr.factors()
    return f.X.cpu(), f.Y.cpu(), tr.lay_i.C


def kmeans(ctx):
    g = np.random.default_rng(0)
    cents = g.normal(0, 8, (12, 16))
    pts = np.concatenate([g.normal(c, 1.0, (2000, 16)) for c in cents])
    res = km.kmeans_train(torch.from_numpy(pts).float().to(dev), 12, 15, runs=1, seed=4,
                          ctx=ctx)
    return res.centers.cpu(), res.counts.cpu()


def rdf(ctx):
    g = np.random.default_rng(6)
    X = g.uniform(-1, 1, (30000, 5))
    y = ((X[:, 0] + 0.5 * X[:, 1] * X[:, 2] + 0.1 * g.standard_normal(30000)) > 0).astype(np.int64)
    data = rdf_ops.bin_features(X, [False] * 5, [0] * 5, 32, dev, seed=2)
    f = rdf_ops.train_forest(data, torch.from_numpy(y), 2, 4, 6, "gini", seed=3, ctx=ctx)

    def walk(nd):
        yield (nd.id, nd.feature, nd.bin, nd.count)
        if nd.feature >= 0:
            yield from walk(nd.left)
            yield from walk(nd.right)
    return [list(walk(r)) for r in f.roots], f.predictor_counts.tolist()


plain = dist.DistContext(device=dev)
ref = {"als": als(plain), "als3": als(plain, precision="fp32"), "km": kmeans(plain),
       "rdf": rdf(plain)}
os.environ["ORYX_FORCE_COLLECTIVES"] = "1"
ctx = dist.init_from_env()
assert ctx.forced and ctx.is_distributed, ctx
got = {"als": als(ctx), "als3": als(ctx, chunks=3, precision="fp32"), "km": kmeans(ctx), "rdf": rdf(ctx)}
out = {"backend": torch.distributed.get_backend(), "chunks3": got["als3"][2]}
for name, a, b in (("als", ref["als"], got["als"]), ("als3", ref["als3"], got["als3"])):
    out[name] = [float((x - y).abs().max()) for x, y in zip(a[:2], b[:2])]
out["km"] = [float((x.double() - y.double()).abs().max()) for x, y in zip(ref["km"], got["km"])]
out["rdf"] = ref["rdf"] == got["rdf"]
print("RESULT " + json.dumps(out))
""".replace("ROOT", repr(ROOT))


@pytest.mark.gpu
def test_forced_nccl_collectives_match_single_process(tmp_path):
    script = tmp_path / "forced.py"
    script.write_text(SCRIPT)
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT",
                        "ORYX_FORCE_COLLECTIVES")}
    env["MASTER_ADDR"] = "127.0.0.1"
    p = subprocess.run([sys.executable, "-u", str(script)], env=env, capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    import json
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["backend"] == "nccl", res
    assert res["chunks3"] == 3
    assert res["als"] == [0.0, 0.0], res
    assert max(res["als3"]) <= 1e-4, res
    # k-means++ draws over a device fp64 cumsum (a decoupled look-back scan: its last bits can
    # differ run to run), so centers are compared to fp32 rounding, counts exactly
    assert res["km"][0] <= 1e-5 and res["km"][1] == 0.0, res
    assert res["rdf"] is True, res
