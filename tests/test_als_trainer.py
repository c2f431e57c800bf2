import os
import subprocess
import sys

import pytest
import torch

from oryx_amd.models.als.trainer import ALSTrainer
from oryx_amd.parallel import dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data(seed=0, n_u=60, n_i=40, nnz=900):
    g = torch.Generator().manual_seed(seed)
    key = torch.unique(torch.randint(0, n_u * n_i, (nnz,), generator=g))
    return key // n_i, key % n_i, (torch.randint(1, 6, (key.numel(),), generator=g).float())


def test_trainer_converges_cpu():
    u, i, r = _data()
    tr = ALSTrainer(6, lam=0.01, alpha=1.0, implicit=False, ctx=dist.DistContext(), seed=1)
    tr.prepare(u, i, r, 60, 40)
    tr.init_factors()
    f0 = tr.factors()
    tr.iterate(10)
    f = tr.factors()
    pred = (f.X[u] * f.Y[i]).sum(1)
    pred0 = (f0.X[u] * f0.Y[i]).sum(1)
    rmse = ((pred - r) ** 2).mean().sqrt().item()
    rmse0 = ((pred0 - r) ** 2).mean().sqrt().item()
    assert rmse < 0.5 * rmse0 and rmse < 1.0


def test_trainer_implicit_ranks_known_items_higher():
    u, i, r = _data(seed=2)
    tr = ALSTrainer(8, lam=0.01, alpha=2.0, implicit=True, ctx=dist.DistContext(), seed=1)
    tr.prepare(u, i, r, 60, 40)
    f = tr.train(8)
    scores = f.X @ f.Y.t()
    known = torch.zeros(60, 40, dtype=torch.bool)
    known[u, i] = True
    assert scores[known].mean() > scores[~known].mean() + 0.2


def test_distributed_matches_single_process_gloo(tmp_path):
    """world_size 2 over gloo (all-to-all shuffle, all-reduce YtY, all-gather) == world 1."""
    script = tmp_path / "run.py"
    script.write_text(f"""
import sys, torch
sys.path.insert(0, {ROOT!r})
from oryx_amd.parallel import dist
from oryx_amd.models.als.trainer import ALSTrainer
ctx = dist.init_from_env(device='cpu')
g = torch.Generator().manual_seed(5)
key = torch.unique(torch.randint(0, 64 * 50, (1500,), generator=g))
u, i = key // 50, key % 50
r = torch.randint(1, 6, (key.numel(),), generator=g).float()
# every rank holds a different slice of the data
sl = slice(ctx.rank, None, ctx.world_size)
tr = ALSTrainer(5, lam=0.05, alpha=1.0, implicit=True, ctx=ctx, seed=3)
tr.prepare(u[sl], i[sl], r[sl], 64, 50)
# deterministic identical init regardless of world size
gi = torch.Generator().manual_seed(11)
X0 = torch.randn(64, 5, generator=gi); Y0 = torch.randn(50, 5, generator=gi)
tr.init_factors(X0, Y0)
tr.iterate(3)
f = tr.factors()
if ctx.rank == 0:
    torch.save({{'X': f.X, 'Y': f.Y}}, sys.argv[1])
""")
    outs = []
    for world in (1, 2):
        out = tmp_path / f"w{world}.pt"
        env = dict(os.environ, OMP_NUM_THREADS="1")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
               f"--master-port={29600 + world}", str(script), str(out)]
        subprocess.run(cmd, check=True, env=env, timeout=180, capture_output=True)
        outs.append(torch.load(out))
    assert torch.allclose(outs[0]["X"], outs[1]["X"], atol=1e-4)
    assert torch.allclose(outs[0]["Y"], outs[1]["Y"], atol=1e-4)


@pytest.mark.gpu
def test_trainer_gpu_matches_cpu_reference(cuda):
    u, i, r = _data(seed=4, n_u=300, n_i=200, nnz=8000)
    res = {}
    for dev in ("cpu", cuda):
        tr = ALSTrainer(16, lam=0.05, alpha=1.0, implicit=True,
                        ctx=dist.DistContext(device=torch.device(dev)), seed=1)
        tr.prepare(u, i, r, 300, 200)
        gi = torch.Generator().manual_seed(11)
        tr.init_factors(torch.randn(300, 16, generator=gi) * 0.3,
                        torch.randn(200, 16, generator=gi) * 0.3)
        tr.iterate(1)
        res[str(dev)] = tr.factors()
    a, b = res["cpu"], res[str(cuda)]
    scale = a.X.abs().max().item()
    assert (a.X - b.X.cpu()).abs().max().item() < 5e-2 * max(1, scale)
