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
    """world_size 2 over gloo (all-to-all shuffle, all-reduce YtY, all-gather; also with the
    factor exchange split into 3 asynchronous ranges; round-robin row ownership) == world 1."""
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
# fp32 factor mode: with bf16 replicated factors a 1-ulp difference in the all-reduced YtY
# (a different summation order per world size) can flip a bf16 rounding and grow to ~1e-4
tr = ALSTrainer(5, lam=0.05, alpha=1.0, implicit=True, ctx=ctx, seed=3,
                gather_chunks=int(sys.argv[2]), precision="fp32")
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
    for world, chunks in ((1, 1), (2, 1), (2, 3)):
        out = tmp_path / f"w{world}c{chunks}.pt"
        env = dict(os.environ, OMP_NUM_THREADS="1")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
               f"--master-port={29600 + world + 10 * chunks}", str(script), str(out),
               str(chunks)]
        subprocess.run(cmd, check=True, env=env, timeout=180, capture_output=True)
        outs.append(torch.load(out))
    for o in outs[1:]:
        assert torch.allclose(outs[0]["X"], o["X"], atol=1e-4)
        assert torch.allclose(outs[0]["Y"], o["Y"], atol=1e-4)


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


def test_row_layout_is_a_bijection():
    from oryx_amd.models.als.trainer import RowLayout
    for n, W, C in ((10, 1, 1), (10, 1, 3), (1000, 8, 4), (7, 2, 5), (1, 4, 4)):
        lay = RowLayout(n, W, C)
        ids = torch.arange(W * lay.s)
        g = lay.remap(ids)
        assert g.unique().numel() == ids.numel() and int(g.max()) < lay.rows
        if C == 1 and W == 1:
            assert torch.equal(g, ids)
        # range c of rank r is one contiguous block of the gathered layout
        r, loc = ids // lay.s, ids % lay.s
        c = loc // lay.cr
        assert torch.equal(g // lay.cr, c * W + r)


@pytest.mark.parametrize("chunks", [2, 3])
def test_chunked_gather_matches_single_range_cpu(chunks):
    u, i, r = _data(seed=6)
    res = []
    for c in (1, chunks):
        tr = ALSTrainer(6, lam=0.05, alpha=1.0, implicit=True, ctx=dist.DistContext(), seed=2,
                        gather_chunks=c)
        tr.prepare(u, i, r, 60, 40)
        gi = torch.Generator().manual_seed(3)
        tr.init_factors(torch.randn(60, 6, generator=gi), torch.randn(40, 6, generator=gi))
        tr.iterate(2)
        res.append(tr.factors())
    assert torch.allclose(res[0].X, res[1].X, atol=1e-5)
    assert torch.allclose(res[0].Y, res[1].Y, atol=1e-5)


@pytest.mark.gpu
def test_chunked_gather_gpu(cuda):
    u, i, r = _data(seed=7, n_u=3000, n_i=900, nnz=60000)
    res = []
    for c in (1, 3):
        tr = ALSTrainer(32, lam=0.05, alpha=1.0, implicit=True,
                        ctx=dist.DistContext(device=cuda), seed=2, gather_chunks=c)
        tr.prepare(u, i, r, 3000, 900)
        gi = torch.Generator().manual_seed(3)
        tr.init_factors(torch.randn(3000, 32, generator=gi) * 0.3,
                        torch.randn(900, 32, generator=gi) * 0.3)
        tr.iterate(2)
        res.append(tr.factors())
    assert torch.allclose(res[0].X, res[1].X, atol=1e-4)
    assert torch.allclose(res[0].Y, res[1].Y, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [16, 100])
def test_trainer_gpu_fp32_factors_match_cpu(cuda, k):
    """fp32 factor precision (bf16 hi|lo SPLIT kernels) tracks the CPU fp32 trainer closely
    after two iterations (the bf16 mode's tolerance is 50x looser)."""
    u, i, r = _data(seed=5, n_u=400, n_i=250, nnz=12000)
    res = {}
    for dev in ("cpu", cuda):
        tr = ALSTrainer(k, lam=0.05, alpha=1.0, implicit=True,
                        ctx=dist.DistContext(device=torch.device(dev)), seed=1,
                        precision="fp32")
        tr.prepare(u, i, r, 400, 250)
        gi = torch.Generator().manual_seed(11)
        tr.init_factors(torch.randn(400, k, generator=gi) * 0.3,
                        torch.randn(250, k, generator=gi) * 0.3)
        tr.iterate(2)
        res[str(dev)] = tr.factors()
    a, b = res["cpu"], res[str(cuda)]
    for m in ("X", "Y"):
        ref, got = getattr(a, m).double(), getattr(b, m).cpu().double()
        rel = (got - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-12)
        assert rel.max().item() < 1e-3, (m, rel.max().item())


def test_trainer_fp32_precision_cpu():
    u, i, r = _data(seed=8)
    out = []
    for prec in ("bf16", "fp32"):
        tr = ALSTrainer(6, lam=0.05, alpha=1.0, implicit=True, ctx=dist.DistContext(), seed=2,
                        precision=prec)
        tr.prepare(u, i, r, 60, 40)
        gi = torch.Generator().manual_seed(3)
        tr.init_factors(torch.randn(60, 6, generator=gi), torch.randn(40, 6, generator=gi))
        tr.iterate(2)
        out.append(tr.factors())
        assert tr.Xb_local.shape[1] == (2 if prec == "fp32" else 1) * tr.kp
    # the CPU path solves from the operand copy: fp32 mode from ~fp32 factors
    assert not torch.equal(out[0].X, out[1].X)


def _planted_implicit(seed=21, n_u=1500, n_i=600, rank=8):
    """Implicit feedback planted from a rank-8 model: each user's positives are the top 5-40
    items of U V^T + noise; 10% of every user's positives are held out."""
    g = torch.Generator().manual_seed(seed)
    U = torch.randn(n_u, rank, generator=g)
    V = torch.randn(n_i, rank, generator=g)
    S = U @ V.t() + 0.5 * torch.randn(n_u, n_i, generator=g)
    m = torch.randint(5, 41, (n_u,), generator=g)
    top = S.argsort(dim=1, descending=True)
    tr_u, tr_i, tr_r, te_u, te_i = [], [], [], [], []
    for a in range(n_u):
        items = top[a, :int(m[a])]
        hold = torch.rand(len(items), generator=g) < 0.1
        tr_u.append(torch.full((int((~hold).sum()),), a))
        tr_i.append(items[~hold])
        tr_r.append(torch.randint(1, 6, (int((~hold).sum()),), generator=g).float())
        te_u.append(torch.full((int(hold.sum()),), a))
        te_i.append(items[hold])
    cat = torch.cat
    return cat(tr_u), cat(tr_i), cat(tr_r), cat(te_u).numpy(), cat(te_i).numpy(), n_u, n_i


@pytest.mark.gpu
def test_auc_drift_bf16_vs_fp32(cuda):
    """End-metric drift of the factor precisions: held-out AUC (the reference's implicit
    evaluation, Evaluation.java:70-136) of the GPU bf16 and fp32 modes vs the CPU fp32 trainer
    from the same initial factors."""
    import json
    from oryx_amd.models.als.evaluation import area_under_curve
    u, i, r, te_u, te_i, n_u, n_i = _planted_implicit()
    k = 32
    auc = {}
    for name, dev, prec in (("cpu_fp32", "cpu", "fp32"), ("gpu_fp32", cuda, "fp32"),
                            ("gpu_bf16", cuda, "bf16")):
        tr = ALSTrainer(k, lam=0.01, alpha=1.0, implicit=True,
                        ctx=dist.DistContext(device=torch.device(dev)), seed=1, precision=prec)
        tr.prepare(u, i, r, n_u, n_i)
        gi = torch.Generator().manual_seed(11)
        tr.init_factors(torch.randn(n_u, k, generator=gi) * 0.1,
                        torch.randn(n_i, k, generator=gi) * 0.1)
        tr.iterate(10)
        f = tr.factors()
        auc[name] = area_under_curve(f.X.cpu(), f.Y.cpu(), te_u, te_i, seed=7)
    print(json.dumps({"als_auc_drift": auc, "k": k, "iterations": 10}))
    assert auc["cpu_fp32"] > 0.8, auc                    # the planted structure is learned
    assert abs(auc["gpu_fp32"] - auc["cpu_fp32"]) < 2e-3, auc
    assert abs(auc["gpu_bf16"] - auc["cpu_fp32"]) < 1e-2, auc


@pytest.mark.gpu
@pytest.mark.parametrize("k,precision,chunks", [(64, "bf16", 1), (128, "fp32", 1),
                                                (32, "bf16", 3)])
def test_graph_replay_matches_eager_gpu(cuda, k, precision, chunks):
    """One process, ORYX_ALS_GRAPH=1: iterations after the first are one captured HIP graph
    replayed (ALSTrainer._replay) -- bitwise the eager launches' factors, over several replays and
    after re-publishing the factors (which drops the captured graph)."""
    u, i, r = _data(seed=9, n_u=4000, n_i=1500, nnz=90000)
    out = []
    for graphs in (False, True):
        tr = ALSTrainer(k, lam=0.05, alpha=1.0, implicit=True,
                        ctx=dist.DistContext(device=cuda), seed=2, precision=precision,
                        gather_chunks=chunks)
        tr._GRAPHS = graphs
        tr.prepare(u, i, r, 4000, 1500)
        gi = torch.Generator().manual_seed(3)
        tr.init_factors(torch.randn(4000, k, generator=gi) * 0.3,
                        torch.randn(1500, k, generator=gi) * 0.3)
        tr.iterate(4)
        assert (tr._graph is not None) == graphs
        f1 = tr.factors()
        tr.init_factors(f1.X.cpu(), f1.Y.cpu())     # new buffers: the graph is dropped
        assert tr._graph is None
        tr.iterate(3)
        torch.cuda.synchronize()
        out.append((f1, tr.factors(), tr.failures))
    (a1, a2, fa), (b1, b2, fb) = out
    assert fa == fb == 0
    for x, y in ((a1, b1), (a2, b2)):
        assert torch.equal(x.X, y.X) and torch.equal(x.Y, y.Y)
