"""Peer-push all-gather of the replicated factor matrices (csrc/kernels/ipc_allgather.hip,
parallel/ipc.py IpcAllGather, models/als/trainer.py RowLayout.gather).

The GPU test runs two ranks as two processes on the one GPU of the test box: each maps the
other's matrices and flag buffer with hipIpc handles (gloo carries them), and the gathered
matrices are compared BITWISE with gloo's staged all-gather of the same ranges, over many
exchanges of two matrices of different shapes (the epoch flags, the READY / DONE ordering and
the chunk-major layout are the code an 8-GPU node runs).  It also times one exchange both
ways.  The CPU test checks RowLayout.gather's dispatch to a gatherer (ranges, offsets, order).
"""

import os
import socket

import pytest
import torch

from oryx_amd.parallel import dist


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import time
    import torch.distributed as tdist
    from oryx_amd.models.als.trainer import RowLayout
    from oryx_amd.parallel import ipc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = dist.DistContext(rank, world, 0, dev, backend="gloo")
    ag = ipc.IpcAllGather(ctx)
    ok = ag.self_test()
    ctx.ipc_gather = ag
    bad = 0
    shapes = {"Y": RowLayout(70001, world, 4), "X": RowLayout(33333, world, 3)}
    cols = {"Y": 64, "X": 256}
    for rep in range(6):
        for name, lay in shapes.items():
            g = torch.Generator(device=dev).manual_seed(1000 * rep + 17 * rank + len(name))
            local = torch.randn((lay.local_rows, cols[name]), device=dev, generator=g) \
                .to(torch.bfloat16)
            solved = []
            got = lay.gather(local, ctx, overlap_with=solved.append, name=name)
            ctx_g = dist.DistContext(rank, world, 0, dev, backend="gloo")
            want = lay.gather(local, ctx_g)         # gloo, staged through the host
            torch.cuda.synchronize()
            bad += int(not torch.equal(got.view(torch.int16), want.view(torch.int16)))
            bad += int(solved != list(range(lay.C)))
    ag.check()
    # one 70001 x 256 bf16 exchange (4 ranges), push vs gloo
    lay = RowLayout(70001, world, 4)
    local = torch.ones((lay.local_rows, 256), device=dev, dtype=torch.bfloat16)
    ms = {}
    for how in ("push", "gloo"):
        c = ctx if how == "push" else dist.DistContext(rank, world, 0, dev, backend="gloo")
        for _ in range(2):
            lay.gather(local, c, name="Z" if how == "push" else None)
        torch.cuda.synchronize()
        tdist.barrier()
        t0 = time.perf_counter()
        for _ in range(5):
            lay.gather(local, c, name="Z" if how == "push" else None)
        torch.cuda.synchronize()
        ms[how] = (time.perf_counter() - t0) * 1e3 / 5
    ag.check()
    tdist.barrier()
    ag.close()
    with open("%s.%d" % (out_path, rank), "w") as f:
        f.write("%d %d %.3f %.3f\n" % (int(ok), bad, ms["push"], ms["gloo"]))
    tdist.destroy_process_group()


@pytest.mark.gpu
def test_ipc_allgather_two_processes_one_gpu_bitwise(tmp_path):
    import torch.multiprocessing as mp
    from oryx_amd import native
    native.require_kernels()
    out = str(tmp_path / "res")
    port = _port()
    mctx = mp.get_context("spawn")
    procs = [mctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=110)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for r in range(2):
        ok, bad, push_ms, gloo_ms = open("%s.%d" % (out, r)).read().split()
        assert int(ok) == 1 and int(bad) == 0
        print("rank %d: 70001 x 256 bf16 exchange: push %.2f ms, gloo %.2f ms"
              % (r, float(push_ms), float(gloo_ms)))


class _FakeGather:
    def __init__(self):
        self.calls = []
        self.bufs = {}

    def buffer(self, name, shape, dtype):
        if name not in self.bufs:
            self.bufs[name] = torch.zeros(shape, dtype=dtype)
        return self.bufs[name]

    def begin(self, name):
        self.calls.append(("begin", name))

    def push(self, name, src, row0, chunks, c):
        self.calls.append(("push", name, int(row0), chunks, c, src.shape[0]))
        self.bufs[name][row0:row0 + src.shape[0]] = src

    def end(self, name, chunks):
        self.calls.append(("end", name, chunks))


def test_row_layout_gather_dispatches_to_gatherer_cpu():
    from oryx_amd.models.als.trainer import RowLayout
    ctx = dist.DistContext(1, 3, 0, torch.device("cpu"))
    ctx.ipc_gather = _FakeGather()
    lay = RowLayout(100, 3, 4)
    local = torch.arange(lay.local_rows * 2, dtype=torch.float32).reshape(-1, 2)
    order = []
    out = lay.gather(local, ctx, overlap_with=lambda c: order.append(("solve", c)), name="Y")
    assert out is ctx.ipc_gather.bufs["Y"] and out.shape == (lay.rows, 2)
    pushes = [c for c in ctx.ipc_gather.calls if c[0] == "push"]
    assert ctx.ipc_gather.calls[0] == ("begin", "Y")
    assert ctx.ipc_gather.calls[-1] == ("end", "Y", lay.C)
    # range c of rank 1 lands at chunk-major row (c * W + 1) * cr
    assert [p[2] for p in pushes] == [(c * 3 + 1) * lay.cr for c in range(lay.C)]
    assert order == [("solve", c) for c in range(lay.C)]
    for c in range(lay.C):
        r0 = (c * 3 + 1) * lay.cr
        assert torch.equal(out[r0:r0 + lay.cr], local[c * lay.cr:(c + 1) * lay.cr])
    ctx.backend = "nccl"
    assert dist.allgather_kind(ctx).startswith("ipc-push")
    ctx.ipc_gather = None
    assert dist.allgather_kind(ctx) == "rccl"
