"""One-shot peer-mapped all-reduce (csrc/kernels/ipc_allreduce.hip, parallel/ipc.py).

The GPU test runs two ranks as two processes on the one GPU of the test box: each allocates
its exchange buffer, the IPC handles travel over gloo, each maps the other's buffer and the
sums are checked exactly (integer-valued probes) over many calls and sizes -- the slot
alternation, the flags and the rank-ordered sum are the same code the node's 8 GPUs run.
The CPU test checks the dispatch rules of dist.all_reduce_sum."""

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
    import torch.distributed as tdist
    from oryx_amd.parallel import ipc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = dist.DistContext(rank, world, 0, dev, backend="gloo")
    red = ipc.IpcAllReduce(ctx, cap_bytes=1 << 20)
    bad = 0
    calls = 0
    for rep in range(3):
        for n in (1, 3, 255, 256, 4097, 65536, (1 << 18) - 5):
            base = torch.arange(n, dtype=torch.float32, device=dev)
            t = base * (rank + 1) + rep
            red.all_reduce_(t)
            calls += 1
            # sum over r of (base (r + 1) + rep)
            want = base * sum(r + 1 for r in range(world)) + rep * world
            bad += int(not torch.equal(t, want))
    torch.cuda.synchronize()
    red.check()
    # latency of a 64 KB (rank-128 Gramian) all-reduce, stream-ordered back to back
    g = torch.ones(128 * 128, dtype=torch.float32, device=dev)
    for _ in range(5):
        red.all_reduce_(g)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(50):
        red.all_reduce_(g)
    ev1.record()
    ev1.synchronize()
    red.check()
    us = ev0.elapsed_time(ev1) * 1e3 / 50
    tdist.barrier()
    red.close()
    with open("%s.%d" % (out_path, rank), "w") as f:
        f.write("%d %d %.2f\n" % (bad, calls, us))
    tdist.destroy_process_group()


@pytest.mark.gpu
def test_ipc_allreduce_two_processes_one_gpu(tmp_path):
    import torch.multiprocessing as mp
    from oryx_amd import native
    native.require_kernels()
    out = str(tmp_path / "res")
    port = _port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for r in range(2):
        bad, calls, us = open("%s.%d" % (out, r)).read().split()
        assert int(bad) == 0 and int(calls) == 21
        print("rank %d: 64 KB one-shot all-reduce %.1f us" % (r, float(us)))


def test_all_reduce_sum_dispatch_cpu():
    class FakeIpc:
        calls = 0

        def fits(self, t):
            return t.numel() <= 4

        def all_reduce_(self, t):
            self.calls += 1
            return t.mul_(2)

    ctx = dist.DistContext(0, 1, 0, torch.device("cpu"))
    ctx.forced = True
    ctx.ipc = FakeIpc()
    t = torch.ones(3)
    dist.all_reduce_sum(t, ctx)
    assert ctx.ipc.calls == 1 and torch.equal(t, torch.full((3,), 2.0))
    # a world of one that is not forced issues nothing
    ctx2 = dist.DistContext(0, 1, 0, torch.device("cpu"))
    ctx2.ipc = FakeIpc()
    dist.all_reduce_sum(t, ctx2)
    assert ctx2.ipc.calls == 0
