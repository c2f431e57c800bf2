"""Fault injection, the rank-health watchdog, ALS checkpoint/resume (including an elastic
restart of a 2-rank gloo group after a killed rank), log corruption detection and ALS warm
start (SURVEY.md sections 5.3 / 5.4)."""

import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest
import torch

from oryx_amd.models.als.trainer import ALSTrainer
from oryx_amd.parallel import dist, watchdog
from oryx_amd.transport import log as tlog
from oryx_amd.utils import faults

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _clean_faults():
    faults.disarm_all()
    yield
    faults.disarm_all()


def test_fault_specs_and_conditions():
    faults.arm("p:raise@iteration=3,count=2;q:corrupt")
    assert faults.point("p", iteration=1) is None
    with pytest.raises(faults.InjectedFault):
        faults.point("p", iteration=3)
    with pytest.raises(faults.InjectedFault):
        faults.point("p", iteration=3)
    assert faults.point("p", iteration=3) is None          # count exhausted
    assert faults.point("q", anything=1) == "corrupt"
    assert faults.point("q") is None
    faults.arm("r", "drop", count=0, rank=1)
    assert faults.point("r", rank=0) is None
    assert [faults.point("r", rank=1) for _ in range(3)] == ["drop"] * 3
    faults.arm("s", "raise", restart=1)
    assert faults.point("s") is None                        # not an elastic restart


def test_faults_from_environment(tmp_path):
    code = ("from oryx_amd.utils import faults\n"
            "try:\n    faults.point('x', k=2)\nexcept faults.InjectedFault:\n    print('hit')\n")
    env = dict(os.environ, ORYX_FAULTS="x:raise@k=2", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert "hit" in r.stdout
    env["ORYX_FAULTS"] = "x:exit@code=7"
    r = subprocess.run([sys.executable, "-c", code], env=env, timeout=120)
    assert r.returncode == 7


def test_watchdog_guard_and_heartbeat():
    fired = []
    wd = watchdog.Watchdog(1.0, on_expire=fired.append, poll_s=0.05)
    with wd.guard("fast"):
        pass
    time.sleep(1.3)
    assert not fired
    with wd.guard("stuck collective"):
        t0 = time.time()
        while not fired and time.time() - t0 < 10:
            time.sleep(0.05)
    assert fired and "stuck collective" in fired[0]
    fired2 = []
    wd2 = watchdog.Watchdog(1.0, on_expire=fired2.append, poll_s=0.05)
    for _ in range(8):
        wd2.heartbeat("loop")
        time.sleep(0.1)
    assert not fired2
    t0 = time.time()
    while not fired2 and time.time() - t0 < 10:
        time.sleep(0.05)
    assert fired2 and "loop" in fired2[0]
    off = watchdog.Watchdog(0)
    with off.guard("x"):
        pass
    assert not off.enabled


def _toy_ratings(seed=0, users=60, items=40, nnz=800):
    g = np.random.default_rng(seed)
    key = g.choice(users * items, nnz, replace=False)
    u, i = key // items, key % items
    s = g.integers(1, 6, nnz).astype(np.float32)
    return torch.from_numpy(u), torch.from_numpy(i), torch.from_numpy(s), users, items


def _trainer(data, seed=7):
    u, i, s, nu, ni = data
    t = ALSTrainer(6, 0.01, 1.0, True, ctx=dist.DistContext(), seed=seed)
    t.prepare(u, i, s, nu, ni)
    return t


def test_als_checkpoint_resume_matches_uninterrupted(tmp_path):
    data = _toy_ratings()
    ref = _trainer(data).train(6)
    ck = str(tmp_path / "ckpt")
    faults.arm("als.iteration", "raise", iteration=5)
    t = _trainer(data)
    with pytest.raises(faults.InjectedFault):
        t.train(6, checkpoint_dir=ck, checkpoint_interval=2, fingerprint="fp")
    meta = json.loads(open(os.path.join(ck, "latest.json")).read())
    assert meta["iteration"] == 4 and sorted(os.listdir(ck)) == ["it4", "latest.json"]
    # a different fingerprint (other data / settings) must not resume
    t_other = _trainer(data)
    assert t_other.load_checkpoint(ck, "other") == 0
    t2 = _trainer(data, seed=99)        # the seed only matters for a fresh start
    out = t2.train(6, checkpoint_dir=ck, checkpoint_interval=2, fingerprint="fp")
    assert t2.resumed_from == 4
    assert torch.equal(out.X, ref.X) and torch.equal(out.Y, ref.Y)
    assert not os.path.exists(ck)        # completed runs clean up


def test_als_warm_start_rows():
    data = _toy_ratings()
    ref = _trainer(data).train(4)
    t = _trainer(data)
    x0 = ref.X.clone()
    x0[3] = float("nan")                 # an ID the previous model did not know
    t.init_factors(x0, ref.Y)
    assert torch.equal(t.X[:60, :6][torch.arange(60) != 3], ref.X[torch.arange(60) != 3])
    assert not torch.isnan(t.X).any()


def test_als_update_warm_start_reads_previous_generation(tmp_path):
    from oryx_amd.models.als import batch as als_batch
    prev = tmp_path / "model" / "1000"
    als_batch.write_features(str(prev / "X"), ["u1", "u2"], np.ones((2, 3), np.float32))
    als_batch.write_features(str(prev / "Y"), ["i1"], np.full((1, 3), 2, np.float32))
    x, y = als_batch._warm_start_factors(str(tmp_path / "model"), 3, ["u2", "u9"], ["i1"])
    assert torch.equal(x[0], torch.ones(3)) and torch.isnan(x[1]).all()
    assert torch.equal(y[0], torch.full((3,), 2.0))
    assert als_batch._warm_start_factors(str(tmp_path / "model"), 4, ["u2"], ["i1"]) == \
        (None, None)


def test_log_corruption_is_detected_not_waited_on(tmp_path):
    t = tlog.Topic(str(tmp_path), "T", create_partitions=1)
    t.append(None, "first")
    faults.arm("log.append", "corrupt")
    t.append(None, "second")
    t.append(None, "third")
    c = tlog.TopicConsumer(t, "earliest")
    got = [m for _, _, _, _, m in c.poll(10, 200)]
    assert got == ["first"]
    with pytest.raises(tlog.LogCorruptionError):
        c.poll(10, 200)
    c.close()
    # the bulk frame poll (serving model loads) reports the same corruption after the good
    # frames, and a torn tail (no later frame) as nothing to read yet
    r = t.reader(0, 0)
    assert r.poll_frames(10, 1 << 16) == 1
    assert [v for _, _, _, v in r.decode_frames(0, 1)] == ["first"]
    with pytest.raises(tlog.LogCorruptionError):
        r.poll_frames(10, 1 << 16)
    r.close()
    # a dropped record never reaches the log
    t2 = tlog.Topic(str(tmp_path), "T2", create_partitions=1)
    faults.arm("log.append", "drop")
    t2.append(None, "lost")
    t2.append(None, "kept")
    assert t2.end_offset(0) == 1


ELASTIC = r"""
import json, os, sys
sys.path.insert(0, ROOT)
import numpy as np, torch
from oryx_amd.models.als.trainer import ALSTrainer
from oryx_amd.parallel import dist
out_dir = sys.argv[1]
ctx = dist.init_from_env(device="cpu")
g = np.random.default_rng(0)
key = g.choice(80 * 50, 1200, replace=False)
u, i = key // 50, key % 50
s = g.integers(1, 6, len(key)).astype(np.float32)
part = slice(ctx.rank, None, ctx.world_size)
t = ALSTrainer(5, 0.01, 1.0, True, ctx=ctx, seed=3)
t.prepare(torch.from_numpy(u[part]), torch.from_numpy(i[part]), torch.from_numpy(s[part]), 80, 50)
f = t.train(6, checkpoint_dir=os.path.join(out_dir, "ckpt"), checkpoint_interval=2,
            fingerprint="elastic")
if ctx.is_main:
    np.save(os.path.join(out_dir, "X.npy"), f.X.numpy())
    np.save(os.path.join(out_dir, "Y.npy"), f.Y.numpy())
    with open(os.path.join(out_dir, "resumed.json"), "w") as fh:
        json.dump({"resumed_from": t.resumed_from,
                   "restart": os.environ.get("TORCHELASTIC_RESTART_COUNT")}, fh)
"""


def _torchrun(script, out, port, extra_env=None):
    env = dict(os.environ, OMP_NUM_THREADS="1", **(extra_env or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--max-restarts=1", "--master-addr=127.0.0.1", "--master-port=%d" % port,
           str(script), str(out)]
    return subprocess.run(cmd, env=env, timeout=400, capture_output=True, text=True)


def test_elastic_restart_resumes_from_checkpoint(tmp_path):
    """Rank 1 is killed (os._exit) in iteration 3 of the first attempt; the elastic agent
    restarts the 2-rank gloo group, which resumes from the iteration-2 checkpoint and ends
    with exactly the factors of an uninterrupted run."""
    script = tmp_path / "run.py"
    script.write_text(ELASTIC.replace("ROOT", repr(ROOT)))
    clean, faulty = tmp_path / "clean", tmp_path / "faulty"
    clean.mkdir()
    faulty.mkdir()
    r = _torchrun(script, clean, 29661)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _torchrun(script, faulty, 29663,
                  {"ORYX_FAULTS": "als.iteration:exit@iteration=3,rank=1,restart=0"})
    assert r.returncode == 0, r.stderr[-3000:]
    info = json.loads((faulty / "resumed.json").read_text())
    assert info == {"resumed_from": 2, "restart": "1"}
    assert json.loads((clean / "resumed.json").read_text())["resumed_from"] == 0
    np.testing.assert_array_equal(np.load(faulty / "X.npy"), np.load(clean / "X.npy"))
    np.testing.assert_array_equal(np.load(faulty / "Y.npy"), np.load(clean / "Y.npy"))


def test_next_world_and_device_failure_classification():
    from oryx_amd.parallel import elastic
    assert elastic.next_world(7, 8) == 4
    assert elastic.next_world(3, 4) == 2
    assert elastic.next_world(1, 2) == 1
    assert elastic.next_world(0, 2) == 0
    assert elastic.next_world(5, 8, min_world=8) == 0
    assert elastic.is_device_failure(RuntimeError("HIP error: hipErrorLaunchFailure"))
    assert not elastic.is_device_failure(ValueError("bad input"))


SHRINK = r"""
import json, os, sys
sys.path.insert(0, ROOT)
import numpy as np, torch
from oryx_amd.models.als.trainer import ALSTrainer
from oryx_amd.parallel import dist
out_dir = sys.argv[1]
ctx = dist.init_from_env(device="cpu")
g = np.random.default_rng(0)
key = g.choice(80 * 50, 1200, replace=False)
u, i = key // 50, key % 50
s = g.integers(1, 6, len(key)).astype(np.float32)
part = slice(ctx.rank, None, ctx.world_size)
t = ALSTrainer(5, 0.01, 1.0, True, ctx=ctx, seed=3)
t.prepare(torch.from_numpy(u[part]), torch.from_numpy(i[part]), torch.from_numpy(s[part]), 80, 50)
f = t.train(6, checkpoint_dir=os.path.join(out_dir, "ckpt"), checkpoint_interval=2,
            fingerprint="shrink")
if ctx.is_main:
    np.save(os.path.join(out_dir, "X.npy"), f.X.numpy())
    np.save(os.path.join(out_dir, "Y.npy"), f.Y.numpy())
    with open(os.path.join(out_dir, "resumed.json"), "w") as fh:
        json.dump({"resumed_from": t.resumed_from, "world": ctx.world_size,
                   "attempt": os.environ.get("ORYX_ELASTIC_ATTEMPT")}, fh)
"""


def test_shrink_world_after_device_loss_resumes_from_checkpoint(tmp_path):
    """Rank 3 of a 4-rank gloo group loses its 'GPU' (device_lost fault) in iteration 3: the
    supervisor drops that device, relaunches the group on 2 ranks (the largest power of two
    below 4 that the 3 healthy devices allow), and the trainer resumes from the world-size
    independent iteration-2 checkpoint; the factors match an uninterrupted 4-rank run up to
    the summation order of the last iterations."""
    from oryx_amd.parallel import elastic
    script = tmp_path / "run.py"
    script.write_text(SHRINK.replace("ROOT", repr(ROOT)))
    runs = {}
    for name, faults_spec, port in (("clean", "", 29671),
                                    ("faulty", "als.iteration:device_lost@iteration=3,rank=3,"
                                               "attempt=0", 29673)):
        out = tmp_path / name
        out.mkdir()

        def build(world, out=out, port=port):
            return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    "--nproc-per-node=%d" % world, "--max-restarts=0",
                    "--master-addr=127.0.0.1", "--master-port=%d" % port, str(script),
                    str(out)]
        env = dict(os.environ, OMP_NUM_THREADS="1", ORYX_FAULTS=faults_spec)
        rc = elastic.supervise(build, 4, env=env)
        assert rc == 0, name
        runs[name] = out
    info = json.loads((runs["faulty"] / "resumed.json").read_text())
    assert info == {"resumed_from": 2, "world": 2, "attempt": "1"}
    # iterations 3-6 ran on 2 ranks instead of 4: same math, different fp32 summation order
    for m in ("X.npy", "Y.npy"):
        a, b = np.load(runs["faulty"] / m), np.load(runs["clean"] / m)
        assert np.linalg.norm(a - b) / np.linalg.norm(b) < 2e-3, m
        np.testing.assert_allclose(a, b, atol=5e-3)


def test_cli_relaunch_rewrites_gpus():
    from oryx_amd import cli
    assert cli._with_gpus(["batch", "--gpus", "8", "--conf", "x"], 4) == \
        ["batch", "--gpus", "4", "--conf", "x"]
    assert cli._with_gpus(["batch", "--gpus=8"], 2) == ["batch", "--gpus=2"]
