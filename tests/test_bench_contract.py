"""The driver's bench.py contract on CPU (gloo): one JSON line from rank 0 with the metric and
config BASELINE.json names, the whole-job value, and world size 2 through
torch.distributed.run on 127.0.0.1."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--ratings-per-gpu", "20000", "--users-per-gpu", "500", "--items",
         "300", "--rank-k", "16", "--steps", "1", "--warmup", "1", "--speed-events", "100"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _check(rec, n):
    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert rec["metric"] == baseline["metric"]
    for key in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in rec, key
    assert rec["n_gpus"] == n and rec["steps"] == 1 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak"
    # whole-job aggregate: ratings of all ranks over the timed step
    assert abs(rec["value"] - rec["config"]["global_batch"] / (rec["ms_per_step"] * 1e-3)) \
        <= 1e-6 * rec["value"]
    assert rec["config"]["global_batch"] == 20000 * n
    assert rec["world_size"] == n and len(rec["rank_devices"]) == n


@pytest.mark.timeout(600)
def test_bench_single_process_cpu():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL,
                         capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    recs = _json_lines(out.stdout)
    assert len(recs) == 1
    _check(recs[0], 1)


@pytest.mark.timeout(600)
def test_bench_two_ranks_gloo():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    recs = _json_lines(out.stdout)
    assert len(recs) == 1                       # rank 0 only
    _check(recs[0], 2)


@pytest.mark.timeout(600)
def test_bench_self_launches_ranks():
    """``python bench.py --gpus 2`` with no external launcher starts 2 ranks itself."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL,
                         capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    recs = _json_lines(out.stdout)
    assert len(recs) == 1
    _check(recs[0], 2)
    assert recs[0]["backend"] == "gloo"


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL,
                         capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 2
    assert "WORLD_SIZE" in out.stderr


@pytest.mark.timeout(600)
def test_bench_forced_collectives_world_one():
    """World of one with ORYX_FORCE_COLLECTIVES=1 runs every collective code path."""
    env = dict(os.environ, ORYX_FORCE_COLLECTIVES="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL,
                         capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = _json_lines(out.stdout)[0]
    _check(rec, 1)
    assert rec["backend"] == "gloo"


def test_bench_lambda_loop_cpu():
    """bench_lambda.py: POST /ingest -> speed UP -> applied in the serving model, end to end
    (tiny model, CPU): every trial's update is published to the update log and applied,
    none lost (no-op fold-ins are counted apart, not as losses)."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench_lambda.py"), "--items", "3000",
                        "--users", "500", "--features", "8", "--trials", "4", "--device", "cpu"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["lost_or_timeouts"] == 0
    assert rec["trials"] + rec["noop_foldins"] >= 4 and rec["trials"] > 0
    assert rec["p50_ms"] > 0 and rec["ingest_to_up_in_log_p50_ms"] <= rec["p90_ms"]


def test_bench_batch_sharded_gloo_world_two():
    """bench_batch.py --gpus 2 on CPU (gloo): the sharded generation (each rank reads its
    share of the input partitions, route + aggregate + train + publish per rank) publishes
    a MODEL and every UP row, with per-phase timings."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench_batch.py"), "--gpus", "2",
                        "--device", "cpu", "--ratings", "60000", "--users", "2000", "--items",
                        "800", "--features", "6", "--iterations", "2"],
                       capture_output=True, text=True, timeout=400, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["sharded"] is True
    ph = rec["phase_s"]
    for key in ("parse", "dictionaries", "route", "aggregate", "train", "publish_up",
                "layer_drain", "layer_update", "layer_save_data"):
        assert key in ph, ph
    # every second of the generation is in some phase (within 10% + a little fixed cost)
    assert rec["unattributed_s"] <= 0.1 * rec["generation_s"] + 0.5, rec
    # MODEL + one UP row per user and item that has ratings
    assert rec["update_messages"] > 2000


def test_bench_batch_kmeans_and_rdf_cpu():
    """bench_batch.py --app kmeans / rdf (CPU, small): a generation from the input log to a
    published MODEL with parse / train / eval phases, every second attributed."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for app, extra in (("kmeans", ["--k", "6", "--iterations", "4"]),
                       ("rdf", ["--trees", "3", "--depth", "3"])):
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench_batch.py"), "--app", app,
                            "--device", "cpu", "--points", "6000", "--dims", "8"] + extra,
                           capture_output=True, text=True, timeout=400, env=env)
        assert p.returncode == 0, p.stderr[-3000:]
        rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
        assert rec["app"] == app and rec["update_messages"] >= 1
        for key in ("parse", "train", "eval", "pmml_write", "layer_update"):
            assert key in rec["phase_s"], rec["phase_s"]
        assert rec["unattributed_s"] <= 0.1 * rec["generation_s"] + 0.5, rec


def test_bench_emulate_world_cpu():
    """bench.py --emulate-world: one process builds rank r's share of a W-rank run (its user
    CSR holds the users id % W == r of every rank, its item CSR the items id % W == r) and
    reports per-iteration time and collective payloads."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--emulate-world", "4",
                        "--emulate-rank", "2", "--device", "cpu", "--rank-k", "8",
                        "--ratings-per-gpu", "8000", "--users-per-gpu", "1000", "--items",
                        "300", "--steps", "1", "--warmup", "1", "--precision", "fp32"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["emulated"] and rec["world"] == 4 and rec["rank"] == 2
    assert rec["rows"]["users"] == 1000 and rec["rows"]["items"] == 75
    # about a quarter of the world's ratings on each side
    assert 0.15 < rec["ratings_user_csr"] / rec["ratings_world"] < 0.35
    assert rec["collectives_per_iteration"]["allgather_recv_bytes"] == \
        3 * rec["collectives_per_iteration"]["allgather_send_bytes"]
    assert rec["solve_failures"] == 0
