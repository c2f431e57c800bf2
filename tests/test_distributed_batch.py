"""Multi-rank batch layer (gloo, world 2): rank 0 drains the input log and announces the
generation; rank 1 follows (run_follower) and joins the trainer's collectives; exactly one
MODEL is published.  Covers the batch layer's distributed protocol and MLUpdate's follower
path with shared-seed candidate splits (the MI355X replacement of the Spark driver/executors)."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, os, sys
sys.path.insert(0, ROOT)
import numpy as np
from oryx_amd.layers.batch import BatchLayer
from oryx_amd.parallel import dist
from oryx_amd.transport.producer import LogTopicProducer
from oryx_amd.utils import config as cfg

tmp = sys.argv[1]
conf = cfg.overlay_on({
    "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.kmeans.KMeansUpdate",
    "oryx.input-topic.broker": "log:" + tmp + "/log",
    "oryx.update-topic.broker": "log:" + tmp + "/log",
    "oryx.batch.storage.data-dir": tmp + "/data",
    "oryx.batch.storage.model-dir": tmp + "/model",
    "oryx.input-schema.num-features": 2,
    "oryx.input-schema.categorical-features": "[]",
    "oryx.kmeans.hyperparams.k": 3,
    "oryx.kmeans.iterations": 10,
    "oryx.kmeans.evaluation-strategy": "SSE",
    "oryx.ml.eval.candidates": 2,
    "oryx.ml.eval.test-fraction": 0.1,
    "oryx.gpu.device": "cpu",
}, cfg.get_default())
ctx = dist.init_from_env(device="cpu")
layer = BatchLayer(conf)
if ctx.is_main:
    layer._context = layer.layer_context()
    layer._update = layer.load_update_instance()
    layer.build_input_consumer()
    g = np.random.default_rng(0)
    pts = np.concatenate([g.normal(c, 0.3, (200, 2)) for c in ([0, 0], [5, 5], [-5, 5])])
    prod = LogTopicProducer("log:" + tmp + "/log", "OryxInput", conf, async_=False)
    prod.send_many([(None, "%r,%r" % (float(a), float(b))) for a, b in pts])
    prod.close()
    layer.run_interval(1000)
    layer.close()
    out = {"rank": 0}
else:
    out = {"rank": 1, "joined": layer.run_follower()}
with open(os.path.join(tmp, "rank%d.json" % ctx.rank), "w") as f:
    json.dump(out, f)
"""


def test_two_rank_batch_generation(tmp_path):
    script = tmp_path / "run.py"
    script.write_text(SCRIPT.replace("ROOT", repr(ROOT)))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29641", str(script), str(tmp_path)]
    r = subprocess.run(cmd, env=env, timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    assert json.loads((tmp_path / "rank1.json").read_text())["joined"] == 1
    from oryx_amd.transport import log as tlog
    topic = tlog.Topic(str(tmp_path / "log"), "OryxUpdate")
    c = tlog.TopicConsumer(topic, "earliest")
    msgs = [(k, m) for _, _, _, k, m in c.poll(100, 100)]
    c.close()
    assert [k for k, _ in msgs] == ["MODEL"]
    from oryx_amd.models.kmeans.common import read_clusters
    from oryx_amd.utils import pmml as pm
    clusters = read_clusters(pm.from_string(msgs[0][1]))
    assert len(clusters) == 3 and sum(c.count for c in clusters) > 500
    # exactly one generation dir was published
    dirs = [d for d in os.listdir(tmp_path / "model") if not d.startswith(".")]
    assert len(dirs) == 1


ALS_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, ROOT)
import numpy as np
from oryx_amd.layers.batch import BatchLayer
from oryx_amd.parallel import dist
from oryx_amd.transport.producer import LogTopicProducer
from oryx_amd.utils import config as cfg

tmp = sys.argv[1]
conf = cfg.overlay_on({
    "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.als.ALSUpdate",
    "oryx.input-topic.broker": "log:" + tmp + "/log",
    "oryx.update-topic.broker": "log:" + tmp + "/log",
    "oryx.input-topic.partitions": 3,
    "oryx.batch.storage.data-dir": tmp + "/data",
    "oryx.batch.storage.model-dir": tmp + "/model",
    "oryx.als.hyperparams.features": 4,
    "oryx.als.iterations": 3,
    "oryx.als.implicit": "true",
    "oryx.ml.eval.candidates": 2,
    "oryx.ml.eval.test-fraction": 0.2,
    "oryx.gpu.device": "cpu",
}, cfg.get_default())
ctx = dist.init_from_env(device="cpu")
layer = BatchLayer(conf)
if ctx.is_main:
    layer._context = layer.layer_context()
    layer._update = layer.load_update_instance()
    layer.build_input_consumer()
    g = np.random.default_rng(1)
    for gen in range(2):
        lines = ["U%d,I%d,%d,%d" % (g.integers(0, 40), g.integers(0, 25), g.integers(1, 5),
                                    1000 * gen + j) for j in range(600)]
        prod = LogTopicProducer("log:" + tmp + "/log", "OryxInput", conf, async_=False)
        prod.send_many([(None, l) for l in lines])
        prod.close()
        with open(os.path.join(tmp, "input%d.txt" % gen), "w") as f:
            f.write("\n".join(lines) + "\n")
        layer.run_interval(1000 + gen)
    layer.close()
    out = {"rank": 0}
else:
    out = {"rank": 1, "joined": layer.run_follower()}
with open(os.path.join(tmp, "rank%d.json" % ctx.rank), "w") as f:
    json.dump(out, f)
"""


def test_two_rank_sharded_als_generations(tmp_path):
    """ALS on 2 gloo ranks with sharded generations: each rank reads its own share of the 3
    input partitions (the part files are disjoint and cover the input), the second generation
    reads past data per rank, one MODEL per generation, Y rows then X rows with known items
    from both ranks."""
    import json
    script = tmp_path / "run.py"
    script.write_text(ALS_SCRIPT.replace("ROOT", repr(ROOT)))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29643", str(script), str(tmp_path)]
    r = subprocess.run(cmd, env=env, timeout=600, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads((tmp_path / "rank1.json").read_text())["joined"] == 2
    for gen in range(2):
        d = tmp_path / "data" / ("oryx-%d.data" % (1000 + gen))
        parts = sorted(os.listdir(d))
        # keyless single-line input: plain-text part files
        assert parts == ["part-00000.txt", "part-00001.txt"]
        got = [open(d / p).read().split() for p in parts]
        assert got[0] and got[1]
        inp = open(tmp_path / ("input%d.txt" % gen)).read().split()
        assert sorted(got[0] + got[1]) == sorted(inp)
    from oryx_amd.transport import log as tlog
    topic = tlog.Topic(str(tmp_path / "log"), "OryxUpdate")
    c = tlog.TopicConsumer(topic, "earliest")
    msgs = []
    while True:
        batch = [(k, m) for _, _, _, k, m in c.poll(10000, 200)]
        if not batch:
            break
        msgs.extend(batch)
    c.close()
    keys = [k for k, _ in msgs]
    assert keys.count("MODEL") == 2
    # the second generation: every item and user of both generations, Y before X
    second = msgs[keys.index("MODEL", keys.index("MODEL") + 1) + 1:]
    ups = [json.loads(m) for k, m in second if k == "UP"]
    kinds = [u[0] for u in ups]
    assert kinds == sorted(kinds, key=lambda t: t != "Y")
    lines = open(tmp_path / "input0.txt").read().split() + \
        open(tmp_path / "input1.txt").read().split()
    users = {l.split(",")[0] for l in lines}
    items = {l.split(",")[1] for l in lines}
    assert {u[1] for u in ups if u[0] == "Y"} == items
    xs = {u[1]: set(u[3]) for u in ups if u[0] == "X"}
    assert set(xs) == users
    # known items = every (user, item) pair seen (no deletes in this data)
    want = {}
    for l in lines:
        a, b = l.split(",")[:2]
        want.setdefault(a, set()).add(b)
    assert xs == want


GROUP_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, ROOT)
import numpy as np
from oryx_amd.layers.batch import BatchLayer
from oryx_amd.parallel import dist
from oryx_amd.transport.producer import LogTopicProducer
from oryx_amd.utils import config as cfg

tmp, app = sys.argv[1], sys.argv[2]
base = {
    "oryx.input-topic.broker": "log:" + tmp + "/log",
    "oryx.update-topic.broker": "log:" + tmp + "/log",
    "oryx.input-topic.partitions": 4,
    "oryx.batch.storage.data-dir": tmp + "/data",
    "oryx.batch.storage.model-dir": tmp + "/model",
    "oryx.ml.eval.candidates": 2,
    "oryx.ml.eval.parallelism": 2,
    "oryx.gpu.device": "cpu",
}
if app == "als":
    base.update({"oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.als.ALSUpdate",
                 "oryx.als.hyperparams.features": "[3,5]", "oryx.als.iterations": 3,
                 "oryx.als.implicit": "true", "oryx.ml.eval.test-fraction": 0.2})
else:
    base.update({"oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.rdf.RDFUpdate",
                 "oryx.input-schema.num-features": 3,
                 "oryx.input-schema.categorical-features": "[]",
                 "oryx.input-schema.target-feature": "\"2\"",
                 "oryx.rdf.num-trees": 3, "oryx.rdf.hyperparams.max-depth": "[2,4]",
                 "oryx.ml.eval.test-fraction": 0.2})
conf = cfg.overlay_on(base, cfg.get_default())
ctx = dist.init_from_env(device="cpu")
layer = BatchLayer(conf)
if ctx.is_main:
    layer._context = layer.layer_context()
    layer._update = layer.load_update_instance()
    layer.build_input_consumer()
    g = np.random.default_rng(3)
    if app == "als":
        lines = ["U%d,I%d,%d,%d" % (g.integers(0, 60), g.integers(0, 30), g.integers(1, 5), j)
                 for j in range(1500)]
    else:
        x = g.normal(0, 1, (800, 2))
        lines = ["%r,%r,%r" % (float(a), float(b), float(3 * a - b)) for a, b in x]
    prod = LogTopicProducer("log:" + tmp + "/log", "OryxInput", conf, async_=False)
    prod.send_many([(None, l) for l in lines])
    prod.close()
    layer.run_interval(1000)
    layer.close()
    out = {"rank": 0}
else:
    out = {"rank": ctx.rank, "joined": layer.run_follower()}
with open(os.path.join(tmp, "rank%d.json" % ctx.rank), "w") as f:
    json.dump(out, f)
"""


def _run_grouped(tmp_path, app, nproc, port):
    import json
    script = tmp_path / "run.py"
    script.write_text(GROUP_SCRIPT.replace("ROOT", repr(ROOT)))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % nproc, "--master-addr=127.0.0.1",
           "--master-port=%d" % port, str(script), str(tmp_path), app]
    r = subprocess.run(cmd, env=env, timeout=600, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    for k in range(1, nproc):
        assert json.loads((tmp_path / ("rank%d.json" % k)).read_text())["joined"] == 1
    from oryx_amd.transport import log as tlog
    topic = tlog.Topic(str(tmp_path / "log"), "OryxUpdate")
    c = tlog.TopicConsumer(topic, "earliest")
    msgs = []
    while True:
        batch = [(k, m) for _, _, _, k, m in c.poll(10000, 200)]
        if not batch:
            break
        msgs.extend(batch)
    c.close()
    dirs = [d for d in os.listdir(tmp_path / "model") if not d.startswith(".")]
    assert len(dirs) == 1
    timing = json.loads((tmp_path / "model" / dirs[0] / "timings.json").read_text())
    return msgs, timing


def test_candidate_groups_sharded_als_four_ranks(tmp_path):
    """Candidate parallelism on disjoint process groups (MLUpdate.java:251-261
    collectInParallel): 4 gloo ranks split into 2 groups of 2, each group trains one ALS
    candidate with its own collectives on the data replicated into it; one MODEL is
    published and every user and item gets an UP row."""
    msgs, timing = _run_grouped(tmp_path, "als", 4, 29651)
    keys = [k for k, _ in msgs]
    assert keys.count("MODEL") == 1
    assert timing["ranks"] == 2          # the winner was trained by a 2-rank group
    assert timing["eval"] is not None
    import json
    ups = [json.loads(m) for k, m in msgs if k == "UP"]
    assert len({u[1] for u in ups if u[0] == "Y"}) == 30
    assert len({u[1] for u in ups if u[0] == "X"}) == 60


def test_candidate_groups_rdf_two_ranks(tmp_path):
    """A non-sharded app (RDF) with 2 ranks and parallelism 2: each rank builds one candidate
    alone; the better of the two is published once."""
    msgs, timing = _run_grouped(tmp_path, "rdf", 2, 29653)
    assert [k for k, _ in msgs] == ["MODEL"]
    assert timing["eval"] is not None


def test_replicate_to_groups_layout():
    """Member m of every group receives the lines of the ranks r with r % size == m."""
    from oryx_amd.parallel import dist, shuffle
    assert shuffle.replicate_to_groups(["a", "b"], dist.DistContext(), 1) == ["a", "b"]
