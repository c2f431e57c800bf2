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
