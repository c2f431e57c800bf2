"""App-tier batch integration tests through the real batch layer and native log, ports of
the reference's ``app/oryx-app-mllib`` ITs:

* ALSModelContentIT -- delete semantics and exact known-item sets in the published model;
* ALSHyperParamTuningIT -- planted 7-category structure: features=7 beats features=1;
* RDFNumericHyperParamTuningIT -- target = number of "A" features, max-depth [1, 8]: the
  winning tree predicts f1+f2+f3 exactly after rounding.
"""

import json
import os

import numpy as np

from oryx_amd.layers.batch import BatchLayer
from oryx_amd.models.classreg import CategoricalFeature, Example
from oryx_amd.models.rdf import pmml as rdf_pmml
from oryx_amd.transport import log as tlog
from oryx_amd.transport.producer import LogTopicProducer
from oryx_amd.utils import config as cfg
from oryx_amd.utils import ioutils
from oryx_amd.utils import pmml as pmmlu


def _sid(i):
    return chr(ord("A") + i % 26) + str(i)


def _run_batch(tmp_path, overlay, lines, generations=1):
    base = {
        "oryx.id": '"app-it"',
        "oryx.transport.log-dir": '"%s"' % (tmp_path / "log"),
        "oryx.batch.storage.data-dir": '"file:%s/"' % (tmp_path / "data"),
        "oryx.batch.storage.model-dir": '"file:%s/"' % (tmp_path / "model"),
        "oryx.gpu.device": '"cpu"',
    }
    base.update(overlay)
    config = cfg.overlay_on(base, cfg.get_default())
    root = str(tmp_path / "log")
    tlog.maybe_create_topic(root, "OryxInput", 4)
    tlog.maybe_create_topic(root, "OryxUpdate", 1)
    batch = BatchLayer(config)
    batch.run_interval()
    prod = LogTopicProducer("localhost:9092", "OryxInput", config, async_=False)
    per = (len(lines) + generations - 1) // generations
    for g in range(generations):
        for j, line in enumerate(lines[g * per:(g + 1) * per]):
            prod.send(str(j), line)
        batch.run_interval()
    prod.close()
    batch.close()
    t = tlog.Topic(root, "OryxUpdate")
    c = tlog.TopicConsumer(t, start="earliest")
    ups = []
    while True:
        recs = c.poll(100000, 50)
        if not recs:
            break
        ups.extend((k, v) for _, _, _, k, v in recs)
    c.close()
    t.close()
    model_dir = ioutils.to_local_path(config.get_string("oryx.batch.storage.model-dir"))
    return config, ups, model_dir


def test_als_model_content(tmp_path):
    # users u interact with items i >= u; then every (i, i) is deleted; then A0->A0 restored
    lines, t = [], 1_600_000_000_000
    for u in range(4):
        for i in range(u, 4):
            lines.append("%s,%s,1,%d" % (_sid(u), _sid(i), t))
            t += 1
    for ui in range(4):
        lines.append("%s,%s,,%d" % (_sid(ui), _sid(ui), t))
        t += 1
    lines.append("A0,A0,1,%d" % t)
    _, ups, _ = _run_batch(tmp_path, {
        "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.als.ALSUpdate",
        "oryx.ml.eval.test-fraction": 0, "oryx.als.implicit": "false",
        "oryx.als.hyperparams.lambda": 0.0001, "oryx.als.hyperparams.features": 2}, lines)
    known, users, items = {}, None, None
    for k, v in ups:
        if k == "UP":
            u = json.loads(v)
            if u[0] == "X":
                known[u[1]] = u[3]
        else:
            assert k in ("MODEL", "MODEL-REF")
            doc = pmmlu.read_pmml_from_update_key_message(k, v)
            users = doc.get_extension_content("XIDs")
            items = doc.get_extension_content("YIDs")
    assert sorted(users) == ["A0", "B1", "C2"]
    assert sorted(items) == ["A0", "B1", "C2", "D3"]
    assert sorted(known["A0"]) == ["A0", "B1", "C2", "D3"]
    assert sorted(known["B1"]) == ["C2", "D3"]
    assert sorted(known["C2"]) == ["D3"]


def test_als_hyperparam_tuning_picks_planted_rank(tmp_path):
    # FeaturesALSDataGenerator: product == user (mod 7) -- 7 distinct categories
    rng = np.random.default_rng(5)
    lines, t = [], 1_600_000_000_000
    for _ in range(2000):
        user = int(rng.integers(100))
        rp = int(rng.integers(100))
        product = ((user % 7) + (rp // 7) * 7) % 100
        lines.append("%s,%s,1,%d" % (_sid(user), _sid(product), t))
        t += 1
    _, ups, model_dir = _run_batch(tmp_path, {
        "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.als.ALSUpdate",
        "oryx.als.hyperparams.features": "[1,7]", "oryx.ml.eval.candidates": 2,
        "oryx.ml.eval.parallelism": 2}, lines)
    gens = sorted(d for d in os.listdir(model_dir) if d.isdigit())
    doc = pmmlu.read(os.path.join(model_dir, gens[-1], "model.pmml"))
    assert len(doc.extensions()) == 8
    assert doc.get_extension_value("X") and doc.get_extension_value("Y")
    assert doc.get_extension_value("features") == "7"
    assert float(doc.get_extension_value("lambda")) == 0.001
    assert doc.get_extension_value("implicit") == "true"
    assert float(doc.get_extension_value("alpha")) == 1.0


def test_rdf_numeric_hyperparam_tuning(tmp_path):
    # RandomNumericRDFDataGenerator(3): id, three of A/B, target = number of A
    rng = np.random.default_rng(11)
    lines = []
    for j in range(2000):
        f = ["A" if rng.random() < 0.5 else "B" for _ in range(3)]
        lines.append(",".join([str(j)] + f + [str(f.count("A"))]))
    _, ups, model_dir = _run_batch(tmp_path, {
        "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.rdf.RDFUpdate",
        "oryx.rdf.num-trees": 1, "oryx.rdf.hyperparams.max-depth": "[1,8]",
        "oryx.rdf.hyperparams.max-split-candidates": 100,
        "oryx.rdf.hyperparams.impurity": "variance",
        "oryx.input-schema.num-features": 5, "oryx.input-schema.numeric-features": '["4"]',
        "oryx.input-schema.id-features": '["0"]', "oryx.input-schema.target-feature": '"4"',
        "oryx.ml.eval.candidates": 2, "oryx.ml.eval.parallelism": 2}, lines)
    gens = sorted(d for d in os.listdir(model_dir) if d.isdigit())
    doc = pmmlu.read(os.path.join(model_dir, gens[-1], "model.pmml"))
    assert len(doc.extensions()) == 3
    assert doc.get_extension_value("maxSplitCandidates") == "100"
    assert doc.get_extension_value("maxDepth") == "8"
    assert doc.get_extension_value("impurity") == "variance"
    forest, enc = rdf_pmml.read(doc)
    for f1 in (0, 1):
        for f2 in (0, 1):
            for f3 in (0, 1):
                feats = [CategoricalFeature.for_encoding(
                    enc.get_value_encoding_map(idx)["A" if f else "B"])
                    for idx, f in ((1, f1), (2, f2), (3, f3))]
                ex = Example(None, None, *feats)
                pred = forest.predict(ex).get_prediction()
                assert round(pred) == f1 + f2 + f3, (f1, f2, f3, pred)
