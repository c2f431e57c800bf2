"""More app-tier integration tests through the real layers and the native log -- ports of the
reference's remaining ITs:

* ``RDFCategoricalHyperParamTuningIT`` (``app/oryx-app-mllib/src/test/.../rdf/``): positive iff
  all three numeric features >= 0.5, max-depth [1, 8], 2 candidates -> the winner has depth
  8 and classifies every 0/1 corner correctly;
* ``KMeansHyperParamTuningIT`` (``.../kmeans/``): k in [2, 100] over uniform points, SSE ->
  the largest k wins (runs 2 instead of 20 to keep the CPU test short);
* ``KMeansSpeedIT`` / ``RDFSpeedIT`` (``app/oryx-app/src/test/.../speed/``): a MODEL on the
  update topic, input points / examples on the input topic, one speed-layer interval; the
  published UP rows match the reference's assertions;
* ``KMeansServingModelManagerIT`` / ``RDFServingModelManagerIT`` / ``ALSServingInputProducerIT``
  (``app/oryx-app-serving/src/test/...``): the serving layer consumes the update topic from the
  log; its input producer writes /ingest-style lines to the input topic.
"""

import json
import math
import os
import time

import numpy as np
import pytest

from oryx_amd.layers.speed import SpeedLayer
from oryx_amd.models.classreg import Example, NumericFeature
from oryx_amd.models.kmeans.common import clustering_model_pmml, read_clusters
from oryx_amd.models.rdf import pmml as rdf_pmml
from oryx_amd.models.schema import CategoricalValueEncodings, InputSchema
from oryx_amd.serving.layer import ServingLayer
from oryx_amd.transport import log as tlog
from oryx_amd.transport.producer import LogTopicProducer
from oryx_amd.utils import config as cfg
from oryx_amd.utils import pmml as pmmlu

from .test_app_its import _run_batch


def _config(tmp_path, **extra):
    overlay = {
        "oryx.id": '"it2"',
        "oryx.transport.log-dir": '"%s"' % (tmp_path / "log"),
        "oryx.batch.storage.data-dir": '"file:%s/"' % (tmp_path / "data"),
        "oryx.batch.storage.model-dir": '"file:%s/"' % (tmp_path / "model"),
        "oryx.gpu.device": '"cpu"',
    }
    overlay.update(extra)
    return cfg.overlay_on(overlay, cfg.get_default())


def _drain(root, topic):
    t = tlog.Topic(root, topic)
    c = tlog.TopicConsumer(t, start="earliest")
    out = []
    while True:
        recs = c.poll(100000, 50)
        if not recs:
            break
        out.extend((k, v) for _, _, _, k, v in recs)
    c.close()
    t.close()
    return out


# ---------------------------------------------------------------- batch ITs

def test_rdf_categorical_hyperparam_tuning(tmp_path):
    # RandomCategoricalRDFDataGenerator(3): id, three uniforms, positive iff all >= 0.5
    rng = np.random.default_rng(3)
    lines = []
    for j in range(4000):
        d = rng.random(3)
        lines.append(",".join([str(j)] + [repr(float(v)) for v in d] +
                              [str(bool((d >= 0.5).all())).lower()]))
    _, ups, model_dir = _run_batch(tmp_path, {
        "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.rdf.RDFUpdate",
        "oryx.rdf.num-trees": 10, "oryx.rdf.hyperparams.max-depth": "[1,8]",
        "oryx.rdf.hyperparams.max-split-candidates": 100,
        "oryx.input-schema.num-features": 5,
        "oryx.input-schema.categorical-features": '["4"]',
        "oryx.input-schema.id-features": '["0"]', "oryx.input-schema.target-feature": '"4"',
        "oryx.ml.eval.candidates": 2, "oryx.ml.eval.parallelism": 2}, lines)
    gens = sorted(d for d in os.listdir(model_dir) if d.isdigit())
    doc = pmmlu.read(os.path.join(model_dir, gens[-1], "model.pmml"))
    assert len(doc.extensions()) == 3
    assert doc.get_extension_value("maxSplitCandidates") == "100"
    assert doc.get_extension_value("maxDepth") == "8"
    assert doc.get_extension_value("impurity") == "entropy"
    forest, enc = rdf_pmml.read(doc)
    target = enc.get_value_encoding_map(4)
    for f1 in (0, 1):
        for f2 in (0, 1):
            for f3 in (0, 1):
                ex = Example(None, None, NumericFeature(float(f1)), NumericFeature(float(f2)),
                             NumericFeature(float(f3)))
                pred = forest.predict(ex)
                want = "true" if f1 == f2 == f3 == 1 else "false"
                assert pred.get_most_probable_category_encoding() == target[want], (f1, f2, f3)


def test_kmeans_hyperparam_tuning_picks_largest_k(tmp_path):
    rng = np.random.default_rng(9)
    lines = [",".join(repr(float(v)) for v in rng.random(5)) for _ in range(3000)]
    _, ups, model_dir = _run_batch(tmp_path, {
        "oryx.batch.update-class": "com.cloudera.oryx.app.batch.mllib.kmeans.KMeansUpdate",
        "oryx.kmeans.hyperparams.k": "[2,100]", "oryx.kmeans.iterations": 20,
        "oryx.kmeans.runs": 2, "oryx.input-schema.num-features": 5,
        "oryx.input-schema.categorical-features": "[]", "oryx.ml.eval.candidates": 3,
        "oryx.ml.eval.parallelism": 2, "oryx.kmeans.evaluation-strategy": "SSE"}, lines)
    gens = sorted(d for d in os.listdir(model_dir) if d.isdigit())
    doc = pmmlu.read(os.path.join(model_dir, gens[-1], "model.pmml"))
    assert len(read_clusters(doc)) == 100


# ---------------------------------------------------------------- speed ITs

def _speed_run(tmp_path, config, model_msgs, inputs):
    root = str(tmp_path / "log")
    tlog.maybe_create_topic(root, "OryxInput", 4)
    tlog.maybe_create_topic(root, "OryxUpdate", 1)
    upd = LogTopicProducer("localhost:9092", "OryxUpdate", config, async_=False)
    for k, m in model_msgs:
        upd.send(k, m)
    speed = SpeedLayer(config).start(start_timer=False)
    try:
        deadline = time.time() + 30
        while time.time() < deadline and speed.manager.model is None:
            time.sleep(0.05)
        time.sleep(0.2)
        inp = LogTopicProducer("localhost:9092", "OryxInput", config, async_=False)
        for line in inputs:
            inp.send(None, line)
        inp.close()
        speed.run_interval()
    finally:
        speed.close()
        upd.close()
    return _drain(root, "OryxUpdate")


def _kmeans_dummy():
    schema = InputSchema(_config_plain(**{"oryx.input-schema.feature-names": '["x","y"]',
                                          "oryx.input-schema.categorical-features": "[]"}))
    return clustering_model_pmml(schema, np.array([[1.0, 0.0], [2.0, -1.0], [-1.0, 0.0]]),
                                 [1, 2, 3])


def _config_plain(**kv):
    return cfg.overlay_on(kv, cfg.get_default())


def test_kmeans_speed_it(tmp_path):
    """KMeansSpeedIT: 300 points cycling the three UPDATE_POINTS -> one update per cluster,
    centers pulled to within 0.1 of the points, sizes = 100 + the model's."""
    config = _config(tmp_path, **{
        "oryx.speed.model-manager-class":
            "com.cloudera.oryx.app.speed.kmeans.KMeansSpeedModelManager",
        "oryx.input-schema.feature-names": '["x","y"]',
        "oryx.input-schema.categorical-features": "[]"})
    update_points = [[1.0, 1.0], [2.0, -2.0], [-2.0, 0.0]]
    inputs = [json.dumps(update_points[j % 3]) for j in range(300)]
    ups = _speed_run(tmp_path, config, [("MODEL", pmmlu.to_string(_kmeans_dummy()))], inputs)
    assert ups[0][0] == "MODEL" and len(ups) >= 4
    model_sizes = {0: 1, 1: 2, 2: 3}
    model_centers = {0: [1.0, 0.0], 1: [2.0, -1.0], 2: [-1.0, 0.0]}
    got = {}
    for k, m in ups[1:]:
        assert k == "UP"
        cid, center, count = json.loads(m)
        got[cid] = (center, count)
    assert set(got) == {0, 1, 2}
    for cid, (center, count) in got.items():
        assert center != model_centers[cid]
        np.testing.assert_allclose(center, update_points[cid], atol=0.1)
        assert count == 100 + model_sizes[cid]


def _rdf_regression_dummy():
    schema = InputSchema(_config_plain(**{"oryx.input-schema.feature-names": '["foo","bar"]',
                                          "oryx.input-schema.categorical-features": "[]",
                                          "oryx.input-schema.target-feature": "bar"}))
    root = rdf_pmml.TreeSpecNode("r", 2.0)
    root.feature, root.threshold = 0, 3.14
    root.left = rdf_pmml.TreeSpecNode("r-", 1.0)
    root.left.mean = -2.0
    root.right = rdf_pmml.TreeSpecNode("r+", 1.0)
    root.right.mean = 2.0
    return rdf_pmml.forest_to_pmml([root], schema, CategoricalValueEncodings({}), [1.0], 1, 2,
                                   "variance")


def _rdf_classification_dummy():
    schema = InputSchema(_config_plain(**{"oryx.input-schema.feature-names":
                                          '["color","fruit"]',
                                          "oryx.input-schema.numeric-features": "[]",
                                          "oryx.input-schema.target-feature": "fruit"}))
    enc = CategoricalValueEncodings({0: ["yellow", "red"], 1: ["banana", "apple"]})
    root = rdf_pmml.TreeSpecNode("r", 2.0)
    root.feature = 0
    root.left_categories = [1]
    root.left = rdf_pmml.TreeSpecNode("r-", 1.0)
    root.left.class_counts = np.array([0.0, 1.0])
    root.right = rdf_pmml.TreeSpecNode("r+", 1.0)
    root.right.class_counts = np.array([1.0, 0.0])
    return rdf_pmml.forest_to_pmml([root], schema, enc, [0.5], 3, 10, "gini")


def _min_max_expected_mean(n, positive):
    lo = hi = 0.0
    max_offset = 5 - n % 5
    for i in range(n):
        if positive:
            lo += 1 + 2 * (i % 5)
            hi += 1 + 2 * ((i + max_offset) % 5)
        else:
            lo += -2 * ((i + max_offset) % 5)
            hi += -2 * (i % 5)
    return lo / n, hi / n


def test_rdf_speed_regression_it(tmp_path):
    """RDFSpeedIT.testRDFSpeedRegression: 500 examples either side of the 3.14 split ->
    updates for r- and r+ in pairs, counts within 1, means in the reference's ranges."""
    config = _config(tmp_path, **{
        "oryx.speed.model-manager-class": "com.cloudera.oryx.app.speed.rdf.RDFSpeedModelManager",
        "oryx.input-schema.feature-names": '["foo","bar"]',
        "oryx.input-schema.categorical-features": "[]",
        "oryx.input-schema.target-feature": "bar"})
    inputs = []
    for j in range(500):
        pos = j % 2 != 0
        pred = 3.14 + j if pos else 3.14 - j
        tgt = (j % 10) if pos else -(j % 10)
        inputs.append("%r,%r" % (pred, float(tgt)))
    ups = _speed_run(tmp_path, config, [("MODEL", pmmlu.to_string(_rdf_regression_dummy()))],
                     inputs)
    n = len(ups)
    assert n >= 3 and n % 2 == 1 and ups[0][0] == "MODEL"
    recs = []
    for k, m in ups[1:]:
        assert k == "UP"
        tree, node, mean, count = json.loads(m)
        assert tree == 0 and node in ("r-", "r+")
        lo, hi = _min_max_expected_mean(count, node == "r+")
        assert lo - 1e-9 <= mean <= hi + 1e-9, (node, mean, count, lo, hi)
        recs.append((node, count))
    for a, b in zip(recs[0::2], recs[1::2]):
        assert abs(a[1] - b[1]) <= 1 and {a[0], b[0]} == {"r-", "r+"}


def test_rdf_speed_classification_it(tmp_path):
    """RDFSpeedIT.testRDFSpeedClassification: yellow => banana 90% of the time; r+ (not red)
    counts are ~9x banana, r- ~9x apple (binomial check at the reference's tolerance)."""
    config = _config(tmp_path, **{
        "oryx.speed.model-manager-class": "com.cloudera.oryx.app.speed.rdf.RDFSpeedModelManager",
        "oryx.input-schema.feature-names": '["color","fruit"]',
        "oryx.input-schema.numeric-features": "[]",
        "oryx.input-schema.target-feature": "fruit"})
    rng = np.random.default_rng(1)
    inputs = []
    for j in range(500):
        pos = j % 2 != 0
        pred = "yellow" if (pos ^ (rng.random() < 0.1)) else "red"
        inputs.append("%s,%s" % (pred, "banana" if pos else "apple"))
    doc = _rdf_classification_dummy()
    ups = _speed_run(tmp_path, config, [("MODEL", pmmlu.to_string(doc))], inputs)
    n = len(ups)
    assert n >= 3 and n % 2 == 1 and ups[0][0] == "MODEL"
    _, enc = rdf_pmml.read(pmmlu.from_string(ups[0][1]))
    fruit = enc.get_value_encoding_map(1)
    banana, apple = str(fruit["banana"]), str(fruit["apple"])
    for k, m in ups[1:]:
        tree, node, counts = json.loads(m)
        assert tree == 0 and node in ("r-", "r+")
        b, a = counts.get(banana, 0), counts.get(apple, 0)
        total = a + b
        assert total > 0
        major = b if node == "r+" else a
        # checkProbability: within 4 standard deviations of Binomial(total, 0.9)
        mean, sd = 0.9 * total, math.sqrt(total * 0.9 * 0.1)
        assert abs(major - mean) <= 4 * sd + 1, (node, counts)


# ---------------------------------------------------------------- serving ITs

def _serving(tmp_path, overlay, model_msgs):
    config = _config(tmp_path, **dict({"oryx.serving.api.port": 0}, **overlay))
    root = str(tmp_path / "log")
    tlog.maybe_create_topic(root, "OryxInput", 4)
    tlog.maybe_create_topic(root, "OryxUpdate", 1)
    layer = ServingLayer(config, host="127.0.0.1").start()
    upd = LogTopicProducer("localhost:9092", "OryxUpdate", config, async_=False)
    for k, m in model_msgs:
        upd.send(k, m)
    upd.close()
    return layer


def _wait(pred, timeout=30):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(0.05)
    return False


def test_kmeans_serving_model_manager_it(tmp_path):
    msgs = [("MODEL", pmmlu.to_string(_kmeans_dummy()))]
    msgs += [("UP", json.dumps([i % 3, [i, i], i])) for i in range(1, 10)]
    layer = _serving(tmp_path, {
        "oryx.serving.application-resources":
            '"com.cloudera.oryx.app.serving,com.cloudera.oryx.app.serving.clustering,'
            'com.cloudera.oryx.app.serving.kmeans"',
        "oryx.serving.model-manager-class":
            "com.cloudera.oryx.app.serving.kmeans.model.KMeansServingModelManager",
        "oryx.input-schema.feature-names": '["x","y"]',
        "oryx.input-schema.categorical-features": "[]"}, msgs)
    try:
        mgr = layer.manager

        def done():
            m = mgr.get_model()
            return m is not None and m.get_cluster(0).get_count() == 9 and \
                m.get_cluster(1).get_count() == 7 and m.get_cluster(2).get_count() == 8
        assert _wait(done)
        m = mgr.get_model()
        assert m.get_num_clusters() == 3
        for cid, center, count in ((0, [9.0, 9.0], 9), (1, [7.0, 7.0], 7), (2, [8.0, 8.0], 8)):
            c = m.get_cluster(cid)
            assert c.get_id() == cid and list(c.get_center()) == center and \
                c.get_count() == count
    finally:
        layer.close()


def test_rdf_serving_model_manager_it(tmp_path):
    msgs = [("MODEL", pmmlu.to_string(_rdf_classification_dummy()))]
    msgs += [("UP", json.dumps([0, "r-" if i % 2 == 0 else "r+", {"0": 1, "1": 2}]))
             for i in range(1, 5)]
    layer = _serving(tmp_path, {
        "oryx.serving.application-resources":
            '"com.cloudera.oryx.app.serving,com.cloudera.oryx.app.serving.classreg,'
            'com.cloudera.oryx.app.serving.rdf"',
        "oryx.serving.model-manager-class":
            "com.cloudera.oryx.app.serving.rdf.model.RDFServingModelManager",
        "oryx.input-schema.feature-names": '["color","fruit"]',
        "oryx.input-schema.numeric-features": "[]",
        "oryx.input-schema.target-feature": "fruit"}, msgs)
    try:
        mgr = layer.manager

        def done():
            m = mgr.get_model()
            if m is None:
                return False
            t = m.get_forest().get_trees()[0]
            return t.find_by_id("r-").get_count() == 7 and t.find_by_id("r+").get_count() == 7
        assert _wait(done)
        m = mgr.get_model()
        enc = m.get_encodings()
        assert enc.get_value_count(0) == 2 and enc.get_value_count(1) == 2
        assert enc.get_encoding_value_map(0) == {0: "yellow", 1: "red"}
        assert enc.get_encoding_value_map(1) == {0: "banana", 1: "apple"}
        forest = m.get_forest()
        assert len(forest.get_trees()) == 1 and list(forest.get_weights()) == [1.0]
        assert m.get_input_schema().get_num_features() == 2
        tree = forest.get_trees()[0]
        root, left, right = (tree.find_by_id(x) for x in ("r", "r-", "r+"))
        assert root.left is left and root.right is right
        assert list(left.get_prediction().get_category_counts()) == [2, 5]
        assert list(right.get_prediction().get_category_counts()) == [3, 4]
    finally:
        layer.close()


def test_als_serving_input_producer_it(tmp_path):
    layer = _serving(tmp_path, {
        "oryx.serving.application-resources":
            '"com.cloudera.oryx.app.serving,com.cloudera.oryx.app.serving.als"',
        "oryx.serving.model-manager-class":
            "com.cloudera.oryx.app.serving.als.model.ALSServingModelManager"}, [])
    inputs = ["abc,123,1.5", "xyz,234,-0.5", "AB,10,0"]
    try:
        prod = layer._input_producer
        assert prod is not None
        for line in inputs:
            prod.send(None, line)
        prod.flush() if hasattr(prod, "flush") else None
        root = str(tmp_path / "log")
        assert _wait(lambda: len(_drain(root, "OryxInput")) == 3)
        got = _drain(root, "OryxInput")
        # one partition per key-less send in order of arrival per partition: compare as sets
        # of (key, value) with null keys, and the full sequence when the topic has one part
        assert all(k is None for k, _ in got)
        assert sorted(v for _, v in got) == sorted(inputs)
    finally:
        layer.close()
