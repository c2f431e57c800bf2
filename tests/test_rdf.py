"""RDF app tests: ports of the reference's decision/tree/forest/prediction tests
(T[app-common]/rdf/**, T[app-common]/classreg/**), the RDF PMML codec tests
(RDFPMMLUtilsTest), the serving endpoint tests with TestRDF{Regression,Classification}
ModelFactory golden values (T[serving-app]/rdf/*Test.java), plus trainer/speed checks."""

import json
import math

import numpy as np
import pytest
import torch

from oryx_amd.api import Dataset, KeyMessage
from oryx_amd.models.classreg import (CategoricalFeature, CategoricalPrediction, Example,
                                      NumericFeature, NumericPrediction, data_to_example,
                                      vote_on_feature)
from oryx_amd.models.rdf import pmml as rdf_pmml
from oryx_amd.models.rdf.batch import RDFUpdate, evaluate_forest, parse_examples
from oryx_amd.models.rdf.serving import RDFServingModel, RDFServingModelManager
from oryx_amd.models.rdf.speed import RDFSpeedModelManager
from oryx_amd.models.rdf.tree import (CategoricalDecision, DecisionForest, DecisionNode,
                                      DecisionTree, NumericDecision, TerminalNode, TreePath)
from oryx_amd.models.schema import CategoricalValueEncodings, InputSchema
from oryx_amd.ops import rdf as rdf_ops
from oryx_amd.transport.producer import MockTopicProducer
from oryx_amd.utils import config as cfg
from oryx_amd.utils import pmml as pm

from .serving_harness import Client


def _conf(**kv):
    return cfg.overlay_on({k.replace("__", "."): v for k, v in kv.items()}, cfg.get_default())


def _schema(**kv):
    return InputSchema(_conf(**kv))


# ---------------------------------------------------------------- decisions / trees

def test_numeric_decision():
    d = NumericDecision(0, -3.1, True)
    assert not d.is_positive(Example(None, NumericFeature(-3.5)))
    assert d.is_positive(Example(None, NumericFeature(-3.1)))
    assert d.is_positive(Example(None, NumericFeature(3.1)))
    assert d.is_positive(Example(None, [None]))
    assert repr(NumericDecision(0, 0.5, True)) == "(#0 >= 0.5)"
    assert NumericDecision(0, 0.5, True) == NumericDecision(0, 0.5, False)
    assert NumericDecision(0, 0.5, True) != NumericDecision(1, 0.5, True)


def test_categorical_decision():
    d = CategoricalDecision(0, {2, 5}, True)
    for i in range(10):
        assert d.is_positive(Example(None, CategoricalFeature.for_encoding(i))) == (i in (2, 5))
    assert d.is_positive(Example(None, [None]))
    assert repr(d) == "(#0 ∈ [2,5])"


def build_test_tree():
    rnn = TerminalNode("r--", NumericPrediction(0.0, 1))
    rnp = TerminalNode("r-+", NumericPrediction(1.0, 1))
    rn = DecisionNode("r-", NumericDecision(0, -1.0, False), rnn, rnp)
    rp = TerminalNode("r+", NumericPrediction(2.0, 1))
    return DecisionTree(DecisionNode("r", NumericDecision(0, 1.0, False), rn, rp))


def test_decision_tree():
    tree = build_test_tree()
    assert tree.predict(Example(None, NumericFeature(0.5))).get_prediction() == 1.0
    assert tree.find_terminal(Example(None, NumericFeature(0.5))).get_prediction() \
        .get_prediction() == 1.0
    assert tree.find_by_id("r-+").get_prediction().get_prediction() == 1.0
    s = repr(tree)
    assert s.startswith("(#0 >= 1.0)") and "(#0 >= -1.0)" in s
    forest = DecisionForest([build_test_tree(), build_test_tree()], [1.0, 2.0], None)
    assert forest.predict(Example(None, NumericFeature(0.5))).get_prediction() == 1.0
    assert repr(forest).startswith("(#0 >= 1.0)")


def test_tree_path():
    lrl = TreePath.EMPTY.extend_left().extend_right().extend_left()
    lrr = TreePath.EMPTY.extend_left().extend_right().extend_right()
    lr = TreePath.EMPTY.extend_left().extend_right()
    r = TreePath.EMPTY.extend_right()
    assert repr(lrl) == "010" and repr(lrr) == "011" and repr(TreePath.EMPTY) == ""
    assert lrl == TreePath.EMPTY.extend_left().extend_right().extend_left()
    assert sorted([lrl, r, lr, lrr]) == [lrl, lr, lrr, r]


def test_predictions_and_vote():
    v = vote_on_feature([NumericPrediction(1.0, 1), NumericPrediction(3.0, 2),
                         NumericPrediction(6.0, 3)], [1.0, 1.0, 1.0])
    assert v.get_prediction() == pytest.approx(10.0 / 3.0)
    c = vote_on_feature([CategoricalPrediction([1, 2, 3]), CategoricalPrediction([10, 30, 50])],
                        [1.0, 2.0])
    np.testing.assert_allclose(c.get_category_probabilities(),
                               [(1 / 6 + 2 * 10 / 90) / 3, (2 / 6 + 2 * 30 / 90) / 3,
                                (3 / 6 + 2 * 50 / 90) / 3])
    p = CategoricalPrediction([1, 2, 3])
    assert p.get_most_probable_category_encoding() == 2 and p.get_count() == 6
    p.update(0, 10)
    assert p.get_most_probable_category_encoding() == 0 and p.get_count() == 16
    n = NumericPrediction(1.0, 1)
    n.update(3.0, 3)
    assert n.get_prediction() == 2.5 and n.get_count() == 4


def test_data_to_example():
    s = _schema(**{"oryx__input-schema__feature-names": '["a","b","c"]',
                   "oryx__input-schema__categorical-features": '["a","c"]',
                   "oryx__input-schema__target-feature": "c"})
    enc = CategoricalValueEncodings({0: ["x", "y"], 2: ["p", "q"]})
    e = data_to_example(["y", "1.5", "q"], s, enc)
    assert e.get_feature(0) == CategoricalFeature.for_encoding(1)
    assert e.get_feature(1) == NumericFeature(1.5)
    assert e.get_feature(2) is None and e.get_target() == CategoricalFeature.for_encoding(1)
    assert data_to_example(["x", "2", ""], s, enc).get_target() is None


# ---------------------------------------------------------------- PMML codec

def _dummy_classification_pmml(num_trees=1):
    s = _schema(**{"oryx__input-schema__feature-names": '["color","fruit"]',
                   "oryx__input-schema__numeric-features": "[]",
                   "oryx__input-schema__target-feature": "fruit"})
    enc = CategoricalValueEncodings({0: ["yellow", "red"], 1: ["banana", "apple"]})
    roots = []
    for _ in range(num_trees):
        root = rdf_pmml.TreeSpecNode("r", 2.0)
        root.feature = 0
        root.left_categories = [1]           # red goes left -> "isNotIn red" on the right
        root.left = rdf_pmml.TreeSpecNode("r-", 1.0)
        root.left.class_counts = np.array([0.0, 1.0])
        root.right = rdf_pmml.TreeSpecNode("r+", 1.0)
        root.right.class_counts = np.array([1.0, 0.0])
        roots.append(root)
    return s, enc, rdf_pmml.forest_to_pmml(roots, s, enc, [0.5], 3, 10, "gini")


def test_pmml_classification_round_trip():
    s, enc, doc = _dummy_classification_pmml()
    doc = pm.from_string(pm.to_string(doc))
    rdf_pmml.validate_pmml_vs_schema(doc, s)
    forest, enc2 = rdf_pmml.read(doc)
    assert len(forest.get_trees()) == 1 and forest.get_weights().tolist() == [1.0]
    assert forest.get_feature_importances().tolist() == [0.5, 0.0]
    assert enc2.get_value_count(0) == 2 and enc2.get_value_count(1) == 2
    root = forest.get_trees()[0].get_root()
    assert isinstance(root.decision, CategoricalDecision) and root.decision.active == {0}
    red = Example(None, CategoricalFeature.for_encoding(1), None)
    assert forest.predict(red).get_most_probable_category_encoding() == 1   # apple
    assert doc.get_extension_value("impurity") == "gini"
    s3, enc3, doc3 = _dummy_classification_pmml(3)
    assert len(rdf_pmml.read(doc3)[0].get_trees()) == 3


def test_pmml_regression_greater_than_ulp():
    s = _schema(**{"oryx__input-schema__feature-names": '["foo","bar"]',
                   "oryx__input-schema__categorical-features": "[]",
                   "oryx__input-schema__target-feature": "bar"})
    enc = CategoricalValueEncodings({})
    root = rdf_pmml.TreeSpecNode("r", 2.0)
    root.feature, root.threshold = 0, 3.14
    root.left = rdf_pmml.TreeSpecNode("r-", 1.0)
    root.left.mean = -2.0
    root.right = rdf_pmml.TreeSpecNode("r+", 1.0)
    root.right.mean = 2.0
    doc = rdf_pmml.forest_to_pmml([root], s, enc, [1.0], 1, 2, "variance")
    rdf_pmml.validate_pmml_vs_schema(doc, s)
    forest, enc2 = rdf_pmml.read(doc)
    assert enc2.get_category_counts() == {}
    d = forest.get_trees()[0].get_root().decision
    assert d.get_threshold() == 3.14 + math.ulp(3.14)
    assert forest.predict(Example(None, NumericFeature(3.14), None)).get_prediction() == -2.0
    assert forest.predict(Example(None, NumericFeature(3.15), None)).get_prediction() == 2.0
    bad = _schema(**{"oryx__input-schema__feature-names": '["foo","bar"]',
                     "oryx__input-schema__numeric-features": "[]",
                     "oryx__input-schema__target-feature": "bar"})
    with pytest.raises(ValueError):
        rdf_pmml.validate_pmml_vs_schema(doc, bad)


# ---------------------------------------------------------------- serving (golden values)

def _forest(preds1, preds2):
    enc_left = CategoricalDecision(0, {1}, True)
    t1 = DecisionTree(DecisionNode("r", enc_left, TerminalNode("r-", preds1[0]),
                                   TerminalNode("r+", preds1[1])))
    t2 = DecisionTree(DecisionNode("r", NumericDecision(1, -3.0, False),
                                   TerminalNode("r-", preds2[0]), TerminalNode("r+", preds2[1])))
    return DecisionForest([t1, t2], [1.0, 2.0], [0.1, 0.3])


def regression_model():
    forest = _forest([NumericPrediction(1.0, 1), NumericPrediction(10.0, 1)],
                     [NumericPrediction(100.0, 1), NumericPrediction(1000.0, 1)])
    enc = CategoricalValueEncodings({0: ["A", "B", "C"]})
    s = _schema(**{"oryx__input-schema__num-features": 3,
                   "oryx__input-schema__categorical-features": '["0"]',
                   "oryx__input-schema__target-feature": '"2"'})
    return RDFServingModel(forest, enc, s)


def classification_model():
    forest = _forest([CategoricalPrediction([1, 2, 3]), CategoricalPrediction([10, 30, 50])],
                     [CategoricalPrediction([100, 400, 900]),
                      CategoricalPrediction([1000, 10000, 100000])])
    enc = CategoricalValueEncodings({0: ["A", "B", "C"], 2: ["X", "Y", "Z"]})
    s = _schema(**{"oryx__input-schema__num-features": 3,
                   "oryx__input-schema__categorical-features": '["0","2"]',
                   "oryx__input-schema__target-feature": '"2"'})
    return RDFServingModel(forest, enc, s)


def _client(model, read_only=False):
    return Client(["oryx_amd.models.rdf.resources"], model, read_only=read_only)


def test_serving_predict():
    c = _client(regression_model())
    assert float(c.get_text("/predict/B,0,")) == pytest.approx((10.0 + 2 * 1000.0) / 3)
    assert float(c.get_text("/predict/A,-5,")) == pytest.approx((1.0 + 2.0 * 100.0) / 3.0)
    r = c.request("POST", "/predict", body="A,-5,\nB,0,")
    assert r.body.decode() == "67.0\n670.0\n"
    assert c.status("GET", "/predict/B,0") == 400


def test_serving_classification_distribution():
    c = _client(classification_model())
    recs = c.get_json("/classificationDistribution/B,0,")
    assert [r["id"] for r in recs] == ["X", "Y", "Z"]
    assert recs[0]["value"] == pytest.approx((10.0 / 90.0 + 2 * (1000.0 / 111000.0)) / 3)
    assert recs[2]["value"] == pytest.approx((50.0 / 90.0 + 2 * (100000.0 / 111000.0)) / 3)
    recs = c.get_json("/classificationDistribution/A,-5,")
    assert recs[1]["value"] == pytest.approx((2.0 / 6.0 + 2 * (400.0 / 1400.0)) / 3)
    assert c.get_text("/predict/A,-5,").strip() == "Z"


def test_serving_feature_importance_and_train():
    c = _client(regression_model())
    assert c.get_json("/feature/importance") == [0.1, 0.3]
    assert float(c.get_text("/feature/importance/1")) == 0.3
    assert c.status("GET", "/feature/importance/5") == 400
    data = "B,0,20\nB,-4,30\nA,0,40\nA,-4,50"
    assert c.status("POST", "/train", body=data) == 204
    assert [m for _, m in MockTopicProducer.get_key_messages()] == data.split("\n")
    assert _client(regression_model(), read_only=True).status("POST", "/train",
                                                              body=data) == 403


def test_serving_manager_updates():
    s, enc, doc = _dummy_classification_pmml()
    conf = _conf(**{"oryx__input-schema__feature-names": '["color","fruit"]',
                    "oryx__input-schema__numeric-features": "[]",
                    "oryx__input-schema__target-feature": "fruit"})
    mgr = RDFServingModelManager(conf)
    mgr.consume(iter([KeyMessage("MODEL", pm.to_string(doc)),
                      KeyMessage("UP", '[0,"r+",{"1":5}]')]))
    leaf = mgr.get_model().get_forest().get_trees()[0].find_by_id("r+")
    assert leaf.get_prediction().get_category_counts().tolist() == [1.0, 5.0]
    assert mgr.get_model().predict(["yellow", ""]) == "apple"


# ---------------------------------------------------------------- training

def _numeric_data(n=3000, seed=0):
    g = np.random.default_rng(seed)
    X = g.uniform(-1, 1, (n, 4))
    y = np.where(X[:, 0] + 0.5 * X[:, 1] > 0.2, 1, 0)
    return X, y


def test_train_single_tree_classification_cpu():
    X, y = _numeric_data()
    data = rdf_ops.bin_features(X, [False] * 4, [0] * 4, 32, torch.device("cpu"))
    f = rdf_ops.train_forest(data, torch.from_numpy(y), 2, 1, 6, "gini", seed=1)
    root = f.roots[0]
    assert root.feature in (0, 1) and root.count == len(y)
    # counts are consistent: children sum to parent
    stack = [root]
    while stack:
        nd = stack.pop()
        if nd.feature >= 0:
            assert nd.left.count + nd.right.count == nd.count
            stack += [nd.left, nd.right]
    assert f.predictor_counts[0] > 0


def _rdf_conf(classification=True, trees=5):
    kv = {"oryx__input-schema__feature-names": '["a","b","c","d","t"]',
          "oryx__input-schema__target-feature": "t",
          "oryx__rdf__num-trees": trees,
          "oryx__rdf__hyperparams__max-depth": 6,
          "oryx__rdf__hyperparams__max-split-candidates": 32,
          "oryx__ml__eval__test-fraction": 0.2,
          "oryx__ml__eval__candidates": 1}
    if classification:
        kv["oryx__input-schema__categorical-features"] = '["d","t"]'
        kv["oryx__rdf__hyperparams__impurity"] = "entropy"
    else:
        kv["oryx__input-schema__categorical-features"] = '["d"]'
        kv["oryx__rdf__hyperparams__impurity"] = "variance"
    return _conf(**kv)


def _lines(n, classification, seed=3):
    g = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        a, b, c = (float(v) for v in g.uniform(-1, 1, 3))
        d = str(g.choice(["red", "green", "blue"]))
        if classification:
            t = "yes" if (a > 0.1) ^ (d == "blue") else "no"
        else:
            t = repr(round(3 * a - 2 * b + (4.0 if d == "red" else 0.0), 4))
        out.append("%r,%r,%r,%s,%s" % (a, b, c, d, t))
    return out


@pytest.mark.parametrize("classification", [True, False])
def test_rdf_update_end_to_end(classification, tmp_path):
    conf = _rdf_conf(classification)
    upd = RDFUpdate(conf)
    lines = _lines(2500, classification)
    MockTopicProducer.clear()
    upd.run_update(None, 1, Dataset([(None, l) for l in lines]), None,
                   str(tmp_path / "model"), MockTopicProducer())
    (k, m), = MockTopicProducer.get_key_messages()
    assert k == "MODEL"
    doc = pm.from_string(m)
    schema = InputSchema(conf)
    rdf_pmml.validate_pmml_vs_schema(doc, schema)
    forest, enc = rdf_pmml.read(doc)
    assert len(forest.get_trees()) == 5
    assert doc.models()[0].tag == pm.q("MiningModel")
    imp = forest.get_feature_importances()
    assert imp[4] == 0.0 and abs(imp.sum() - 1.0) < 1e-9
    test = _lines(500, classification, seed=9)
    rows = [l.split(",") for l in test]
    _, target, full = parse_examples(rows, schema, enc)
    ev = evaluate_forest(forest, enc, schema, full, target, torch.device("cpu"))
    if classification:
        assert ev > 0.9
    else:
        assert ev < 1.0
    # host tree walk agrees with the flattened device-style walk
    from oryx_amd.models.classreg import data_to_example
    preds = [forest.predict(data_to_example(r, schema, enc)) for r in rows[:50]]
    flat = rdf_ops.flatten_forest(forest, torch.device("cpu"),
                                  enc.get_value_count(4) if classification else 0)
    leaves = rdf_ops.forest_leaves(flat, torch.from_numpy(full[:50]))
    for e in range(50):
        for t in range(5):
            assert flat.nodes[int(leaves[e, t])] is forest.get_trees()[t].find_terminal(
                data_to_example(rows[e], schema, enc))


def test_speed_manager_leaf_updates():
    conf = _rdf_conf(False, trees=2)
    upd = RDFUpdate(conf)
    MockTopicProducer.clear()
    upd.run_update(None, 1, Dataset([(None, l) for l in _lines(800, False)]), None, "/tmp/rdfm",
                   MockTopicProducer())
    (k, m), = MockTopicProducer.get_key_messages()
    mgr = RDFSpeedModelManager(conf)
    mgr.consume(iter([KeyMessage(k, m)]))
    ups = [json.loads(u) for u in mgr.build_updates(Dataset([(None, l)
                                                             for l in _lines(20, False, 5)]))]
    assert ups and all(len(u) == 4 for u in ups)
    assert sum(u[3] for u in ups if u[0] == 0) == 20
    serving = RDFServingModelManager(conf)
    serving.consume(iter([KeyMessage(k, m)] + [KeyMessage("UP", json.dumps(u)) for u in ups]))


@pytest.mark.gpu
@pytest.mark.parametrize("classification", [True, False])
def test_speed_manager_device_path_matches_host(cuda, classification):
    """The GPU speed path (leaf kernel, one device bincount, native message formatting)
    emits the same updates in the same order as the host path, from a TextLines buffer."""
    from oryx_amd.textlines import TextLines
    conf = _rdf_conf(classification, trees=3)
    upd = RDFUpdate(conf)
    MockTopicProducer.clear()
    upd.run_update(None, 1, Dataset([(None, l) for l in _lines(800, classification)]), None,
                   "/tmp/rdfm_dev", MockTopicProducer())
    (k, m), = MockTopicProducer.get_key_messages()
    lines = _lines(300, classification, 9)
    outs = []
    for device in (torch.device(cuda), torch.device("cpu")):
        mgr = RDFSpeedModelManager(conf)
        mgr.device = device
        mgr.consume(iter([KeyMessage(k, m)]))
        outs.append([json.loads(u) for u in mgr.build_updates(
            Dataset.from_values(TextLines.from_strings(lines)))])
    dev, host = outs
    assert len(dev) == len(host) > 0
    for a, b in zip(dev, host):
        assert a[:2] == b[:2]
        if classification:
            assert a[2] == b[2]
        else:
            assert a[3] == b[3] and a[2] == pytest.approx(b[2], rel=1e-12)


# ---------------------------------------------------------------- GPU kernels

@pytest.mark.gpu
@pytest.mark.parametrize("classification", [True, False])
def test_gpu_training_matches_cpu(cuda, classification):
    X, y = _numeric_data(20000, seed=4)
    yr = X[:, 0] * 2 - X[:, 2]
    res = {}
    for dev in (torch.device("cpu"), cuda):
        data = rdf_ops.bin_features(X, [False] * 4, [0] * 4, 32, dev, seed=2)
        tgt = torch.from_numpy(y if classification else yr)
        f = rdf_ops.train_forest(data, tgt, 2 if classification else 0, 1, 5,
                                 "gini" if classification else "variance", seed=3)
        res[dev.type] = f
    # single tree, no bootstrap, all features: identical structure (up to fp32 ties)
    a, b = res["cpu"].roots[0], res["cuda"].roots[0]
    assert (a.feature, a.bin, a.count) == (b.feature, b.bin, b.count)
    assert (a.left.feature, a.left.bin) == (b.left.feature, b.left.bin)
    np.testing.assert_allclose(res["cpu"].predictor_counts, res["cuda"].predictor_counts)


@pytest.mark.gpu
def test_gpu_forest_leaves_match_cpu(cuda):
    conf = _rdf_conf(True, trees=4)
    upd = RDFUpdate(conf)
    MockTopicProducer.clear()
    upd.run_update(None, 1, Dataset([(None, l) for l in _lines(3000, True)]), None, "/tmp/rdfg",
                   MockTopicProducer())
    (k, m), = MockTopicProducer.get_key_messages()
    forest, enc = rdf_pmml.read(pm.from_string(m))
    schema = InputSchema(conf)
    rows = [l.split(",") for l in _lines(1000, True, seed=11)]
    _, target, full = parse_examples(rows, schema, enc)
    flat_c = rdf_ops.flatten_forest(forest, torch.device("cpu"), 2)
    flat_g = rdf_ops.flatten_forest(forest, cuda, 2)
    lc = rdf_ops.forest_leaves(flat_c, torch.from_numpy(full))
    lg = rdf_ops.forest_leaves(flat_g, torch.from_numpy(full).to(cuda)).cpu()
    assert torch.equal(lc, lg)
    # fused traversal + weighted vote (K15) == leaves then the gathered vote on the host
    vc = rdf_ops.forest_vote(flat_c, torch.from_numpy(full))
    vg = rdf_ops.forest_vote(flat_g, torch.from_numpy(full).to(cuda)).cpu()
    torch.testing.assert_close(vg, vc, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("cls", [True, False])
@pytest.mark.parametrize("n,P", [(40000, 12), (40001, 13)])
def test_histogram_and_route_kernels_match_cpu(cuda, cls, n, P):
    """Level kernels on a wide level (200 node slots -> several LDS node chunks per tree,
    bootstrap weights, 3 trees) against the CPU index_add / gather implementations.  P = 13
    puts rows off dword boundaries and leaves a partial dword at the end of the bins."""
    g = torch.Generator().manual_seed(5)
    B, T, nodes, Fs = 40, 3, 200, 5
    Xb = torch.randint(0, B, (n, P), generator=g).to(torch.uint8)
    data = rdf_ops.BinnedData(Xb, [B] * P, [np.arange(B - 1, dtype=np.float64)] * P,
                              [False] * P, B)
    node_of = torch.randint(-1, nodes, (T, n), generator=g).to(torch.int32)
    weight = torch.randint(0, 3, (T, n), generator=g).to(torch.uint8)
    feats = torch.stack([torch.stack([torch.randperm(P, generator=g)[:Fs]
                                      for _ in range(nodes)]) for _ in range(T)]).int()
    if cls:
        label, y, S = torch.randint(0, 4, (n,), generator=g).int(), None, 4
    else:
        label, y, S = None, torch.randn(n, generator=g), 3
    h_cpu = rdf_ops._histogram(data, label, y, S, cls, weight, node_of, 0, nodes, feats, B)
    gd = rdf_ops.BinnedData(Xb.to(cuda), data.n_bins, data.thresholds, data.categorical, B)
    h_gpu = rdf_ops._histogram(gd, label.to(cuda) if cls else None,
                               None if cls else y.to(cuda), S, cls, weight.to(cuda),
                               node_of.to(cuda), 0, nodes, feats.to(cuda), B)
    assert torch.allclose(h_gpu.cpu(), h_cpu, rtol=1e-4, atol=1e-3)
    # grouped rows (counting sort by (tree, node)) through the segmented kernel, in two node
    # chunks
    groups = rdf_ops.RowGroups.from_nodes(node_of.to(cuda), nodes, weight.to(cuda))
    assert groups is not None
    assert int(groups.counts.sum()) == int(((node_of >= 0) & (weight > 0)).sum())
    h_grp = torch.cat([rdf_ops._histogram_groups(
        gd, label.to(cuda) if cls else None, None if cls else y.to(cuda), S, cls,
        weight.to(cuda), groups, lo, hi - lo, feats[:, lo:hi].to(cuda), B, T)
        for lo, hi in ((0, 77), (77, nodes))], 1)
    assert torch.allclose(h_grp.cpu(), h_cpu, rtol=1e-4, atol=1e-3)
    root = rdf_ops.RowGroups.root(T, n)
    h_root = rdf_ops._histogram_groups(gd, label.to(cuda) if cls else None,
                                       None if cls else y.to(cuda), S, cls, weight.to(cuda),
                                       root, 0, 1, feats[:, :1].to(cuda), B, T)
    h_root_cpu = rdf_ops._histogram(data, label, y, S, cls, weight,
                                    torch.zeros((T, n), dtype=torch.int32), 0, 1, feats[:, :1],
                                    B)
    assert torch.allclose(h_root.cpu(), h_root_cpu, rtol=1e-4, atol=1e-2)
    # routing: half the nodes split on a random feature/bin, the rest become leaves
    sf = torch.where(torch.rand(T, nodes, generator=g) < 0.5,
                     torch.randint(0, P, (T, nodes), generator=g), torch.full((T, nodes), -1))
    sb = torch.randint(0, B, (T, nodes), generator=g)
    is_split = sf >= 0
    rank = torch.cumsum(is_split.int(), 1) - is_split.int()
    cb = torch.where(is_split, 2 * rank, torch.full_like(rank, -1))
    split = rdf_ops.LevelSplits(sf, sb, None, torch.zeros(T, nodes, S), torch.zeros(T, nodes))
    no_c = node_of.clone()
    v_cpu = rdf_ops._route(data, no_c, nodes, split, cb, B)
    no_g = node_of.to(cuda)
    split_g = rdf_ops.LevelSplits(sf.to(cuda), sb.to(cuda), None, split.totals.to(cuda),
                                  split.gain.to(cuda))
    v_gpu = rdf_ops._route(gd, no_g, nodes, split_g, cb.to(cuda), B)
    assert torch.equal(v_gpu.cpu(), v_cpu)
    assert torch.equal(no_g.cpu(), no_c)
    # all-trees-per-row route (no visit counters) moves rows identically, and the counting
    # sort's visit counts (weight-0 rows included) equal the routing tallies
    no_r = node_of.to(cuda)
    assert rdf_ops._route(gd, no_r, nodes, split_g, cb.to(cuda), B, count_visits=False) is None
    assert torch.equal(no_r.cpu(), no_c)
    assert groups.visits is not None
    assert np.array_equal(groups.visits, v_cpu.numpy())


def test_csv_block_fast_path_matches_general_parse():
    """parse_csv_block (pandas C parser) returns exactly what parse_input_line +
    parse_examples return, declines blocks it cannot take (quotes, JSON arrays, unknown
    categories), and keeps an empty target as NaN."""
    from oryx_amd.models.rdf.batch import parse_csv_block
    from oryx_amd.utils import text
    schema = InputSchema(cfg.overlay_on({
        "oryx.input-schema.feature-names": '["a","b","c","t"]',
        "oryx.input-schema.categorical-features": '["b","t"]',
        "oryx.input-schema.target-feature": '"t"'}, cfg.get_default()))
    enc = CategoricalValueEncodings({1: ["x", "y"], 3: ["no", "yes"]})
    lines = ["1.5,x,-2,yes", "0.25,y,3e2,no", "7,x,0,", "-1,y,1.125,yes"]
    got = parse_csv_block(lines, schema, enc)
    want = parse_examples([text.parse_input_line(v) for v in lines], schema, enc,
                          require_target=False)
    assert got is not None
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    assert np.isnan(got[1][2])
    assert parse_csv_block(['1,"x",2,yes'], schema, enc) is None
    assert parse_csv_block(['[1,"x",2,"yes"]'], schema, enc) is None
    assert parse_csv_block(["1,z,2,yes"], schema, enc) is None


def test_regression_split_with_large_target_offset():
    """Targets 1e4 + N(0,1) with a step of 1 at x0 = 0.3: the root split must be the one a
    float64 host search over the same bins picks (no E[y^2] - mean^2 cancellation)."""
    g = np.random.default_rng(11)
    n = 20000
    X = g.uniform(-1, 1, (n, 3))
    y = 1e4 + g.standard_normal(n) + (X[:, 0] > 0.3) * 1.0
    data = rdf_ops.bin_features(X, [False] * 3, [0] * 3, 32, torch.device("cpu"))
    f = rdf_ops.train_forest(data, torch.from_numpy(y), 0, 1, 1, "variance", seed=1)
    root = f.roots[0]
    # brute-force float64 variance-reduction search over the bins
    Xb = data.Xb.numpy().astype(np.int64)
    best = (-np.inf, None, None)
    tot_var = y.var() * n
    for j in range(3):
        for b in range(data.B - 1):
            left = Xb[:, j] <= b
            nl = left.sum()
            if nl == 0 or nl == n:
                continue
            gain = tot_var - (y[left].var() * nl + y[~left].var() * (n - nl))
            if gain > best[0]:
                best = (gain, j, b)
    assert (root.feature, root.bin) == (best[1], best[2])
    # leaf statistics are reported un-centred
    assert abs(root.stats[1] / root.stats[0] - y.mean()) < 1e-6


def _random_level(T, N, Fs, B, S, P, cls, seed, rows=300):
    """Level histograms of random rows (float weights, so no exact gain ties): every feature
    slot of a node bins the same rows, so all slots share the node totals."""
    g = torch.Generator().manual_seed(seed)
    hist = torch.zeros((T, N, Fs, B, S), dtype=torch.float64)
    for t in range(T):
        for nd in range(N):
            w = torch.rand(rows, generator=g, dtype=torch.float64) * 2
            if cls:
                lab = torch.randint(0, S, (rows,), generator=g)
                stat = torch.zeros((rows, S), dtype=torch.float64)
                stat[torch.arange(rows), lab] = w
            else:
                yv = torch.randn(rows, generator=g, dtype=torch.float64) + \
                    torch.linspace(-1, 1, rows, dtype=torch.float64)
                stat = torch.stack([w, w * yv, w * yv * yv], 1)
            for j in range(Fs):
                b = torch.randint(0, B, (rows,), generator=g)
                hist[t, nd, j].index_add_(0, b, stat)
    feats = torch.stack([torch.randperm(P, generator=g)[:Fs] for _ in range(T * N)]) \
        .view(T, N, Fs).int()
    return hist.float(), feats


@pytest.mark.gpu
@pytest.mark.parametrize("cls,kind", [(True, "gini"), (True, "entropy"), (False, "variance")])
@pytest.mark.parametrize("with_cat", [False, True])
def test_split_kernel_matches_tensor_search(cuda, cls, kind, with_cat):
    """rdf_best_split (one wave per node, fp64) against the tensor-op split search."""
    T, N, Fs, B, S, P = 3, 9, 6, 11, 3, 10
    hist, feats = _random_level(T, N, Fs, B, S, P, cls, seed=7 + int(with_cat))
    cat = [with_cat and (f % 3 == 0) for f in range(P)]
    data = rdf_ops.BinnedData(torch.zeros((1, P), dtype=torch.uint8, device=cuda), [B] * P,
                              [None] * P, cat, B)
    # the reference search on the same fp32 statistics, evaluated in fp64
    ref = rdf_ops._choose_splits(hist.double().to(cuda), feats.to(cuda), data, kind, False)
    got = rdf_ops._choose_splits_kernel(hist.to(cuda), feats.to(cuda), data, kind, False)
    assert torch.equal(got.feat.cpu(), ref.feat.cpu())
    assert torch.equal(got.bin.cpu(), ref.bin.cpu())
    np.testing.assert_allclose(got.totals.cpu().numpy(), ref.totals.double().cpu().numpy())
    if with_cat:
        assert torch.equal(got.cat_left.cpu(), ref.cat_left.cpu())
    leaf = rdf_ops._choose_splits_kernel(hist.to(cuda), feats.to(cuda), data, kind, True)
    assert (leaf.feat == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("Fs,B", [(6, 32), (1, 32), (5, 17), (7, 100)])
def test_split_kernel_lane_chunks_past_the_last_bin(cuda, Fs, B):
    """Shapes whose per-feature lane chunks start past the last split position ((64 // Fs - 1)
    * ceil((B - 1) / (64 // Fs)) > B - 1: B = 32, Fs = 6 is the world-2 RDF test's level) --
    the chunk start is clamped, so no lane reads bins of the next feature (or past the end of
    the histogram), and the search still matches the tensor search.  A non-finite histogram
    entry sets the error flag and turns its node into a leaf."""
    T, N, S, P = 2, 3, 2, 8
    hist, feats = _random_level(T, N, Fs, B, S, P, True, seed=B + Fs)
    data = rdf_ops.BinnedData(torch.zeros((1, P), dtype=torch.uint8, device=cuda), [B] * P,
                              [None] * P, [False] * P, B)
    ref = rdf_ops._choose_splits(hist.double().to(cuda), feats.to(cuda), data, "gini", False)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    got = rdf_ops._choose_splits_kernel(hist.to(cuda), feats.to(cuda), data, "gini", False,
                                        err=err)
    assert int(err.item()) == 0
    assert torch.equal(got.feat.cpu(), ref.feat.cpu())
    assert torch.equal(got.bin.cpu(), ref.bin.cpu())
    bad = hist.clone()
    bad[1, 2, Fs - 1, B - 1, 1] = float("nan")
    got = rdf_ops._choose_splits_kernel(bad.to(cuda), feats.to(cuda), data, "gini", False,
                                        err=err)
    assert int(err.item()) == 1
    assert int(got.feat[1, 2]) == -1
    with pytest.raises(RuntimeError, match="non-finite"):
        rdf_ops._check_split_err(err, 3, type("C", (), {"rank": 0, "is_distributed": False}))
    assert int(err.item()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("classification", [True, False])
def test_device_level_loop_matches_host_loop(cuda, classification, monkeypatch):
    """The sync-free level loop (device pieces, split kernel, pipelined host tree build)
    grows the same single full-feature tree as the host-driven loop."""
    X, y = _numeric_data(30000, seed=6)
    yr = X[:, 0] * 2 - X[:, 2] + 0.1 * X[:, 1]
    data = rdf_ops.bin_features(X, [False] * 4, [0] * 4, 32, cuda, seed=2)
    tgt = torch.from_numpy(y if classification else yr)
    kind = "entropy" if classification else "variance"
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(rdf_ops, "_DEVICE_LOOP", flag)
        out[flag] = rdf_ops.train_forest(data, tgt, 2 if classification else 0, 1, 6, kind,
                                         seed=3)

    def walk(nd):
        yield (nd.id, nd.feature, nd.bin, nd.count)
        if nd.feature >= 0:
            yield from walk(nd.left)
            yield from walk(nd.right)
    assert list(walk(out[False].roots[0])) == list(walk(out[True].roots[0]))
    np.testing.assert_allclose(out[False].predictor_counts, out[True].predictor_counts)
    # a bootstrapped multi-tree forest through the device loop: every tree has a root split
    monkeypatch.setattr(rdf_ops, "_DEVICE_LOOP", True)
    f = rdf_ops.train_forest(data, tgt, 2 if classification else 0, 6, 5, kind, seed=4)
    assert all(r.feature >= 0 and r.count == 30000 for r in f.roots)


@pytest.mark.gpu
def test_device_poisson_bootstrap_weights(cuda):
    """rdf_poisson_weights: Poisson(1) counts (mean 1, variance 1, P(0) = 1/e), deterministic
    per seed, different across seeds, any length (tail handling)."""
    from oryx_amd import native
    lib = native.require_kernels()
    out = {}
    for seed, total in ((5, 4_000_003), (5, 4_000_003), (6, 4_000_003)):
        w = torch.empty(total, dtype=torch.uint8, device=cuda)
        native.check(lib.oryx_rdf_poisson_weights(seed, total, w.data_ptr(),
                                                  native.stream_ptr(cuda)), "poisson")
        out.setdefault(seed, []).append(w.cpu())
    a = out[5][0].double()
    assert abs(a.mean().item() - 1.0) < 3e-3 and abs(a.var().item() - 1.0) < 5e-3
    assert abs((a == 0).double().mean().item() - np.exp(-1.0)) < 2e-3
    assert abs((a == 2).double().mean().item() - np.exp(-1.0) / 2) < 2e-3
    assert torch.equal(out[5][0], out[5][1])
    assert not torch.equal(out[5][0], out[6][0])
