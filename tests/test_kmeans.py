"""k-means app tests: ports of the reference's KMeansEvalIT / KMeansPMMLUtilsTest /
ClusterInfoTest / KMeansUtilsTest / kmeans serving tests (T[mllib]/kmeans, T[app-common]/kmeans,
T[serving-app]/kmeans) with their golden values, plus trainer, speed and distributed checks."""

import math
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oryx_amd.api import Dataset, KeyMessage
from oryx_amd.models import app_pmml
from oryx_amd.models.kmeans import evaluation as ev
from oryx_amd.models.kmeans.batch import KMeansUpdate
from oryx_amd.models.kmeans.common import (ClusterInfo, closest_cluster, check_unique_ids,
                                           clustering_model_pmml, features_from_tokens,
                                           parse_feature_matrix, read_clusters,
                                           validate_pmml_vs_schema)
from oryx_amd.models.kmeans.serving import KMeansServingModel, KMeansServingModelManager
from oryx_amd.models.kmeans.speed import KMeansSpeedModelManager
from oryx_amd.models.schema import CategoricalValueEncodings, InputSchema
from oryx_amd.ops import kmeans as km
from oryx_amd.parallel import dist
from oryx_amd.transport.producer import MockTopicProducer
from oryx_amd.utils import config as cfg
from oryx_amd.utils import pmml as pm

from .serving_harness import Client

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _conf(**kv):
    return cfg.overlay_on({k.replace("__", "."): v for k, v in kv.items()}, cfg.get_default())


def _schema(**kv):
    return InputSchema(_conf(**kv))


def dummy_pmml():
    """KMeansPMMLUtilsTest.buildDummyClusteringModel: x,y; clusters (1,0)x1, (2,-1)x2, (-1,0)x3."""
    schema = _schema(**{"oryx__input-schema__feature-names": '["x","y"]',
                        "oryx__input-schema__categorical-features": "[]"})
    return clustering_model_pmml(schema, np.array([[1.0, 0.0], [2.0, -1.0], [-1.0, 0.0]]),
                                 [1, 2, 3])


EVAL_POINTS = np.array([[1.0, 0.0], [2.0, -2.0], [2.0, 0.0], [-2.0, 0.0], [-0.5, -1.0],
                        [-0.5, 1.0]])


# ---------------------------------------------------------------- schema

def test_schema_num_features_and_predictors():
    s = _schema(**{"oryx__input-schema__num-features": 4,
                   "oryx__input-schema__categorical-features": "[]",
                   "oryx__input-schema__ignored-features": "[0,2]"})
    assert s.get_feature_names() == ["0", "1", "2", "3"]
    assert s.get_num_predictors() == 2
    assert not s.is_active(0) and s.is_active(1) and s.is_numeric("3")
    assert s.feature_to_predictor_index(3) == 1
    assert s.predictor_to_feature_index(0) == 1
    with pytest.raises(ValueError):
        s.feature_to_predictor_index(0)


def test_schema_target_and_categorical():
    s = _schema(**{"oryx__input-schema__feature-names": '["a","b","c","d"]',
                   "oryx__input-schema__id-features": '["a"]',
                   "oryx__input-schema__numeric-features": '["b"]',
                   "oryx__input-schema__target-feature": "d"})
    assert s.is_id("a") and s.is_categorical("c") and s.is_categorical("d")
    assert s.has_target() and s.get_target_feature_index() == 3 and s.is_classification()
    assert s.get_num_predictors() == 2
    assert s.predictor_feature_indices == [1, 2]


def test_schema_errors():
    with pytest.raises(ValueError):
        _schema()   # neither feature-names nor num-features
    with pytest.raises(ValueError):
        _schema(**{"oryx__input-schema__num-features": 2})   # no numeric/categorical set
    with pytest.raises(ValueError):
        _schema(**{"oryx__input-schema__feature-names": '["a","a"]',
                   "oryx__input-schema__categorical-features": "[]"})


def test_categorical_encodings_and_dictionary():
    enc = CategoricalValueEncodings({1: ["x", "y", "z"]})
    assert enc.get_value_encoding_map(1) == {"x": 0, "y": 1, "z": 2}
    assert enc.get_encoding_value_map(1)[2] == "z"
    assert enc.get_value_count(1) == 3 and enc.get_category_counts() == {1: 3}
    s = _schema(**{"oryx__input-schema__feature-names": '["n","c"]',
                   "oryx__input-schema__categorical-features": '["c"]'})
    dd = app_pmml.build_data_dictionary(s, enc)
    back = app_pmml.build_categorical_value_encodings(dd)
    assert back.get_value_encoding_map(1) == enc.get_value_encoding_map(1)
    ms = app_pmml.build_mining_schema(s, [0.25, 0.75])
    fields = ms.findall(pm.q("MiningField"))
    assert [f.get("importance") for f in fields] == ["0.25", "0.75"]


# ---------------------------------------------------------------- common

def test_cluster_info_update():
    info = ClusterInfo(0, [-1.0, 2.0], 2)
    assert repr(info) == "0 [-1.0, 2.0] 2"
    info.update([-1.0, -1.0], 1)
    assert repr(info) == "0 [-1.0, 1.0] 3"
    info.update([0.0, 0.0], 3)
    assert repr(info) == "0 [-0.5, 0.5] 6"


def test_closest_cluster():
    clusters = [ClusterInfo(2, [1.0, 2.0], 1), ClusterInfo(4, [0.0, -2.0], 1),
                ClusterInfo(1, [3.0, 1.0], 1)]
    c, d = closest_cluster(clusters, [0.0, -2.0])
    assert c.id == 4 and d == 0.0
    c, d = closest_cluster(clusters, [6.0, 5.0])
    assert c.id == 1 and d == 5.0
    with pytest.raises(ValueError):
        closest_cluster([], [1.0])


def test_features_from_tokens_and_matrix():
    s = _schema(**{"oryx__input-schema__num-features": 4,
                   "oryx__input-schema__categorical-features": "[]",
                   "oryx__input-schema__ignored-features": "[0,2]"})
    assert features_from_tokens(["1.0", "2.0", "0.0", "-3.5"], s).tolist() == [2.0, -3.5]
    m = parse_feature_matrix(["1,2,3,4", "[5,6,7,8]", '"9",10,11,12'], s)
    assert m.tolist() == [[2.0, 4.0], [6.0, 8.0], [10.0, 12.0]]


def test_unique_ids():
    check_unique_ids([ClusterInfo(2, [1.0], 1), ClusterInfo(4, [0.0], 1)])
    with pytest.raises(ValueError):
        check_unique_ids([ClusterInfo(2, [1.0], 1), ClusterInfo(2, [0.0], 1)])


def test_pmml_round_trip_and_validate():
    doc = dummy_pmml()
    back = pm.from_string(pm.to_string(doc))
    s = _schema(**{"oryx__input-schema__feature-names": '["x","y"]',
                   "oryx__input-schema__num-features": 2,
                   "oryx__input-schema__categorical-features": "[]"})
    validate_pmml_vs_schema(back, s)
    clusters = read_clusters(back)
    assert len(clusters) == 3 and len(clusters[0].center) == 2 and clusters[1].count == 2
    model = back.models()[0]
    assert model.get("modelClass") == "centerBased"
    assert model.find(pm.q("ComparisonMeasure")).get("kind") == "distance"
    bad = _schema(**{"oryx__input-schema__feature-names": '["x","z"]',
                     "oryx__input-schema__categorical-features": "[]"})
    with pytest.raises(ValueError):
        validate_pmml_vs_schema(back, bad)


# ---------------------------------------------------------------- evaluation (KMeansEvalIT)

def test_eval_golden_values():
    clusters = read_clusters(dummy_pmml())
    dev = torch.device("cpu")
    assert ev.dunn_index(clusters, EVAL_POINTS, dev) == pytest.approx(1.3110480733464633,
                                                                       abs=1e-12)
    assert ev.davies_bouldin_index(clusters, EVAL_POINTS, dev) == pytest.approx(
        0.9702216688254247, abs=1e-12)
    assert ev.silhouette_coefficient(clusters, EVAL_POINTS, dev) == pytest.approx(
        0.30648167401009796, abs=1e-12)
    assert ev.sum_squared_error(clusters, EVAL_POINTS, dev) == pytest.approx(5.5, abs=1e-12)
    assert len(ev.fetch_sample_data(EVAL_POINTS)) == 6


def test_silhouette_helper():
    assert ev.silhouette_of(-0.8, 0.2) == 5.0
    assert ev.silhouette_of(0.8, -0.2) == -1.25
    assert ev.silhouette_of(1.5, 1.5) == 0.0
    assert ev.silhouette_of(1.5, float("inf")) == 1.0
    assert ev.silhouette_of(float("inf"), 1.5) == -1.0


def test_silhouette_tiled_matches_direct():
    g = np.random.default_rng(3)
    pts = np.concatenate([g.normal(c, 0.5, (150, 3)) for c in (-3, 0, 3)])
    clusters = [ClusterInfo(i, [c] * 3, 1) for i, c in enumerate((-3.0, 0.0, 3.0))]
    fast = ev.silhouette_coefficient(clusters, pts, torch.device("cpu"))
    # direct O(n^2) reference
    assign = np.argmin(((pts[:, None] - np.array([[c] * 3 for c in (-3, 0, 3)])[None]) ** 2)
                       .sum(2), 1)
    d = np.sqrt(((pts[:, None] - pts[None]) ** 2).sum(2))
    tot = 0.0
    for p in range(len(pts)):
        own = assign == assign[p]
        a = d[p, own].sum() / (own.sum() - 1)
        b = min(d[p, assign == o].mean() for o in range(3) if o != assign[p])
        tot += ev.silhouette_of(a, b)
    assert fast == pytest.approx(tot / len(pts), abs=1e-9)


# ---------------------------------------------------------------- trainer

def _blobs(n_per=400, seed=0):
    g = np.random.default_rng(seed)
    cents = np.array([[0, 0, 0, 0], [8, 8, 0, 0], [-8, 8, 3, 0], [0, -9, -3, 4]], float)
    pts = np.concatenate([g.normal(c, 0.6, (n_per, 4)) for c in cents])
    return pts, cents


def test_kmeans_train_recovers_blobs():
    pts, cents = _blobs()
    res = km.kmeans_train(torch.from_numpy(pts).float(), 4, 30, runs=2, seed=1)
    got = res.centers.numpy()
    for c in cents:
        assert np.min(np.linalg.norm(got - c, axis=1)) < 0.3
    assert res.counts.sum().item() == len(pts) and (res.counts > 0).all()


def test_kmeans_random_init_is_lloyd_fixed_point():
    pts, _ = _blobs()
    x = torch.from_numpy(pts).float()
    res = km.kmeans_train(x, 4, 50, runs=3, init="random", seed=1)
    idx, d2 = km.assign(x, res.centers, exact=True)
    sums, counts, _ = km.accumulate(x, idx, 4)
    assert torch.allclose(sums / counts[:, None], res.centers, atol=1e-3)
    assert res.cost == pytest.approx(float(d2.double().sum()), rel=1e-6)


def test_kmeans_reseeds_empty_clusters():
    # 3 distinct points, k=3 but random init may duplicate: every cluster must end non-empty
    x = torch.tensor([[0.0, 0.0]] * 5 + [[10.0, 0.0]] * 5 + [[0.0, 10.0]] * 5)
    res = km.kmeans_train(x, 3, 10, runs=1, init="random", seed=2)
    assert sorted(res.counts.tolist()) == [5, 5, 5]


def test_kmeans_keep_empty_cluster_like_mllib():
    """reseed_empty=False (oryx.kmeans.reseed-empty-clusters = false): an empty cluster keeps
    its center (MLlib's Lloyd loop) and survives with size 0; the default moves it to the
    farthest point, so every cluster ends non-empty."""
    x = torch.tensor([[0.0, 0.0]] * 6 + [[10.0, 0.0]] * 6 + [[0.0, 30.0]])
    # seed 0: the random init draws two centers from one of the dense points
    kept = km.kmeans_train(x, 3, 10, runs=1, init="random", seed=0, reseed_empty=False)
    reseeded = km.kmeans_train(x, 3, 10, runs=1, init="random", seed=0, reseed_empty=True)
    assert sorted(kept.counts.tolist()) == [0, 6, 7]
    empty = int((kept.counts == 0).nonzero()[0])
    assert kept.centers[empty].tolist() in ([0.0, 0.0], [10.0, 0.0])   # not moved
    assert sorted(reseeded.counts.tolist()) == [1, 6, 6]


def _update_config(tmp_path, strategy="SILHOUETTE"):
    return _conf(**{"oryx__input-schema__num-features": 4,
                    "oryx__input-schema__categorical-features": "[]",
                    "oryx__kmeans__hyperparams__k": 4,
                    "oryx__kmeans__iterations": 10,
                    "oryx__kmeans__runs": 1,
                    "oryx__kmeans__evaluation-strategy": strategy,
                    "oryx__ml__eval__test-fraction": 0.2,
                    "oryx__ml__eval__candidates": 2,
                    "oryx__ml__eval__parallelism": 1})


@pytest.mark.parametrize("strategy", ["SILHOUETTE", "SSE", "DUNN", "DAVIES_BOULDIN"])
def test_kmeans_update_publishes_model(tmp_path, strategy):
    pts, _ = _blobs(n_per=100)
    lines = [",".join(repr(float(v)) for v in p) for p in pts]
    upd = KMeansUpdate(_update_config(tmp_path, strategy))
    MockTopicProducer.clear()
    prod = MockTopicProducer()
    upd.run_update(None, 1000, Dataset([(None, l) for l in lines]), None,
                   str(tmp_path / "model"), prod)
    msgs = MockTopicProducer.get_key_messages()
    assert len(msgs) == 1 and msgs[0][0] == "MODEL"
    doc = pm.from_string(msgs[0][1])
    model = doc.models()[0]
    assert model.get("numberOfClusters") == "4"
    assert len(model.findall(pm.q("ClusteringField"))) == 4
    clusters = read_clusters(doc)
    assert len(clusters) == 4 and all(c.count > 0 for c in clusters)
    assert len(clusters[0].center) == 4


def test_kmeans_update_rejects_categorical():
    c = _conf(**{"oryx__input-schema__num-features": 2,
                 "oryx__input-schema__categorical-features": '["1"]'})
    with pytest.raises(ValueError):
        KMeansUpdate(c)


# ---------------------------------------------------------------- speed

def test_speed_manager_running_mean():
    conf = _conf(**{"oryx__input-schema__feature-names": '["x","y"]',
                    "oryx__input-schema__categorical-features": "[]"})
    mgr = KMeansSpeedModelManager(conf)
    assert mgr.build_updates(Dataset([(None, "1,1")])) == []
    mgr.consume(iter([KeyMessage("MODEL", pm.to_string(dummy_pmml())),
                      KeyMessage("UP", "ignored")]))
    ups = mgr.build_updates(Dataset([(None, "1,1"), (None, "3,-1"), (None, "-3,0")]))
    import json
    got = [json.loads(u) for u in ups]
    # (1,1) -> cluster 0 (1,0) count 1: mean (1,1) -> center (1,0.5), count 2
    # (3,-1) -> cluster 1 (2,-1) count 2 -> center (2+1/3, -1), count 3
    # (-3,0) -> cluster 2 (-1,0) count 3 -> center (-1.5, 0), count 4
    assert got[0] == [0, [1.0, 0.5], 2]
    assert got[1][0] == 1 and got[1][2] == 3
    assert got[1][1] == pytest.approx([2 + 1 / 3, -1.0])
    assert got[2] == [2, [-1.5, 0.0], 4]


@pytest.mark.gpu
def test_speed_manager_device_path_matches_host(cuda):
    """The GPU speed path (native parse to a device fp64 matrix, exact fp64 nearest-center
    kernel, index_add sums, vectorised running means, native message formatting) gives the
    golden running-mean example exactly, and on 20k random points over 300 clusters x 64
    dims the same touched clusters, counts and centers (to summation order) as the host
    path; the model's clusters end up updated alike."""
    import json
    from oryx_amd.models.kmeans.speed import KMeansSpeedModel
    conf = _conf(**{"oryx__input-schema__feature-names": '["x","y"]',
                    "oryx__input-schema__categorical-features": "[]"})
    mgr = KMeansSpeedModelManager(conf)
    mgr.consume(iter([KeyMessage("MODEL", pm.to_string(dummy_pmml()))]))
    assert mgr.model.clusters.device.type == "cuda"
    ups = mgr.build_updates(Dataset([(None, "1,1"), (None, "3,-1"), (None, "-3,0")]))
    got = [json.loads(u) for u in ups]
    assert got[0] == [0, [1.0, 0.5], 2] and got[2] == [2, [-1.5, 0.0], 4]
    assert got[1][0] == 1 and got[1][2] == 3
    assert got[1][1] == pytest.approx([2 + 1 / 3, -1.0])
    g = np.random.default_rng(3)
    k, d, n = 300, 64, 20000
    names = "[%s]" % ",".join('"f%d"' % j for j in range(d))
    conf = _conf(**{"oryx__input-schema__feature-names": names,
                    "oryx__input-schema__categorical-features": "[]"})
    centers = g.standard_normal((k, d)) * 3
    batches = []
    for _ in range(3):
        pts = centers[g.integers(0, k, n)] + g.standard_normal((n, d))
        batches.append([",".join(repr(float(v)) for v in row) for row in pts])
    outs, models = [], []
    for device in (torch.device(cuda), None):
        m = KMeansSpeedModelManager(conf)
        m.model = KMeansSpeedModel([ClusterInfo(10 + j, centers[j], 1 + j % 7)
                                    for j in range(k)], device)
        if device is None:
            m.model.clusters.device = None
        # consecutive micro-batches: the device path updates its device centers / counts in
        # place after the first one
        outs.append([[json.loads(u) for u in m.build_updates(Dataset([(None, l) for l in b]))]
                     for b in batches])
        models.append(m.model.clusters)
    for dev, host in zip(*outs):
        assert [u[0] for u in dev] == [u[0] for u in host]
        assert [u[2] for u in dev] == [u[2] for u in host]
        np.testing.assert_allclose(np.array([u[1] for u in dev]),
                                   np.array([u[1] for u in host]), rtol=1e-11, atol=1e-11)
    # the in-place device state is the state a rebuild from the host clusters gives
    cs = models[0]
    c, ct, cnt = cs.device_state()
    np.testing.assert_array_equal(c.cpu().numpy(), cs.centers())
    np.testing.assert_array_equal(ct.cpu().numpy(), cs.centers().T)
    assert cnt.cpu().tolist() == [ci.count for ci in cs.clusters]
    np.testing.assert_allclose(cs.centers(), models[1].centers(), rtol=1e-11, atol=1e-11)


# ---------------------------------------------------------------- serving

def _test_model():
    s = _schema(**{"oryx__input-schema__num-features": 2,
                   "oryx__input-schema__categorical-features": "[]"})
    return KMeansServingModel([ClusterInfo(2, [1.0, 0.0], 1), ClusterInfo(3, [2.0, -1.0], 1),
                               ClusterInfo(4, [-1.0, 0.0], 1)], s)


def _client(read_only=False):
    return Client(["oryx_amd.models.kmeans.resources"], _test_model(), read_only=read_only)


def test_serving_assign():
    c = _client()
    assert int(c.get_text("/assign/1,0")) == 2
    assert int(c.get_text("/assign/10,-1.0")) == 3
    r = c.request("POST", "/assign", body="-1.5,0.5\n-1,0")
    assert r.status == 200 and r.body.decode() == "4\n4\n"
    assert c.status("GET", "/assign/1,0,3") == 400


def test_serving_distance_to_nearest():
    c = _client()
    assert float(c.get_text("/distanceToNearest/1,0")) == 0.0
    assert float(c.get_text("/distanceToNearest/10,-1.0")) == 8.0


def test_serving_add_and_read_only():
    data = "1.0,0.0,20.0\n1.0,-4.0,30.0\n0.0,0.0,40.0\n0.0,-4.0,50.0"
    c = _client()
    assert c.status("POST", "/add", body=data) == 204
    assert [m for _, m in MockTopicProducer.get_key_messages()] == data.split("\n")
    MockTopicProducer.clear()
    assert c.status("POST", "/add/1.0,0.0,20.0") == 204
    assert [m for _, m in MockTopicProducer.get_key_messages()] == ["1.0,0.0,20.0"]
    ro = _client(read_only=True)
    assert ro.status("POST", "/add", body=data) == 403


def test_serving_console_and_ready():
    c = _client()
    r = c.get("/index.html")
    assert r.status == 200 and b"<html" in r.body.lower()
    assert c.status("GET", "/ready") == 200


def test_serving_manager_consume():
    conf = _conf(**{"oryx__input-schema__feature-names": '["x","y"]',
                    "oryx__input-schema__categorical-features": "[]"})
    mgr = KMeansServingModelManager(conf)
    mgr.consume(iter([KeyMessage("UP", "[0,[1.0,1.0],5]")]))
    assert mgr.get_model() is None
    mgr.consume(iter([KeyMessage("MODEL", pm.to_string(dummy_pmml())),
                      KeyMessage("UP", "[1,[5.0,5.0],7]")]))
    m = mgr.get_model()
    assert m.get_num_clusters() == 3
    assert m.get_cluster(1).center.tolist() == [5.0, 5.0] and m.get_cluster(1).count == 7
    assert m.nearest_cluster_id(["4.5", "4"]) == 1
    assert m.nearest_cluster_ids([["4.5", "4"], ["-1", "0"]]) == [1, 2]


# ---------------------------------------------------------------- distributed (gloo)

def test_kmeans_distributed_gloo(tmp_path):
    """world 2 over gloo: each rank holds half the points; the centers recover the blobs."""
    script = tmp_path / "run.py"
    script.write_text(f"""
import sys, torch, numpy as np
sys.path.insert(0, {ROOT!r})
from oryx_amd.parallel import dist
from oryx_amd.ops import kmeans as km
from oryx_amd.parallel import dist
ctx = dist.init_from_env(device='cpu')
g = np.random.default_rng(0)
cents = np.array([[0, 0], [9, 9], [-9, 9]], float)
pts = np.concatenate([g.normal(c, 0.5, (300, 2)) for c in cents])
x = torch.from_numpy(pts[ctx.rank::ctx.world_size]).float()
res = km.kmeans_train(x, 3, 20, runs=1, seed=4, ctx=ctx)
if ctx.rank == 0:
    torch.save({{'c': res.centers, 'n': res.counts}}, sys.argv[1])
""")
    out = tmp_path / "w2.pt"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29633", str(script), str(out)]
    subprocess.run(cmd, check=True, env=env, timeout=180, capture_output=True)
    r = torch.load(out)
    got = r["c"].numpy()
    for c in ([0, 0], [9, 9], [-9, 9]):
        assert np.min(np.linalg.norm(got - np.array(c), axis=1)) < 0.3
    assert int(r["n"].sum()) == 900


# ---------------------------------------------------------------- GPU kernels

@pytest.mark.gpu
@pytest.mark.parametrize("d,k", [(2, 3), (20, 64), (64, 100), (100, 257), (256, 50), (256, 1000),
                                 (500, 130)])
def test_assign_kernel_bf16_matches_fp32_on_rounded_inputs(cuda, d, k):
    g = torch.Generator().manual_seed(d * 1000 + k)
    x = torch.randn(5000, d, generator=g)
    c = torch.randn(k, d, generator=g)
    idx, dist = km.assign(x.to(cuda), c.to(cuda), precision="bf16")
    # reference on the same bf16-rounded inputs, fp32 math
    xb, cb = x.bfloat16().float(), c.bfloat16().float()
    d2 = ((xb[:, None, :] - cb[None]) ** 2).sum(2)
    ref_v, ref_i = d2.min(1)
    got_i = idx.cpu()
    got_v = dist.cpu()
    # argmin agrees except within fp32-rounding near-ties
    chosen = d2.gather(1, got_i[:, None].long())[:, 0]
    assert torch.all(chosen <= ref_v + 1e-3 * (1 + ref_v))
    assert (got_i == ref_i).float().mean() > 0.995
    assert torch.allclose(got_v, ref_v, rtol=1e-3, atol=1e-3 * d)


def _fp64_d2(x, c):
    x, c = x.double(), c.double()
    return ((x[:, None, :] - c[None]) ** 2).sum(2)


@pytest.mark.gpu
@pytest.mark.parametrize("d,k", [(2, 3), (64, 100), (100, 257), (128, 64), (256, 50),
                                 (256, 1000), (500, 130)])
def test_assign_fp32_is_exact_argmin_on_true_data(cuda, d, k):
    """fp32 precision (certified kernel + fp32 rescore, or the exact scan for shapes without
    it) on UN-rounded fp32 data: the chosen center is an fp64 argmin up to the fp32 tie band
    (3e-5 relative), and all but a handful of points pick exactly the fp64 argmin."""
    g = torch.Generator().manual_seed(d * 7 + k)
    x = torch.randn(6000, d, generator=g)
    c = torch.randn(k, d, generator=g)
    idx, dist = km.assign(x.to(cuda), c.to(cuda), precision="fp32")
    d64 = _fp64_d2(x, c)
    ref_v, ref_i = d64.min(1)
    got_i = idx.cpu().long()
    chosen = d64.gather(1, got_i[:, None])[:, 0]
    assert torch.all(chosen <= ref_v * (1 + 3e-5) + 1e-9), (chosen - ref_v).max()
    assert (got_i == ref_i).float().mean() >= 0.999


@pytest.mark.gpu
@pytest.mark.parametrize("d", [64, 256])
def test_assign_fp32_resolves_bf16_near_ties(cuda, d):
    """Centers 3 apart in a cloud of radius ~16 (bf16 cannot separate them for most points):
    two-way ties (rescored top-2) and three-way ties (full rescan) still get the fp64 argmin,
    where the bf16 argmin is wrong for a measurable share of the points."""
    g = torch.Generator().manual_seed(d)
    base = torch.randn(d, generator=g) * 8
    cents = torch.stack([base + 0.02 * torch.randn(d, generator=g) for _ in range(3)] +
                        [torch.randn(d, generator=g) * 8 for _ in range(61)])
    x = base + torch.randn(20000, d, generator=g)
    d64 = _fp64_d2(x, cents)
    ref_v, ref_i = d64.min(1)
    from oryx_amd.ops import kmeans as kmo
    kmo.CERT_STATS.clear()
    idx, _ = km.assign(x.to(cuda), cents.to(cuda), precision="fp32")
    got_i = idx.cpu().long()
    chosen = d64.gather(1, got_i[:, None])[:, 0]
    assert torch.all(chosen <= ref_v * (1 + 3e-5) + 1e-9)
    st = kmo.CERT_STATS[torch.device(cuda)].cpu().tolist()
    assert st[0] + st[1] > 0, st          # the rescore kernel decided some points
    bidx, _ = km.assign(x.to(cuda), cents.to(cuda), precision="bf16")
    wrong_bf16 = (bidx.cpu().long() != ref_i).float().mean().item()
    assert (got_i == ref_i).float().mean().item() > 1 - 1e-3
    assert wrong_bf16 > 1e-3, wrong_bf16   # the data really defeats a plain bf16 argmin


@pytest.mark.gpu
def test_lloyd_sse_fp32_vs_bf16(cuda):
    """End-metric drift: SSE of fp32-certified Lloyd matches the fp64-checked CPU run; the bf16
    run's SSE is reported against it (within 0.5%)."""
    g = torch.Generator().manual_seed(5)
    true_c = torch.randn(12, 64, generator=g) * 3
    x = true_c[torch.randint(0, 12, (30000,), generator=g)] + torch.randn(30000, 64, generator=g)
    out = {}
    for prec, dev in (("fp32", cuda), ("bf16", cuda), ("fp32", "cpu")):
        res = km.kmeans_train(x.to(dev), 16, 15, runs=1, seed=3, init="random",
                              ctx=dist.DistContext(device=torch.device(dev)), precision=prec)
        out[(prec, str(dev))] = res.cost
    assert out[("fp32", str(cuda))] == pytest.approx(out[("fp32", "cpu")], rel=1e-5)
    assert out[("bf16", str(cuda))] == pytest.approx(out[("fp32", "cpu")], rel=5e-3)


@pytest.mark.gpu
def test_accumulate_kernel_matches_reference(cuda):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(20000, 37, generator=g)
    idx = torch.randint(0, 11, (20000,), generator=g)
    mind = torch.rand(20000, generator=g)
    sums, counts, stats = km.accumulate(x.to(cuda), idx.to(cuda), 11, mind.to(cuda))
    rs = torch.zeros(11, 37).index_add_(0, idx, x)
    rc = torch.bincount(idx, minlength=11)
    dd = mind.double().sqrt()
    assert torch.allclose(sums.cpu(), rs, atol=1e-3)
    assert torch.equal(counts.cpu(), rc)
    assert torch.allclose(stats[:, 0].cpu(), torch.zeros(11, dtype=torch.float64)
                          .index_add_(0, idx, dd), rtol=1e-9)


@pytest.mark.gpu
def test_kmeans_train_gpu(cuda):
    pts, cents = _blobs(n_per=2000)
    res = km.kmeans_train(torch.from_numpy(pts).float().to(cuda), 4, 30, runs=1, seed=1)
    got = res.centers.cpu().numpy()
    for c in cents:
        assert np.min(np.linalg.norm(got - c, axis=1)) < 0.3


@pytest.mark.gpu
def test_eval_metrics_gpu_match_cpu(cuda):
    pts, cents = _blobs(n_per=500)
    clusters = [ClusterInfo(i, c, 1) for i, c in enumerate(cents)]
    for fn in (ev.sum_squared_error, ev.dunn_index, ev.davies_bouldin_index):
        assert fn(clusters, pts, cuda) == pytest.approx(fn(clusters, pts, torch.device("cpu")),
                                                        rel=1e-9)
    # the silhouette's distances come from fp32 MFMA dot products, d^2 = |a|^2 + |b|^2 - 2 a.b
    # of the centred sample: each carries ~eps32 (|a|^2 + |b|^2) of cancellation error (the
    # difference form's ~eps32 d^2), so the mean agrees with fp64 to ~1e-8, not 1e-9
    assert ev.silhouette_coefficient(clusters, pts, cuda) == pytest.approx(
        ev.silhouette_coefficient(clusters, pts, torch.device("cpu")), rel=2e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("sorted_path", [True, False])
@pytest.mark.parametrize("n,d,k", [(50000, 256, 1000), (30000, 37, 300), (20000, 16, 9000),
                                   (70000, 300, 5)])
def test_accumulate_kernel_lds_slices(cuda, n, d, k, sorted_path, monkeypatch):
    """Sort-based segmented sums (clusters split into 2048-row pieces; d > 256 columns), the
    LDS column-slice path (k=1000 d=256: 8 slices; d < slice width) and the L2-atomic
    fallback (k=9000 does not fit LDS) against index_add."""
    monkeypatch.setattr(km, "_SORTED", sorted_path)
    g = torch.Generator().manual_seed(n + d + k)
    x = torch.randn(n, d, generator=g)
    idx = torch.randint(0, k, (n,), generator=g)
    mind = torch.rand(n, generator=g)
    sums, counts, stats = km.accumulate(x.to(cuda), idx.to(cuda).int(), k, mind.to(cuda))
    rs = torch.zeros(k, d, dtype=torch.float64).index_add_(0, idx, x.double())
    assert torch.allclose(sums.cpu().double(), rs, atol=1e-3)
    assert torch.equal(counts.cpu(), torch.bincount(idx, minlength=k))
    dd = mind.double().sqrt()
    ref = torch.zeros(k, dtype=torch.float64).index_add_(0, idx, dd)
    assert torch.allclose(stats[:, 0].cpu(), ref, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_lloyd_step_matches_cpu(cuda):
    pts, _ = _blobs(n_per=3000)
    x = torch.from_numpy(pts).float()
    c0 = x[torch.randperm(x.shape[0], generator=torch.Generator().manual_seed(3))[:6]].clone()
    ctx = dist.DistContext(device=cuda)
    new_g, counts_g, _, _ = km.lloyd_step(km.PointSet(x.to(cuda)), c0.to(cuda), ctx,
                                          precision="bf16")
    new_c, counts_c, _, _ = km.lloyd_step(km.PointSet(x), c0, dist.DistContext())
    assert int(counts_g.sum()) == x.shape[0]
    # bf16 distances may flip near-tie assignments (several initial centers share a blob)
    assert (counts_g.cpu() - counts_c).abs().sum() <= 0.005 * x.shape[0]
    # fp32 precision: the same counts as the fp32 CPU step up to fp32 near-ties
    _, counts_f, _, _ = km.lloyd_step(km.PointSet(x.to(cuda)), c0.to(cuda), ctx,
                                      precision="fp32")
    assert (counts_f.cpu() - counts_c).abs().sum() <= 2
    # given the kernel's own assignment the update is exact: centers = per-cluster means
    idx, _ = km.assign(km.PointSet(x.to(cuda)), c0.to(cuda), precision="bf16")
    idx = idx.long().cpu()
    ref = torch.zeros(6, x.shape[1], dtype=torch.float64).index_add_(0, idx, x.double())
    ref /= torch.bincount(idx, minlength=6).clamp_min(1)[:, None]
    assert torch.allclose(new_g.cpu().double(), ref, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k", [(1, 1), (1000, 3), (300_001, 1000), (2_000_003, 5121)])
def test_counting_sort_kernel_groups_every_row(cuda, n, k):
    """oryx_counting_sort (used by the k-means sorted accumulate and the RDF level grouping)
    against torch: counts equal bincount, every row appears once, each group holds its key."""
    from oryx_amd import native
    lib = native.require_kernels()
    g = torch.Generator().manual_seed(n + k)
    keys = (k * torch.rand(n, generator=g).pow(2)).to(torch.int32).clamp_(0, k - 1)
    keys_d = keys.to(cuda)
    perm = torch.empty(n, dtype=torch.int32, device=cuda)
    counts = torch.empty(k, dtype=torch.int64, device=cuda)
    ws = torch.empty(int(lib.oryx_kmeans_sorted_ws_bytes(n, k)), dtype=torch.uint8, device=cuda)
    native.check(lib.oryx_counting_sort(keys_d.data_ptr(), n, k, perm.data_ptr(),
                                        counts.data_ptr(), ws.data_ptr(),
                                        native.stream_ptr(cuda)), "oryx_counting_sort")
    torch.cuda.synchronize()
    ref_counts = torch.bincount(keys.long(), minlength=k)
    assert torch.equal(counts.cpu(), ref_counts)
    p = perm.cpu().long()
    assert torch.equal(torch.sort(p).values, torch.arange(n))
    grouped = keys.long()[p]
    assert torch.equal(grouped, torch.repeat_interleave(torch.arange(k), ref_counts))


def test_vectorised_db_dunn_match_loops():
    """The K x K matrix forms of Davies-Bouldin / Dunn equal the reference's double loops."""
    pts, cents = _blobs(n_per=300)
    g = np.random.default_rng(4)
    clusters = [ClusterInfo(i, c + g.normal(0, 0.2, 4), 1) for i, c in enumerate(cents)]
    m = ev.fetch_cluster_metrics(clusters, pts, "cpu")
    vals = []
    for ci in clusters:
        si = m[ci.id].get_mean_dist()
        vals.append(max((si + m[cj.id].get_mean_dist()) / np.linalg.norm(ci.center - cj.center)
                        for cj in clusters if cj.id != ci.id))
    assert ev.davies_bouldin_index(clusters, pts, "cpu") == pytest.approx(np.mean(vals), 1e-12)
    inter = min(np.linalg.norm(a.center - b.center) for a in clusters for b in clusters
                if a.id < b.id)
    intra = max(x.get_mean_dist() for x in m.values())
    assert ev.dunn_index(clusters, pts, "cpu") == pytest.approx(inter / intra, 1e-12)


EVAL_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, ROOT)
import numpy as np
from oryx_amd.models.kmeans import evaluation as ev
from oryx_amd.models.kmeans.common import ClusterInfo
from oryx_amd.parallel import dist
from oryx_amd.utils import rng
ctx = dist.init_from_env(device="cpu")
g = np.random.default_rng(0)
cents = np.array([[0, 0, 0], [6, 6, 0], [-6, 6, 2]], float)
pts = np.concatenate([g.normal(c, 0.7, (400, 3)) for c in cents])
clusters = [ClusterInfo(i, c, 1) for i, c in enumerate(cents)]
mine = pts[ctx.rank::ctx.world_size]
out = {}
for s in ("SSE", "DAVIES_BOULDIN", "DUNN"):
    out[s] = ev.evaluate_sharded(s, clusters, mine, ctx, device="cpu")
    out[s + "_1"] = ev.evaluate(s, clusters, pts, device="cpu")
with rng.shared_seed_scope(5):
    out["SIL"] = ev.evaluate_sharded("SILHOUETTE", clusters, mine, ctx, device="cpu")
out["SIL_1"] = ev.evaluate("SILHOUETTE", clusters, pts, device="cpu")
with open(os.path.join(sys.argv[1], "r%d.json" % ctx.rank), "w") as f:
    json.dump(out, f)
"""


def test_sharded_eval_metrics_equal_single_process(tmp_path):
    """World-2 (gloo) cluster metrics over point shards == world-1 over all points."""
    import json, os, subprocess, sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "ev.py"
    script.write_text(EVAL_SCRIPT.replace("ROOT", repr(root)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29647", str(script), str(tmp_path)]
    r = subprocess.run(cmd, env=dict(os.environ, OMP_NUM_THREADS="1"), timeout=300,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    a = json.loads((tmp_path / "r0.json").read_text())
    b = json.loads((tmp_path / "r1.json").read_text())
    for s in ("SSE", "DAVIES_BOULDIN", "DUNN"):
        assert a[s] == pytest.approx(a[s + "_1"], rel=1e-12) and a[s] == b[s]
    # 1200 points < the 100k cap: the sample is everything on both sides
    assert a["SIL"] == pytest.approx(a["SIL_1"], rel=1e-9) and a["SIL"] == b["SIL"]


@pytest.mark.gpu
def test_silhouette_kernel_matches_host(cuda):
    """km_silhouette (sorted sample, streamed distances, running per-cluster sums) against the
    fp64 tensor path, on the golden points and on a wide sample with an empty cluster and a
    singleton cluster."""
    clusters = read_clusters(dummy_pmml())
    assert ev.silhouette_coefficient(clusters, EVAL_POINTS, cuda) == pytest.approx(
        0.30648167401009796, abs=1e-6)
    g = np.random.default_rng(8)
    cs = [g.normal(0, 4, 70) for _ in range(12)]
    pts = np.concatenate([g.normal(c, 1.0, (300, 70)) for c in cs[:10]] + [cs[10][None]])
    clusters = [ClusterInfo(i, c.tolist(), 1) for i, c in enumerate(cs)]
    host = ev.silhouette_coefficient(clusters, pts, torch.device("cpu"))
    dev = ev.silhouette_coefficient(clusters, pts, cuda)
    assert dev == pytest.approx(host, rel=1e-5)
    # many column ranges (300 clusters of skewed sizes, 20k points: 64 ranges at cluster
    # boundaries) and a dimension that is not a multiple of the 64-wide tiles
    cs = [g.normal(0, 6, 37) for _ in range(300)]
    sizes = np.minimum(g.zipf(1.6, 300), 800)
    pts = np.concatenate([g.normal(c, 1.0, (int(m), 37)) for c, m in zip(cs, sizes)])
    clusters = [ClusterInfo(i, c.tolist(), 1) for i, c in enumerate(cs)]
    host = ev.silhouette_coefficient(clusters, pts, torch.device("cpu"))
    dev = ev.silhouette_coefficient(clusters, pts, cuda)
    assert dev == pytest.approx(host, rel=1e-5)


@pytest.mark.gpu
def test_kmeanspp_native_draws_match_torch_path(cuda):
    """The k-means++ kernels (fixed-order fp64 scan + inverse-CDF draw, D^2 update) choose the
    same candidates as the torch path on the CPU from the same host uniforms."""
    g = torch.Generator().manual_seed(5)
    cands = torch.randn(3000, 24, generator=g)
    w = torch.randint(1, 50, (3000,), generator=g).double()
    out = []
    for dev in ("cpu", cuda):
        gen = torch.Generator().manual_seed(11)
        out.append(km._kmeanspp_weighted(cands.to(dev), w, 150, gen).cpu())
    same = (out[0] == out[1]).all(1)
    # one rounding-level flip would change every later draw; demand a long identical prefix
    first_diff = int(torch.nonzero(~same)[0]) if not same.all() else len(same)
    assert first_diff >= 100, first_diff


@pytest.mark.parametrize("strategy", ["SSE", "DAVIES_BOULDIN"])
def test_kmeans_evaluate_reuses_parsed_training_points(tmp_path, strategy):
    """evaluate() scores train + test points: taking the rows build_model parsed plus a parse
    of the test lines gives the same value as parsing the joined text again."""
    from oryx_amd.textlines import TextLines
    pts, _ = _blobs(n_per=60)
    lines = [",".join(repr(float(v)) for v in p) for p in pts]
    train, test = TextLines.from_strings(lines[:150]), TextLines.from_strings(lines[150:])
    upd = KMeansUpdate(_update_config(tmp_path, strategy))
    model = upd.build_model(None, train, [4], None)
    cached = upd.evaluate(None, model, None, test, train)
    upd._train_points = None                  # forces the joined parse
    fresh = upd.evaluate(None, model, None, test, train)
    assert cached == pytest.approx(fresh, rel=1e-9, abs=1e-12)


def test_kmeans_update_evaluation_is_double_precision(tmp_path):
    """Evaluation scores the parsed points in float64 (KMeansUpdate.java:139-178): features
    with a large offset and a small spread (1e6 + O(0.01): float32 spacing there is 0.0625)
    give the fp64 SSE of the text values, not of float32-rounded points."""
    rs = np.random.default_rng(3)
    pts = 1e6 + rs.normal(0, 0.02, (400, 4)) + np.repeat(np.arange(4)[:, None] * 4.0, 100, 0)
    lines = ["%.6f,%.6f,%.6f,%.6f" % tuple(p) for p in pts]
    upd = KMeansUpdate(_update_config(tmp_path, "SSE"))
    pmml = upd.build_model(None, lines, [4], str(tmp_path / "cand"))
    ev = upd.evaluate(None, pmml, str(tmp_path), [], lines)
    cen = np.stack([c.center for c in read_clusters(pmml)])
    x = np.array([[float(t) for t in l.split(",")] for l in lines])
    d2 = ((x[:, None, :] - cen[None, :, :]) ** 2).sum(2).min(1)
    assert ev == pytest.approx(-d2.sum(), rel=1e-9)
    x32 = x.astype(np.float32).astype(np.float64)
    d32 = ((x32[:, None, :] - cen[None, :, :]) ** 2).sum(2).min(1)
    assert abs(-d32.sum() - ev) > 1e-6 * abs(ev)      # float32 points would differ


@pytest.mark.gpu
def test_device_double_formatter_matches_host(cuda):
    """fmt64.hip (Ryu on the device) writes the host formatter's bytes for every double, and
    the cluster update block built from its slots equals the host-formatted one."""
    from oryx_amd import ingest, native
    native.require_kernels()
    from tests.test_speed_batch import _double_cases
    v = _double_cases(2_000_000, seed=11)
    hs, hl = ingest.f64_repr_slots(v)
    ds, dl = ingest.f64_repr_slots(torch.from_numpy(v).to(cuda))
    assert np.array_equal(hl, dl)
    mask = np.arange(24)[None, :] < hl[:, None].astype(np.int64)
    assert np.array_equal(np.where(mask, hs, 0), np.where(mask, ds, 0))
    g = np.random.default_rng(2)
    centers = g.standard_normal((300, 256)) * 10.0 ** g.integers(-8, 8, (300, 1))
    centers[0, :5] = [0.0, -0.0, 1.0, 1e16, 5e-324]
    ids = g.integers(0, 10 ** 9, 300)
    counts = g.integers(1, 10 ** 6, 300)
    host = ingest.format_cluster_updates(ids, centers, counts)
    dev = ingest.format_cluster_updates(ids, centers, counts,
                                        device_centers=torch.from_numpy(centers).to(cuda))
    assert list(host) == list(dev)
    assert np.array_equal(host.ends, dev.ends)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,d", [(3000, 77, 37), (1000, 600, 1), (257, 1000, 256)])
def test_device_nearest_matches_sequential_scan(cuda, n, k, d):
    """oryx_kmeans_nearest_f64 (cluster chunks merged in order, points through the scalar
    unit) == the sequential scan: squared differences summed over the features in order, the
    first strictly smaller distance winning -- the same indices, odd feature counts and
    duplicate centers (ties) included; distances to the rounding of the kernel's fused
    multiply-adds (the scan here rounds the square and the sum separately)."""
    from oryx_amd.models.kmeans.common import ClusterSet
    g = np.random.default_rng(n + k + d)
    centers = g.standard_normal((k, d))
    centers[k // 2] = centers[k // 3]            # a tie: the lower index must win
    x = centers[g.integers(0, k, n)] + 0.3 * g.standard_normal((n, d))
    cs = ClusterSet([ClusterInfo(j, centers[j], 1) for j in range(k)], torch.device(cuda))
    idx, dist = cs.nearest_batch_device(torch.from_numpy(x).to(cuda))
    acc = np.zeros((n, k))
    for f in range(d):
        df = x[:, f, None] - centers[None, :, f]
        acc += df * df
    want = np.argmin(acc, axis=1)                # first occurrence of the minimum
    assert np.array_equal(idx.cpu().numpy(), want)
    np.testing.assert_allclose(dist.cpu().numpy(), np.sqrt(acc[np.arange(n), want]),
                               rtol=1e-14, atol=0)
