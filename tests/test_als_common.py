"""ALSUtilsTest / FeatureVectorsTest / ALSUpdateTest / speed fold-in ports."""

import math
import threading

import numpy as np
import pytest
import torch

from oryx_amd.models.als import common
from oryx_amd.models.als.batch import aggregate_scores, decay_rating, known_items
from oryx_amd.models.als.common import FeatureVectors, compute_target_qui, compute_updated_xu
from oryx_amd.ops import als as als_ops
from oryx_amd.utils import mathx


def test_implicit_qui():
    for v, c in ((0.0, 1.0), (0.0, 0.0), (0.0, -1.0), (0.5, 1.0), (-0.5, 0.0)):
        assert math.isnan(compute_target_qui(True, v, c))
    assert compute_target_qui(True, 1.0, 0.5) == 0.75
    assert compute_target_qui(True, -1.0, 0.5) == 0.25
    for d in (-1.0, 0.0, 0.5, 1.0, 2.0):
        assert compute_target_qui(False, d, 0.0) == d


def _solver():
    rows = [[1.0, 2.0], [3.0, 0.0], [0.0, 1.0]]
    return mathx.get_solver(mathx.transpose_times_self(rows))


def test_compute_updated_xu():
    s = _solver()
    assert compute_updated_xu(s, 1.0, None, None, True) is None
    np.testing.assert_allclose(compute_updated_xu(s, 1.0, None, np.array([2.0, 1.0]), True),
                               [0.13043478, 0.097826086], rtol=1e-6)
    np.testing.assert_allclose(compute_updated_xu(s, 0.5, None, np.array([2.0, 1.0]), True),
                               [0.11594203, 0.08695652], rtol=1e-6)
    np.testing.assert_allclose(compute_updated_xu(s, 1.0, np.array([0.1, 0.1]),
                                                  np.array([2.0, 1.0]), True),
                               [0.16086957, 0.14565217], rtol=1e-6)


def test_batched_fold_in_matches_scalar():
    s = _solver()
    inv = torch.from_numpy(s.inverse())
    xu = torch.tensor([[0.0, 0.0], [0.0, 0.0], [0.1, 0.1], [0.5, 0.9]])
    pres = torch.tensor([False, False, True, True])
    yi = torch.tensor([[2.0, 1.0], [2.0, 1.0], [2.0, 1.0], [1.0, 1.0]])
    vals = torch.tensor([1.0, 0.5, 1.0, 1.0])
    new, valid = als_ops.fold_in(inv, vals, xu, pres, yi, True)
    for j in range(4):
        ref = compute_updated_xu(s, float(vals[j]), xu[j].numpy() if pres[j] else None,
                                 yi[j].numpy(), True)
        if ref is None:
            assert not valid[j]
        else:
            assert valid[j]
            np.testing.assert_allclose(new[j].numpy(), ref, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("device", ["cpu"])
def test_feature_vectors(device):
    fv = FeatureVectors(1, torch.device(device))
    assert fv.size() == 0
    fv.set_vector("foo", [1.0])
    assert fv.size() == 1 and fv.get_vector("foo").tolist() == [1.0]
    fv.remove_vector("foo")
    assert fv.size() == 0 and fv.get_vector("foo") is None
    fv3 = FeatureVectors(3, torch.device(device))
    fv3.set_vector("foo", [1.0, 2.0, 4.0])
    fv3.set_vector("bar", [1.5, -1.0, 0.0])
    np.testing.assert_allclose(fv3.get_vtv(), [[3.25, 0.5, 4.0], [0.5, 5.0, 8.0],
                                               [4.0, 8.0, 16.0]])
    out = []
    fv3.for_each(lambda i, v: out.append("%s%s" % (i, v[0])))
    assert sorted(out) == ["bar1.5", "foo1.0"]
    fv = FeatureVectors(1)
    fv.set_vector("foo", [1.0])
    fv.retain_recent_and_ids({"foo"})
    assert fv.size() == 1
    fv.retain_recent_and_ids({"bar"})
    assert fv.size() == 0
    fv.set_vector("foo", [1.0])
    ids = set()
    fv.add_all_ids_to(ids)
    assert ids == {"foo"}
    fv.remove_all_ids_from(ids)
    assert not ids
    rec = set()
    fv.add_all_recent_to(rec)
    assert rec == {"foo"}
    fv.retain_recent_and_ids({"foo"})
    rec.clear()
    fv.add_all_recent_to(rec)
    assert not rec


def test_feature_vectors_concurrent_and_device_mirror():
    fv = FeatureVectors(2, torch.device("cpu"))
    counter = iter(range(10 ** 9))
    lock = threading.Lock()

    def work():
        for _ in range(2000):
            with lock:
                c = next(counter)
            fv.set_vector(str(c), [float(c), 1.0])

    ts = [threading.Thread(target=work) for _ in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert fv.size() == 16000
    mat, valid, norms = fv.device_view()
    assert int(valid.sum()) == 16000
    fv.remove_vector("5")
    mat, valid, _ = fv.device_view()
    assert int(valid.sum()) == 15999
    assert mat.sum(0)[1].item() == 15999.0


def test_decay():
    assert decay_rating(2.0, 1000, 1000, 0.5) == 2.0
    assert abs(decay_rating(2.0, 0, 86400000, 0.5) - 1.0) < 1e-12
    assert abs(decay_rating(2.0, 0, 2 * 86400000, 0.5) - 0.5) < 1e-12


def test_aggregate_and_known_items():
    u = np.array([0, 0, 0, 1, 1, 2, 2])
    i = np.array([0, 0, 0, 1, 1, 2, 2])
    s = np.array([1, 2, np.nan, 3, 4, np.nan, 5.0])
    ts = np.array([1, 2, 3, 1, 2, 1, 2])
    uu, ii, ss = aggregate_scores(u, i, s, ts, True)
    assert uu.tolist() == [1, 2] and ss.tolist() == [7.0, 5.0]
    uu, ii, ss = aggregate_scores(u, i, s, ts, False)
    assert ss.tolist() == [4.0, 5.0]
    k = known_items(["a,x,1,1", "a,y,1,2", "a,x,,3", "b,z,1,4", "c,w,1,5", "c,w,,6"])
    assert k == {"a": {"y"}, "b": {"z"}, "c": set()}


def test_known_items_json_matches_sets():
    import json
    from oryx_amd.models.als.batch import known_items, known_items_json
    lines = ["a,x,1,1", "a,y,1,2", "a,x,,3", "b,z,1,4", "c,w,1,5", "c,w,,6", "b,\"q\\\\r\",2,7",
             "d,b10,1,1", "d,b9,1,2", "d,a,1,3"]
    sets = known_items(lines)
    js = known_items_json(lines)
    assert set(js) == set(sets)
    for u in sets:
        assert json.loads(js[u]) == sorted(sets[u])


def test_device_aggregation_matches_host():
    import numpy as np
    from oryx_amd.models.als.batch import aggregate_scores, aggregate_scores_device
    g = np.random.default_rng(3)
    n = 20000
    u = g.integers(0, 50, n)
    i = g.integers(0, 40, n)
    s = g.integers(1, 5, n).astype(np.float64)
    s[g.random(n) < 0.1] = np.nan
    # many time ties (arrival order decides): one composite-key sort; a time range too wide
    # to pack next to the (user, item) key: the two-sort path
    from oryx_amd.models.als.batch import aggregate_scores_reference
    for ts in (g.integers(0, 1000, n), g.integers(0, 1 << 60, n) // 977 * 977):
        for implicit in (True, False):
            ref = aggregate_scores_reference(u, i, s, ts, implicit)
            for got in (aggregate_scores(u, i, s, ts, implicit),            # native
                        aggregate_scores_device(u, i, s, ts, implicit, "cpu")):
                for x, y in zip(ref, got):
                    assert np.array_equal(x, y) or np.allclose(x, y, rtol=1e-12,
                                                               equal_nan=True)


@pytest.mark.gpu
def test_device_aggregation_matches_host_gpu(cuda):
    import numpy as np
    from oryx_amd.models.als.batch import aggregate_scores, aggregate_scores_device
    g = np.random.default_rng(4)
    n = 200000
    u = g.integers(0, 500, n)
    i = g.integers(0, 400, n)
    s = g.integers(1, 5, n).astype(np.float64)
    s[g.random(n) < 0.1] = np.nan
    ts = g.integers(0, 1000, n)
    for implicit in (True, False):
        a = aggregate_scores(u, i, s, ts, implicit)
        b = aggregate_scores_device(u, i, s, ts, implicit, cuda)
        for x, y in zip(a, b):
            assert np.allclose(x, y, rtol=1e-12, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("implicit", [True, False])
@pytest.mark.parametrize("k", [8, 64, 100])
def test_fused_foldin_matches_unfused(cuda, implicit, k):
    """oryx_als_foldin == the torch fold_in path (dot, target, inverse solve, axpy), with
    absent users / items and NaN targets (negative strengths on implicit data)."""
    import torch
    from oryx_amd import native
    g = torch.Generator().manual_seed(k)
    nu, ni, n = 300, 200, 5000
    X = torch.randn(nu, k, generator=g) * 0.3
    Y = torch.randn(ni, k, generator=g) * 0.3
    xrow = torch.randint(-1, nu, (n,), generator=g)
    yrow = torch.randint(-1, ni, (n,), generator=g)
    vals = (torch.rand(n, generator=g) * 4 - 1).float()
    xinv = torch.linalg.inv((X.T @ X).double() + torch.eye(k, dtype=torch.float64))
    yinv = torch.linalg.inv((Y.T @ Y).double() + torch.eye(k, dtype=torch.float64))
    dev = torch.device(cuda)
    out = {nm: torch.empty((n, k), device=dev) for nm in ("nx", "ny")}
    vx = torch.empty(n, dtype=torch.uint8, device=dev)
    vy = torch.empty(n, dtype=torch.uint8, device=dev)
    Xd, Yd = X.to(dev), Y.to(dev)
    xr, yr = xrow.to(dev), yrow.to(dev)
    vd = vals.to(dev)
    xi, yi = xinv.to(dev), yinv.to(dev)
    rc = native.require_kernels().oryx_als_foldin(
        Xd.data_ptr(), Yd.data_ptr(), k, xr.data_ptr(), yr.data_ptr(), vd.data_ptr(),
        xi.data_ptr(), yi.data_ptr(), int(implicit), n, out["nx"].data_ptr(),
        out["ny"].data_ptr(), vx.data_ptr(), vy.data_ptr(), native.stream_ptr(dev))
    assert rc == 0
    torch.cuda.synchronize()
    xp, yp = xrow >= 0, yrow >= 0
    xu = torch.where(xp[:, None], X[xrow.clamp_min(0)], torch.zeros(()))
    yv = torch.where(yp[:, None], Y[yrow.clamp_min(0)], torch.zeros(()))
    v64 = vals.double()
    rx, okx = als_ops.fold_in(yinv, v64, xu, xp, yv, implicit)
    ry, oky = als_ops.fold_in(xinv, v64, yv, yp, xu, implicit)
    okx, oky = okx & yp, oky & xp
    assert torch.equal(vx.cpu().bool(), okx) and torch.equal(vy.cpu().bool(), oky)
    assert torch.allclose(out["nx"].cpu()[okx], rx[okx], rtol=1e-5, atol=1e-6)
    assert torch.allclose(out["ny"].cpu()[oky], ry[oky], rtol=1e-5, atol=1e-6)


def test_native_rows_follow_inserts_and_removals():
    """FeatureVectors.native_rows (native id -> row mirror kept current from a journal)
    agrees with the Python index through bulk loads, single inserts, removals and row reuse."""
    import numpy as np
    from oryx_amd import ingest
    from oryx_amd.models.als.common import FeatureVectors
    fv = FeatureVectors(3, None)
    fv.set_vectors(["a%d" % j for j in range(100)], np.ones((100, 3), np.float32))
    d = ingest.IdDict()
    d.encode(["a5", "zz", "a99", "b1"])
    assert fv.native_rows(d).tolist() == [fv.row_of("a5"), -1, fv.row_of("a99"), -1]
    fv.set_vector("b1", [1, 2, 3])
    fv.remove_vector("a5")
    fv.set_vector("c7", [0, 0, 1])            # reuses a5's row
    fv.set_vectors(["zz", "a99"], np.zeros((2, 3), np.float32))
    fv.retain_recent_and_ids({"a99", "zz", "b1", "c7"})
    d.encode(["c7"])
    want = [fv.row_of(k) if fv.row_of(k) is not None else -1 for k in d.keys()]
    assert fv.native_rows(d).tolist() == want
    assert want[0] == -1 and want[-1] == fv.row_of("c7")


@pytest.mark.gpu
def test_speed_device_inverses_match_host_rrqr(cuda):
    """ALSSpeedModel.solver_inverses on a GPU (fused Gramian + fp64 device Cholesky) equals
    the host RRQR inverses; a rank-deficient factor matrix still raises the reference's
    SingularMatrixSolverException (the device certificate fails, the host path decides)."""
    import numpy as np
    import torch
    from oryx_amd.models.als.speed import ALSSpeedModel
    from oryx_amd.utils import mathx
    g = np.random.default_rng(5)
    k = 32
    m = ALSSpeedModel(k, True, torch.device(cuda))
    X = g.standard_normal((3000, k)).astype(np.float32)
    Y = g.standard_normal((2000, k)).astype(np.float32)
    m.X.set_vectors(["U%d" % j for j in range(len(X))], X)
    m.Y.set_vectors(["I%d" % j for j in range(len(Y))], Y)
    xi, yi = m.solver_inverses()
    assert xi.device.type == "cuda" and xi.dtype == torch.float64
    for inv, mat in ((xi, X), (yi, Y)):
        ref = mathx.get_solver(mat.astype(np.float64).T @ mat.astype(np.float64)).inverse()
        np.testing.assert_allclose(inv.cpu().numpy(), ref, rtol=1e-4, atol=1e-7)
    bad = ALSSpeedModel(k, True, torch.device(cuda))
    Yb = Y.copy()
    Yb[:, 1] = Yb[:, 0]                       # rank k - 1
    bad.X.set_vectors(["U%d" % j for j in range(len(X))], X)
    bad.Y.set_vectors(["I%d" % j for j in range(len(Yb))], Yb)
    with pytest.raises(mathx.SingularMatrixSolverException):
        bad.solver_inverses()


def test_item_filter_rescorer_forms_agree_cpu():
    """ItemFilterRescorer: per-item, array and device forms give the same filter / scores;
    the store's cached ID array and row mask line up with its rows."""
    import torch
    from oryx_amd.models.als.common import FeatureVectors
    from oryx_amd.models.als.rescorer import ItemFilterRescorer, ItemFilterRescorerProvider
    store = FeatureVectors(2)
    ids = ["I%d" % j for j in range(20)]
    store.set_vectors(ids, np.ones((20, 2), dtype=np.float32))
    store.remove_vector("I4")
    arr = store.id_array()
    assert arr[4] is None and list(arr[:4]) == ids[:4]
    r = ItemFilterRescorer(["I3", "I7", "I4"], 2.0)
    rows = torch.arange(20)
    scores = torch.linspace(0, 1, 20)
    live = np.array([i is not None for i in arr])     # row 4 is free (its ID removed)
    dev = r.rescore_device(rows, scores, store).double().numpy()[live]
    lids = [i for i in arr if i is not None]
    host = r.rescore_many(lids, scores.double().numpy()[live])
    per = np.array([r.rescore(i, float(v)) for i, v in zip(lids, scores.numpy()[live])])
    np.testing.assert_allclose(dev, host, rtol=1e-6, equal_nan=True)
    np.testing.assert_allclose(host, per, rtol=1e-12, equal_nan=True)
    assert [lids[j] for j in np.flatnonzero(np.isnan(host))] == ["I3", "I7"]
    p = ItemFilterRescorerProvider()
    assert p.get_recommend_rescorer(["U1"], []) is None
    assert p.get_recommend_rescorer(["U1"], ["exclude:I2", "factor:3"]).is_filtered("I2")
    # the provider reuses one rescorer per argument list (its device mask survives requests)
    assert p.get_recommend_rescorer(["U2"], ["exclude:I2", "factor:3"]) is \
        p.get_recommend_rescorer(["U1"], ["exclude:I2", "factor:3"])


def test_mod_exclude_rescorer_native_suffixes_cpu(monkeypatch):
    """The benchmark's example rescorer (drop IDs whose numeric suffix is divisible by N):
    its device mask comes from the store's native ID map (key_suffixes) and agrees with the
    per-item form, also after rows are removed and reused; value updates keep the mask."""
    import torch
    from oryx_amd.models.als.common import FeatureVectors
    from oryx_amd.models.als.rescorer import ItemFilterRescorerProvider
    monkeypatch.setenv("ORYX_EXAMPLE_RESCORER_EXCLUDE_MOD", "7")
    store = FeatureVectors(2)
    ids = ["I%d" % j for j in range(50)] + ["x", "item-0042", "a12b"]
    store.set_vectors(ids, np.ones((len(ids), 2), dtype=np.float32))
    store.remove_vector("I14")
    store.set_vector("Z21", np.ones(2, dtype=np.float32))        # reuses row 14
    suf = store.key_suffixes()
    arr = store.id_array()
    for row, i in enumerate(arr):
        want = -1 if i is None or not i[-1].isdigit() else \
            int(i[len(i.rstrip("0123456789")):])
        assert suf[row] == want, (row, i)
    r = ItemFilterRescorerProvider().get_recommend_rescorer(["U1"], ["factor:2", "exclude:I3"])
    rows = torch.arange(len(arr))
    scores = torch.ones(len(arr))
    dev = r.rescore_device(rows, scores, store).numpy()
    per = np.array([r.rescore(i, 1.0) if i is not None else np.nan for i in arr])
    np.testing.assert_allclose(dev, per, equal_nan=True)
    assert np.isnan(dev[arr.tolist().index("Z21")]) and np.isnan(dev[3])
    v_ids = store.id_version
    store.set_vector("I1", np.zeros(2, dtype=np.float32))
    assert store.id_version == v_ids and r._mask[1] == v_ids


@pytest.mark.gpu
@pytest.mark.parametrize("k", [50, 64, 128])
def test_spd_inverse_pair_kernel(cuda, k):
    """oryx_spd_inverse_pair (csrc/kernels/spdinv.hip): fp64 Gauss-Jordan inverses of two
    fp32 Gramians against torch.linalg.inv of the same matrices in fp64 (fp32-reference
    style: the same op in plain PyTorch); an indefinite matrix and a near-singular one are
    not certified (ok = 0)."""
    from oryx_amd import native
    g = torch.Generator().manual_seed(k)
    A = torch.randn(4 * k, k, generator=g)
    B = torch.randn(3 * k, k, generator=g)
    lib = native.require_kernels()

    def run(G0, G1):
        G0 = G0.to(cuda, torch.float32).contiguous()
        G1 = G1.to(cuda, torch.float32).contiguous()
        I0 = torch.empty((k, k), dtype=torch.float64, device=cuda)
        I1 = torch.empty_like(I0)
        ok = torch.zeros(2, dtype=torch.int32, device=cuda)
        rc = lib.oryx_spd_inverse_pair(G0.data_ptr(), G1.data_ptr(), k, I0.data_ptr(),
                                       I1.data_ptr(), float(mathx.SINGULARITY_THRESHOLD_RATIO),
                                       ok.data_ptr(), native.stream_ptr(torch.device(cuda)))
        assert rc == 0
        torch.cuda.synchronize()
        return I0.cpu(), I1.cpu(), ok.cpu().tolist()

    G0, G1 = A.T @ A, B.T @ B
    I0, I1, ok = run(G0, G1)
    assert ok == [1, 1]
    for inv, G in ((I0, G0), (I1, G1)):
        ref = torch.linalg.inv(G.double())
        torch.testing.assert_close(inv, ref, rtol=1e-9, atol=1e-12)
    indefinite = G0.clone()
    indefinite[3, 3] = -1.0
    near = B.T @ B
    near[:, 1] = near[:, 0]
    near[1, :] = near[0, :]                 # rank deficient
    _, _, ok = run(indefinite, near)
    assert ok == [0, 0]


def test_incremental_gramian_tracks_writes_and_removals_cpu():
    """FeatureVectors.gramian: one full product, then rank-one corrections per written /
    removed row (speed layer micro-batches), equal to VtV of the current rows."""
    import torch
    from oryx_amd.models.als.common import FeatureVectors
    rs = np.random.default_rng(4)
    k = 12
    fv = FeatureVectors(k, device=torch.device("cpu"))

    def ref():
        n = fv._n_rows
        m = fv._host[:n][fv._host_valid[:n]].astype(np.float64)
        return m.T @ m

    ids = ["i%d" % j for j in range(3000)]
    fv.set_vectors(ids, rs.normal(0, 1, (3000, k)).astype(np.float32))
    g = fv.gramian().numpy()
    assert np.allclose(g, ref(), rtol=1e-5, atol=1e-3)
    assert fv.gram_stats == {"full": 1, "incremental": 0}
    for rnd in range(6):
        for j in rs.integers(0, 3000, 40):                  # overwrite existing rows
            fv.set_vector("i%d" % j, rs.normal(0, 1, k).astype(np.float32))
        for j in range(5):                                  # new rows
            fv.set_vector("n%d_%d" % (rnd, j), rs.normal(0, 1, k).astype(np.float32))
        sel = ["i%d" % j for j in rs.choice(3000, 30, replace=False)]
        fv.set_vectors(sel, rs.normal(0, 1, (30, k)).astype(np.float32))   # bulk, existing
        fv.remove_vector("i%d" % rs.integers(0, 3000))
        g = fv.gramian().numpy()
        assert np.allclose(g, ref(), rtol=1e-6, atol=1e-6), rnd
    assert fv.gram_stats["full"] == 1 and fv.gram_stats["incremental"] == 6
    # a batch repeating an ID drops the corrections: the next call recomputes in full
    fv.set_vectors(["i1", "i1"], rs.normal(0, 1, (2, k)).astype(np.float32))
    assert np.allclose(fv.gramian().numpy(), ref(), rtol=1e-5, atol=1e-3)
    assert fv.gram_stats["full"] == 2
