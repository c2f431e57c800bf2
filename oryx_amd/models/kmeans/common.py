"""k-means shared model types: clusters, nearest-cluster search, feature extraction, PMML.

Equivalents of ``ClusterInfo`` (``[app-common]/kmeans/ClusterInfo.java:26-71``),
``KMeansUtils`` (``[app-common]/kmeans/KMeansUtils.java:40-77``), ``EuclideanDistanceFn``
(``[app-common]/kmeans/EuclideanDistanceFn.java:23-37``) and ``KMeansPMMLUtils``
(``[app-common]/kmeans/KMeansPMMLUtils.java:37-83``), plus :class:`ClusterSet`, the MI355X
addition: the cluster centers kept as one matrix (host float64 mirror + device copy) so that a
batch of points is assigned with one distance GEMM + argmin instead of a per-point scan.
"""

from __future__ import annotations

import threading
import xml.etree.ElementTree as ET
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...utils import pmml as pm
from ...utils import text
from .. import app_pmml
from ..schema import InputSchema

__all__ = ["ClusterInfo", "closest_cluster", "euclidean", "features_from_tokens",
           "parse_feature_matrix", "check_unique_ids", "read_clusters",
           "validate_pmml_vs_schema", "ClusterSet", "clustering_model_pmml"]


def euclidean(a, b) -> float:
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        raise ValueError("length mismatch")
    d = a - b
    return float(np.sqrt(np.dot(d, d)))


class ClusterInfo:
    """Cluster id, center and count; ``update`` folds in a batch mean (running mean)."""

    def __init__(self, id_: int, center, initial_count: int):
        center = np.asarray(center, dtype=np.float64).copy()
        if center.ndim != 1 or len(center) == 0:
            raise ValueError("empty center")
        if initial_count < 1:
            raise ValueError("count must be >= 1")
        self.id = int(id_)
        self.center = center
        self.count = int(initial_count)
        self._lock = threading.Lock()

    # instances built by _owned share this lock (update() is rare on them)
    _lock = threading.Lock()

    @classmethod
    def _owned_many(cls, ids, rows, counts) -> List["ClusterInfo"]:
        """No validation and no copies: ``rows`` are float64 center rows the caller hands
        over (the speed layer's 1k-cluster updates spent ~1 ms in the checked constructor)."""
        new = cls.__new__
        out = []
        for i, row, c in zip(ids, rows, counts):
            info = new(cls)
            info.__dict__ = {"id": i, "center": row, "count": c}
            out.append(info)
        return out

    def get_id(self) -> int:
        return self.id

    def get_center(self) -> np.ndarray:
        return self.center

    def get_count(self) -> int:
        return self.count

    def update(self, new_point, new_count: int) -> None:
        p = np.asarray(new_point, dtype=np.float64)
        if p.shape != self.center.shape:
            raise ValueError("length mismatch")
        with self._lock:
            total = int(new_count) + self.count
            frac = float(new_count) / total
            self.center = self.center + frac * (p - self.center)
            self.count = total

    def __repr__(self):
        return "%d [%s] %d" % (self.id, ", ".join(text.java_double_str(float(v))
                                                  for v in self.center), self.count)


def closest_cluster(clusters: Sequence[ClusterInfo], vector) -> Tuple[ClusterInfo, float]:
    """Linear scan, first strictly-smaller distance wins (reference tie order)."""
    if not clusters:
        raise ValueError("no clusters")
    v = np.asarray(vector, dtype=np.float64)
    centers = np.stack([c.center for c in clusters])
    if centers.shape[1] != v.shape[0]:
        raise ValueError("length mismatch")
    d = np.sqrt(((centers - v[None, :]) ** 2).sum(1))
    i = int(np.argmin(d))   # argmin returns the first minimum
    dist = float(d[i])
    if not np.isfinite(dist):
        raise ValueError("non-finite distance")
    return clusters[i], dist


def features_from_tokens(data: Sequence[str], schema: InputSchema) -> np.ndarray:
    """Predictor vector from one parsed record (active features, parsed as doubles)."""
    out = np.zeros(schema.get_num_predictors(), dtype=np.float64)
    for fi, tok in enumerate(data):
        if schema.is_active(fi):
            out[schema.feature_to_predictor_index(fi)] = _parse_double(tok)
    return out


def _parse_double(tok: str) -> float:
    t = tok.strip()
    if t and t[-1] in "dDfF" and not t.lower().endswith("inf"):
        t = t[:-1]
    if t in ("Infinity", "+Infinity"):
        return float("inf")
    if t == "-Infinity":
        return float("-inf")
    if t.lower() in ("inf", "+inf", "-inf", "infinity", "-infinity", "nan") and t != "NaN":
        raise ValueError("For input string: \"%s\"" % tok)
    return float(t)


def parse_feature_matrix(lines: Sequence[str], schema: InputSchema) -> np.ndarray:
    """All records -> float64 [n, num_predictors] (vectorised for plain CSV input)."""
    n = len(lines)
    p = schema.get_num_predictors()
    if n == 0:
        return np.zeros((0, p), dtype=np.float64)
    cols = schema.predictor_feature_indices
    plain = not any(('"' in l) or l.startswith("[") for l in lines)
    if plain:
        try:
            toks = np.array([l.split(",") for l in lines], dtype=object)
            if toks.ndim == 2 and toks.shape[1] == schema.get_num_features():
                return toks[:, cols].astype(np.float64)
        except (ValueError, TypeError):
            pass
    out = np.zeros((n, p), dtype=np.float64)
    for r, line in enumerate(lines):
        out[r] = features_from_tokens(text.parse_input_line(line), schema)
    return out


def check_unique_ids(clusters: Iterable[ClusterInfo]) -> None:
    ids = [c.id for c in clusters]
    if len(set(ids)) != len(ids):
        raise ValueError("cluster IDs are not unique: %s" % ids)


# ---------------------------------------------------------------- PMML

def _clustering_model(pmml: pm.PMMLDoc) -> ET.Element:
    models = pmml.models()
    if len(models) != 1:
        raise ValueError("Should have exactly one model, but had %d" % len(models))
    m = models[0]
    if m.tag != pm.q("ClusteringModel"):
        raise ValueError("not a ClusteringModel")
    return m


def validate_pmml_vs_schema(pmml: pm.PMMLDoc, schema: InputSchema) -> None:
    m = _clustering_model(pmml)
    if m.get("functionName") != "clustering":
        raise ValueError("function is not clustering")
    dd = pmml.find("DataDictionary")
    if dd is None or schema.feature_names != app_pmml.feature_names_of(dd):
        raise ValueError("Feature names in schema don't match names in PMML")
    ms = m.find(pm.q("MiningSchema"))
    if ms is None or schema.feature_names != app_pmml.feature_names_of(ms):
        raise ValueError("Feature names in schema don't match MiningSchema")


def read_clusters(pmml: pm.PMMLDoc) -> List[ClusterInfo]:
    m = _clustering_model(pmml)
    out = []
    for c in m.findall(pm.q("Cluster")):
        arr = c.find(pm.q("Array"))
        out.append(ClusterInfo(int(c.get("id")), pm.parse_array(arr), int(c.get("size"))))
    return out


def clustering_model_pmml(schema: InputSchema, centers: np.ndarray, sizes: Sequence[int]
                          ) -> pm.PMMLDoc:
    """PMML ClusteringModel (CENTER_BASED, squared Euclidean) + DataDictionary
    (``KMeansUpdate.kMeansModelToPMML`` / ``pmmlClusteringModel``,
    ``[mllib]/kmeans/KMeansUpdate.java:180-221``)."""
    doc = pm.build_skeleton_pmml()
    doc.add(app_pmml.build_data_dictionary(schema, None))
    model = ET.Element(pm.q("ClusteringModel"), {
        "functionName": "clustering", "modelClass": "centerBased",
        "numberOfClusters": str(len(centers))})
    model.append(app_pmml.build_mining_schema(schema))
    cm = pm.sub(model, "ComparisonMeasure", {"kind": "distance"})
    pm.sub(cm, "squaredEuclidean")
    for fi, name in enumerate(schema.feature_names):
        if schema.is_active(fi):
            pm.sub(model, "ClusteringField", {"field": name, "isCenterField": "true"})
    for i, (c, s) in enumerate(zip(centers, sizes)):
        cl = pm.sub(model, "Cluster", {"id": str(i), "size": str(int(s))})
        cl.append(pm.to_array([float(v) for v in c]))
    doc.add(model)
    return doc


# ---------------------------------------------------------------- batched nearest search

_DEVICE_MIN_BATCH = 256


class ClusterSet:
    """Clusters as a matrix: ``nearest`` for one point (host), ``nearest_batch`` on the GPU.

    Index ``i`` in the set is list position ``i`` (cluster ``id`` is stored separately), as
    the reference's ``List<ClusterInfo>`` whose ``get(id)``/``set(id)`` use positions.
    """

    def __init__(self, clusters: List[ClusterInfo], device: Optional[torch.device] = None):
        if not clusters:
            raise ValueError("no clusters")
        check_unique_ids(clusters)
        self.clusters = list(clusters)
        self.device = device
        self._lock = threading.RLock()
        self._dev_centers = None
        self._version = 0
        self._dev_version = -1

    def __len__(self):
        return len(self.clusters)

    def get(self, index: int) -> ClusterInfo:
        with self._lock:
            return self.clusters[index]

    def set(self, index: int, info: ClusterInfo) -> None:
        with self._lock:
            self.clusters[index] = info
            self._version += 1

    def touch(self) -> None:
        with self._lock:
            self._version += 1

    def centers(self) -> np.ndarray:
        with self._lock:
            return np.stack([c.center for c in self.clusters])

    def nearest(self, vector) -> Tuple[ClusterInfo, float]:
        with self._lock:
            snapshot = list(self.clusters)
        return closest_cluster(snapshot, vector)

    def _device_centers(self) -> torch.Tensor:
        with self._lock:
            if self._dev_version != self._version or self._dev_centers is None:
                self._dev_centers = torch.from_numpy(self.centers()).to(self.device,
                                                                         torch.float64)
                self._dev_version = self._version
            return self._dev_centers

    def device_state(self) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(centers fp64 [k, d], centers feature-major fp64 [d, k], counts int64 [k]) on the
        device, rebuilt when the clusters changed."""
        with self._lock:
            st = getattr(self, "_dev_state", None)
            if st is None or st[0] != self._version:
                c = self._device_centers()
                cnt = torch.tensor([ci.count for ci in self.clusters], dtype=torch.int64,
                                   device=self.device)
                st = (self._version, c, c.t().contiguous(), cnt)
                self._dev_state = st
            return st[1], st[2], st[3]

    def set_many(self, positions: Sequence[int], centers: np.ndarray,
                 counts: Sequence[int], device_update=None) -> None:
        """Replace the centers and counts of the clusters at ``positions`` (one version bump).

        ``device_update``: (positions, centers fp64, counts int64) as device tensors of the
        same values -- written into the current device state in place instead of rebuilding
        it (a 1000 x 256 re-stack and upload per speed-layer micro-batch otherwise); the
        host ``centers`` rows are then kept without a copy."""
        with self._lock:
            owned = device_update is not None
            if owned:
                cl = self.clusters
                infos = ClusterInfo._owned_many([cl[p].id for p in positions], list(centers),
                                                [int(c) for c in counts])
                for pos, info in zip(positions, infos):
                    cl[pos] = info
            else:
                for j, pos in enumerate(positions):
                    old = self.clusters[pos]
                    self.clusters[pos] = ClusterInfo(old.id, centers[j], int(counts[j]))
            st = getattr(self, "_dev_state", None)
            current = (st is not None and st[0] == self._version and
                       self._dev_version == self._version)
            self._version += 1
            if owned and current:
                pos_t, c_t, n_t = device_update
                _, c, ct, cnt = st
                c[pos_t] = c_t
                ct[:, pos_t] = c_t.t()
                cnt[pos_t] = n_t
                self._dev_version = self._version
                self._dev_state = (self._version, c, ct, cnt)

    def nearest_batch_device(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(positions int64 [n], distances fp64 [n]) of device points ``x`` fp64 [n, d] by the
        exact fp64 kernel (``oryx_kmeans_nearest_f64``, csrc/kernels/kmeans_speed.hip)."""
        from ... import native
        _, ct, _ = self.device_state()
        x = x.to(torch.float64).contiguous()
        n0 = x.shape[0]
        if 0 < n0 < 16:       # the kernel takes at least 16 points: repeat the last one
            x = torch.cat([x, x[-1:].expand(16 - n0, -1)]).contiguous()
        n, d = x.shape
        idx = torch.empty(n, dtype=torch.int64, device=x.device)
        dist = torch.empty(n, dtype=torch.float64, device=x.device)
        lib = native.require_kernels()
        k = int(ct.shape[1])
        # per-point minima of each cluster chunk, merged by the kernel's second pass
        nch = int(lib.oryx_kmeans_nearest_chunks(n, k))
        part_b = torch.empty(max(n * nch, 1), dtype=torch.float64, device=x.device)
        part_i = torch.empty(max(n * nch, 1), dtype=torch.int32, device=x.device)
        rc = lib.oryx_kmeans_nearest_f64(
            x.data_ptr(), n, d, ct.data_ptr(), k, idx.data_ptr(), dist.data_ptr(),
            part_b.data_ptr(), part_i.data_ptr(), native.stream_ptr(x.device))
        native.check(rc, "oryx_kmeans_nearest_f64")
        return idx[:n0], dist[:n0]

    def nearest_batch(self, x: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """(positions int64 [n], Euclidean distances float64 [n]) for points ``x``.

        Exact float64 (differences, not the |x|^2 - 2xc + |c|^2 expansion) so that ties and
        distances match the per-point scan.  Large batches on the device, chunked.
        """
        x = np.asarray(x, dtype=np.float64)
        n = x.shape[0]
        if n == 0:
            return np.zeros(0, np.int64), np.zeros(0, np.float64)
        use_dev = self.device is not None and self.device.type == "cuda" and n >= _DEVICE_MIN_BATCH
        if use_dev:
            c = self._device_centers()
            xt = torch.from_numpy(x).to(self.device)
        else:
            c = torch.from_numpy(self.centers())
            xt = torch.from_numpy(x)
        k, d = c.shape
        chunk = max(1, (1 << 26) // max(1, k * d))
        idx = torch.empty(n, dtype=torch.int64, device=xt.device)
        dist = torch.empty(n, dtype=torch.float64, device=xt.device)
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            diff = xt[lo:hi, None, :] - c[None, :, :]
            dd = diff.pow(2).sum(2)
            v, i = dd.min(1)
            idx[lo:hi] = i
            dist[lo:hi] = v.sqrt()
        return idx.cpu().numpy(), dist.cpu().numpy()
