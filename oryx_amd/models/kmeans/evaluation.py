"""k-means model evaluation: SSE, Davies-Bouldin, Dunn and Silhouette.

Equivalents of ``AbstractKMeansEvaluation.fetchClusterMetrics``
(``[mllib]/kmeans/AbstractKMeansEvaluation.java:59-74``), ``ClusterMetric``,
``SumSquaredError`` (``SumSquaredError.java:31-34``), ``DaviesBouldinIndex``
(``DaviesBouldinIndex.java:38-64``), ``DunnIndex`` (``DunnIndex.java:38-58``) and
``SilhouetteCoefficient`` (``SilhouetteCoefficient.java:39-147``, sample cap 100 000).

The per-point nearest-center assignment and the per-cluster (count, sum d, sum d^2) reduction
run as batched float64 tensor ops on the device; the silhouette's O(S^2) pairwise distances
are computed tile by tile and reduced per cluster with one GEMM against the cluster one-hot
matrix (sum_j d(p, j) for every cluster at once), never materialising S x S.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...utils import rng
from .common import ClusterInfo

__all__ = ["ClusterMetric", "fetch_cluster_metrics", "sum_squared_error", "davies_bouldin_index",
           "dunn_index", "silhouette_coefficient", "silhouette_of", "fetch_sample_data",
           "MAX_SAMPLE_SIZE", "EVAL_STRATEGIES", "evaluate"]

MAX_SAMPLE_SIZE = 100000
EVAL_STRATEGIES = ("SSE", "DAVIES_BOULDIN", "DUNN", "SILHOUETTE")


class ClusterMetric:
    __slots__ = ("count", "sum_dist", "sum_squared_dist")

    def __init__(self, count: int, sum_dist: float, sum_squared_dist: float):
        self.count = int(count)
        self.sum_dist = float(sum_dist)
        self.sum_squared_dist = float(sum_squared_dist)

    def get_mean_dist(self) -> float:
        return self.sum_dist / self.count

    def add(self, other: "ClusterMetric") -> "ClusterMetric":
        return ClusterMetric(self.count + other.count, self.sum_dist + other.sum_dist,
                             self.sum_squared_dist + other.sum_squared_dist)


def _device(device) -> torch.device:
    if device is not None:
        return torch.device(device)
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def _centers(clusters: Sequence[ClusterInfo], dev) -> torch.Tensor:
    return torch.from_numpy(np.stack([c.center for c in clusters])).to(dev, torch.float64)


def _assign(x: torch.Tensor, c: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact float64 nearest center (first minimum wins) and its Euclidean distance."""
    n, d = x.shape
    k = c.shape[0]
    idx = torch.empty(n, dtype=torch.int64, device=x.device)
    dist = torch.empty(n, dtype=torch.float64, device=x.device)
    chunk = max(1, (1 << 25) // max(1, k * d))
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        dd = (x[lo:hi, None, :] - c[None]).pow(2).sum(2)
        v, i = dd.min(1)
        idx[lo:hi] = i
        dist[lo:hi] = v.sqrt()
    return idx, dist


def fetch_cluster_metrics(clusters: Sequence[ClusterInfo], data, device=None
                          ) -> Dict[int, ClusterMetric]:
    """cluster id -> ClusterMetric over the points assigned to it (absent if none)."""
    dev = _device(device)
    x = torch.as_tensor(np.asarray(data, dtype=np.float64)).to(dev)
    c = _centers(clusters, dev)
    k = len(clusters)
    idx, dist = _assign(x, c)
    cnt = torch.bincount(idx, minlength=k)
    s1 = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(0, idx, dist)
    s2 = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(0, idx, dist * dist)
    cnt, s1, s2 = cnt.cpu().tolist(), s1.cpu().tolist(), s2.cpu().tolist()
    return {clusters[j].id: ClusterMetric(cnt[j], s1[j], s2[j]) for j in range(k) if cnt[j] > 0}


def sum_squared_error(clusters, data, device=None) -> float:
    return math.fsum(m.sum_squared_dist for m in fetch_cluster_metrics(clusters, data,
                                                                        device).values())


def _center_dist(a: ClusterInfo, b: ClusterInfo) -> float:
    d = a.center - b.center
    return float(np.sqrt(np.dot(d, d)))


def davies_bouldin_index(clusters, data, device=None) -> float:
    """Mean over clusters i of max_j (s_i + s_j) / d(c_i, c_j) (not symmetric in i, j)."""
    metrics = fetch_cluster_metrics(clusters, data, device)
    by_id = sorted(clusters, key=lambda c: c.id)
    vals = []
    for ci in by_id:
        if ci.id not in metrics:
            continue
        si = metrics[ci.id].get_mean_dist()
        best = 0.0
        for cj in by_id:
            if cj.id == ci.id or cj.id not in metrics:
                continue
            r = (si + metrics[cj.id].get_mean_dist()) / _center_dist(ci, cj)
            best = max(best, r)
        vals.append(best)
    return sum(vals) / len(vals) if vals else 0.0


def dunn_index(clusters, data, device=None) -> float:
    """min inter-center distance / max mean intra-cluster distance."""
    metrics = fetch_cluster_metrics(clusters, data, device)
    max_intra = max((m.get_mean_dist() for m in metrics.values()), default=float("nan"))
    min_inter = float("inf")
    cl = list(clusters)
    for i in range(len(cl)):
        for j in range(i + 1, len(cl)):
            min_inter = min(min_inter, _center_dist(cl[i], cl[j]))
    return min_inter / max_intra


def silhouette_of(ai: float, bi: float) -> float:
    if ai < bi:
        return 1.0 - ai / bi
    if ai > bi:
        return bi / ai - 1.0
    return 0.0


def fetch_sample_data(data: np.ndarray, max_size: int = MAX_SAMPLE_SIZE) -> np.ndarray:
    n = len(data)
    if n > max_size:
        keep = rng.get_random().generator.random(n) < (max_size / n)
        return data[keep]
    return data


def silhouette_coefficient(clusters, data, device=None, max_sample: int = MAX_SAMPLE_SIZE
                           ) -> float:
    dev = _device(device)
    sample = fetch_sample_data(np.asarray(data, dtype=np.float64), max_sample)
    s = len(sample)
    if s == 0:
        return 0.0
    x = torch.from_numpy(sample).to(dev)
    c = _centers(clusters, dev)
    k = len(clusters)
    idx, _ = _assign(x, c)
    onehot = torch.zeros((s, k), dtype=torch.float64, device=dev)
    onehot[torch.arange(s, device=dev), idx] = 1.0
    size = onehot.sum(0)                                     # [k]
    xn = x.pow(2).sum(1)
    d = x.shape[1]
    exact = s * s * d <= (1 << 24)
    rows = max(1, min(s, (1 << 24) // max(1, s)))
    total = torch.zeros((), dtype=torch.float64, device=dev)
    for lo in range(0, s, rows):
        hi = min(s, lo + rows)
        if exact:
            dist = (x[lo:hi, None, :] - x[None]).pow(2).sum(2).sqrt()
        else:
            g = x[lo:hi].matmul(x.t())
            dist = (xn[lo:hi, None] + xn[None] - 2.0 * g).clamp_min_(0).sqrt_()
        per_cluster = dist.matmul(onehot)                    # [rows, k]: sum d(p, cluster)
        own = idx[lo:hi]
        own_size = size[own]
        a = per_cluster.gather(1, own[:, None])[:, 0] / (own_size - 1.0)
        mean_other = per_cluster / size[None, :]
        mean_other[torch.arange(hi - lo, device=dev), own] = float("inf")
        mean_other[:, size == 0] = float("inf")
        b = mean_other.min(1).values
        sil = torch.where(a < b, 1.0 - a / b, torch.where(a > b, b / a - 1.0,
                                                          torch.zeros_like(a)))
        sil = torch.where(own_size > 1, sil, torch.zeros_like(sil))
        total += sil.sum()
    return float(total) / s


def evaluate(strategy: str, clusters, data, device=None) -> float:
    """Eval for MLUpdate (higher is better): -DB, Dunn, Silhouette, -SSE."""
    if strategy == "DAVIES_BOULDIN":
        return -davies_bouldin_index(clusters, data, device)
    if strategy == "DUNN":
        return dunn_index(clusters, data, device)
    if strategy == "SILHOUETTE":
        return silhouette_coefficient(clusters, data, device)
    if strategy == "SSE":
        return -sum_squared_error(clusters, data, device)
    raise ValueError("Unknown evaluation strategy " + strategy)
