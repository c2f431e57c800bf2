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

Sharded (:func:`evaluate_sharded`): every rank assigns its own points with the certified fp32
MFMA kernel (large GPU shares) or the float64 scan, takes float64 distances to the chosen
centers, and the K x 3 cluster metrics are all-reduced; Davies-Bouldin and Dunn then come from
one K x K center-distance matrix; the silhouette sample is drawn per rank (the same keep
probability everywhere) and gathered, and rank 0's value is broadcast.
"""

from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...utils import rng
from .common import ClusterInfo

__all__ = ["ClusterMetric", "fetch_cluster_metrics", "sum_squared_error", "davies_bouldin_index",
           "dunn_index", "silhouette_coefficient", "silhouette_of", "fetch_sample_data",
           "MAX_SAMPLE_SIZE", "EVAL_STRATEGIES", "evaluate", "evaluate_sharded",
           "local_cluster_stats"]

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


def _rows(data) -> int:
    return int(data.shape[0]) if isinstance(data, torch.Tensor) else len(data)


def _as_dev(data, dev) -> torch.Tensor:
    """Points as a device tensor (a device matrix -- the batch layer's parse -- stays put)."""
    if isinstance(data, torch.Tensor):
        return data.to(dev)
    return torch.as_tensor(np.asarray(data, dtype=np.float64)).to(dev)


def fetch_cluster_metrics(clusters: Sequence[ClusterInfo], data, device=None
                          ) -> Dict[int, ClusterMetric]:
    """cluster id -> ClusterMetric over the points assigned to it (absent if none)."""
    st = local_cluster_stats(clusters, data, device)
    return _metrics_from_arrays(clusters, st[:, 0], st[:, 1], st[:, 2])


def sum_squared_error(clusters, data, device=None) -> float:
    return math.fsum(m.sum_squared_dist for m in fetch_cluster_metrics(clusters, data,
                                                                        device).values())


def _center_dist(a: ClusterInfo, b: ClusterInfo) -> float:
    d = a.center - b.center
    return float(np.sqrt(np.dot(d, d)))


def davies_bouldin_index(clusters, data, device=None) -> float:
    """Mean over clusters i of max_j (s_i + s_j) / d(c_i, c_j) (not symmetric in i, j); one
    K x K center-distance matrix instead of the reference's double loop."""
    by_id = sorted(clusters, key=lambda c: c.id)
    return _db_from(by_id, fetch_cluster_metrics(by_id, data, device))


def dunn_index(clusters, data, device=None) -> float:
    """min inter-center distance / max mean intra-cluster distance."""
    return _dunn_from(list(clusters), fetch_cluster_metrics(clusters, data, device))


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
    if isinstance(data, torch.Tensor):
        n = int(data.shape[0])
        if n > max_sample:
            keep = torch.from_numpy(rng.get_random().generator.random(n) < (max_sample / n))
            data = data[keep.to(data.device)]
        sample = data.double().cpu().numpy()
    else:
        sample = fetch_sample_data(np.asarray(data, dtype=np.float64), max_sample)
    s = len(sample)
    if s == 0:
        return 0.0
    x = torch.from_numpy(sample).to(dev)
    c = _centers(clusters, dev)
    k = len(clusters)
    idx, _ = _assign(x, c)
    if dev.type == "cuda":
        return _silhouette_kernel(x, idx, k)
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


_SIL_MFMA = os.environ.get("ORYX_KM_SIL_MFMA", "1") != "0"


def _silhouette_kernel(x: torch.Tensor, idx: torch.Tensor, k: int) -> float:
    """Mean silhouette on the GPU: the sample sorted by cluster, one pass over the columns
    per row block with running per-cluster sums.  Dimensions <= 256: the distances come from
    fp32 MFMA dot products of the centred sample (``km_silhouette_mfma``); wider samples (or
    ``ORYX_KM_SIL_MFMA=0``) stream packed fp32 differences on the VALU
    (``km_silhouette_part``)."""
    from ... import native
    lib = native.require_kernels()
    s, d = x.shape
    order = torch.argsort(idx, stable=True)
    cl = idx[order].to(torch.int32).contiguous()
    size = torch.bincount(idx.long(), minlength=k).to(torch.int32)
    mfma = _SIL_MFMA and d <= 256
    if mfma:
        ks = 16 if d <= 64 else (32 if d <= 128 else 64)
        rows = int(lib.oryx_kmeans_silhouette_mfma_rows(ks))
        sp = -(-s // rows) * rows
        # centred in fp64 (distances unchanged; small norms: less cancellation in
        # |a|^2 + |b|^2 - 2 a.b), rows and dimensions zero-padded to the kernel's tiles
        xc = x[order].to(torch.float64)
        xc = xc - xc.mean(0, keepdim=True)
        xp = torch.zeros((sp, 4 * ks), dtype=torch.float32, device=x.device)
        xp[:s, :d] = xc.to(torch.float32)
        xn = torch.zeros(sp, dtype=torch.float32, device=x.device)
        xn[:s] = xp[:s].to(torch.float64).pow(2).sum(1).to(torch.float32)
        del xc
        row_blocks = sp // rows
    else:
        xs = x[order].to(torch.float32).contiguous()
        xt = xs.t().contiguous()
        row_blocks = (s + 255) // 256
    # column ranges at cluster boundaries, enough of them for >= ~2048 blocks
    want = max(1, min(64, -(-2048 // row_blocks)))
    starts = np.concatenate([[0], np.cumsum(size.cpu().numpy().astype(np.int64))])
    cuts = np.unique(starts[np.searchsorted(starts, np.arange(1, want) * s / want)])
    bounds = np.unique(np.concatenate([[0], cuts[(cuts > 0) & (cuts < s)], [s]]))
    nsplit = len(bounds) - 1
    d_bounds = torch.from_numpy(bounds.astype(np.int32)).to(x.device)
    work = torch.empty(2 * nsplit * s, dtype=torch.float64, device=x.device)
    partial = torch.empty((s + 255) // 256, dtype=torch.float64, device=x.device)
    if mfma:
        rc = lib.oryx_kmeans_silhouette_mfma(xp.data_ptr(), xn.data_ptr(), cl.data_ptr(),
                                             size.data_ptr(), s, ks, d_bounds.data_ptr(),
                                             nsplit, work.data_ptr(), partial.data_ptr(),
                                             native.stream_ptr(x.device))
        native.check(rc, "oryx_kmeans_silhouette_mfma")
    else:
        rc = lib.oryx_kmeans_silhouette(xs.data_ptr(), xt.data_ptr(), cl.data_ptr(),
                                        size.data_ptr(), s, d, d_bounds.data_ptr(), nsplit,
                                        work.data_ptr(), partial.data_ptr(),
                                        native.stream_ptr(x.device))
        native.check(rc, "oryx_kmeans_silhouette")
    return float(partial.sum()) / s


def _metrics_from_arrays(clusters, cnt, s1, s2) -> Dict[int, ClusterMetric]:
    return {clusters[j].id: ClusterMetric(int(cnt[j]), float(s1[j]), float(s2[j]))
            for j in range(len(clusters)) if cnt[j] > 0}


def local_cluster_stats(clusters, x, device=None) -> np.ndarray:
    """[K, 3] float64 (count, sum d, sum d^2) of this rank's points ``x`` (numpy or a device
    tensor)."""
    dev = _device(device)
    k = len(clusters)
    out = np.zeros((k, 3), dtype=np.float64)
    if _rows(x) == 0:
        return out
    c = _centers(clusters, dev)
    if dev.type == "cuda" and _rows(x) >= 65536:
        from ...ops import kmeans as km_ops
        # nearest center on the MFMA assignment kernel (certified fp32), the distance to it
        # in fp64, in slices (no fp64 copy of a multi-GB point matrix)
        xf = x.to(dev, torch.float32) if isinstance(x, torch.Tensor) else \
            torch.from_numpy(np.asarray(x, dtype=np.float32)).to(dev)
        idx, _ = km_ops.assign(xf.contiguous(), c.float(), precision="fp32")
        idx = idx.long()
        dist = torch.empty(xf.shape[0], dtype=torch.float64, device=dev)
        step = max(1, (1 << 26) // max(1, xf.shape[1]))
        xs = x.to(dev) if isinstance(x, torch.Tensor) else None
        for lo in range(0, xf.shape[0], step):
            hi = min(xf.shape[0], lo + step)
            src = xs[lo:hi] if xs is not None else \
                torch.from_numpy(np.asarray(x[lo:hi], dtype=np.float64)).to(dev)
            dist[lo:hi] = (src.double() - c[idx[lo:hi]]).pow(2).sum(1).sqrt()
    else:
        idx, dist = _assign(_as_dev(x, dev).double(), c)
    out[:, 0] = torch.bincount(idx, minlength=k).double().cpu().numpy()
    out[:, 1] = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(
        0, idx, dist).cpu().numpy()
    out[:, 2] = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(
        0, idx, dist * dist).cpu().numpy()
    return out


def _db_from(clusters, metrics) -> float:
    ids = [c.id for c in clusters]
    present = np.array([i in metrics for i in ids])
    if not present.any():
        return 0.0
    cen = np.stack([c.center for c in clusters]).astype(np.float64)
    mean = np.array([metrics[i].get_mean_dist() if i in metrics else 0.0 for i in ids])
    dd = np.sqrt(((cen[:, None, :] - cen[None]) ** 2).sum(2))
    with np.errstate(divide="ignore", invalid="ignore"):
        r = (mean[:, None] + mean[None, :]) / dd
    r[~present[:, None] | ~present[None, :]] = 0.0
    np.fill_diagonal(r, 0.0)
    r = np.where(np.isfinite(r), r, 0.0)
    return float(r.max(1)[present].mean())


def _dunn_from(clusters, metrics) -> float:
    max_intra = max((m.get_mean_dist() for m in metrics.values()), default=float("nan"))
    cen = np.stack([c.center for c in clusters]).astype(np.float64)
    dd = np.sqrt(((cen[:, None, :] - cen[None]) ** 2).sum(2))
    iu = np.triu_indices(len(clusters), 1)
    min_inter = float(dd[iu].min()) if len(iu[0]) else float("inf")
    return min_inter / max_intra


def evaluate_sharded(strategy: str, clusters, x_local: np.ndarray, ctx, device=None) -> float:
    """Like :func:`evaluate` over the union of every rank's ``x_local`` (collective)."""
    from ...parallel import shuffle, dist as dist_
    if strategy == "SILHOUETTE":
        n_local = _rows(x_local)
        n_all = sum(shuffle.all_gather_int(n_local, ctx))
        p = min(1.0, MAX_SAMPLE_SIZE / max(1, n_all))
        keep = rng.get_random().generator.random(n_local) < p
        if isinstance(x_local, torch.Tensor):
            samp = x_local[torch.from_numpy(keep).to(x_local.device)].double().cpu().numpy()
            d = int(x_local.shape[1]) if x_local.dim() == 2 else len(clusters[0].center)
        else:
            samp = np.asarray(x_local, dtype=np.float64)[keep]
            d = np.asarray(x_local).shape[1] if np.asarray(x_local).ndim == 2 else \
                len(clusters[0].center)
        parts = shuffle.all_gather_var(samp.reshape(-1), ctx)
        sample = np.concatenate(parts).reshape(-1, d)
        val = silhouette_coefficient(clusters, sample, device, max_sample=len(sample) + 1) \
            if ctx.is_main else 0.0
        return float(dist_.broadcast_object(val, ctx))
    stats = shuffle.all_reduce_np(local_cluster_stats(clusters, x_local, device), ctx)
    metrics = _metrics_from_arrays(clusters, stats[:, 0], stats[:, 1], stats[:, 2])
    if strategy == "SSE":
        return -math.fsum(m.sum_squared_dist for m in metrics.values())
    if strategy == "DAVIES_BOULDIN":
        return -_db_from(clusters, metrics)
    if strategy == "DUNN":
        return _dunn_from(clusters, metrics)
    raise ValueError("Unknown evaluation strategy " + strategy)


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
