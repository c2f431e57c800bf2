"""Random-decision-forest training and scoring on the device.

Replaces Spark MLlib ``RandomForest.trainClassifier/trainRegressor`` as invoked at
``[mllib]/rdf/RDFUpdate.java:140-158`` plus the node/feature example counting of
``RDFUpdate.treeNodeExampleCounts`` / ``predictorExampleCounts`` (``:269-333``); SURVEY.md
K12-K14.  The algorithm is MLlib's histogram (binned) level-wise random forest:

* continuous predictors are binned on quantile thresholds of a sample (<= max-split-candidates
  bins; features with fewer distinct values split between every value), categorical predictors
  use their encodings as bins;
* every tree gets Poisson(1) bootstrap weights (one tree: no bootstrap) and, at every node, a
  random feature subset ("auto": all features for one tree, sqrt(P) for classification, P/3 for
  regression);
* level by level, ALL trees at once: the HIP histogram kernel (``oryx_rdf_histogram``,
  csrc/kernels/rdf.hip) aggregates label statistics per (tree, node, feature, bin); the best
  split per node (max impurity decrease: gini / entropy / variance; categorical bins ordered by
  label centroid) is chosen with batched tensor ops; ``oryx_rdf_route`` moves every row one
  level down (and counts node visits unless the level's counting sort already did);
* a node becomes a leaf at max depth, when pure, with < 2 weighted examples, or when no split
  improves impurity.

Multi-GPU: histograms are additive, so ranks holding disjoint row slices all-reduce each
level's histogram (one RCCL call per level) and choose identical splits.

On CPU the same algorithm runs with ``index_add`` (tests / the ``local[*]`` plumbing path).
"""

from __future__ import annotations

import math
import time
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import native
from ..parallel import dist, watchdog
from ..utils import faults

__all__ = ["BinnedData", "bin_features", "train_forest", "TrainedForest", "FlatForest",
           "flatten_forest", "forest_leaves", "forest_vote"]

_HIST_BUDGET = 1 << 26          # floats per histogram pass (256 MB)
# GPU level histograms from rows grouped by node (counting sort per level); ORYX_RDF_GROUPED=0
# selects the scan-all-rows kernel
_GROUPED = os.environ.get("ORYX_RDF_GROUPED", "1") != "0"


@dataclass
class BinnedData:
    Xb: torch.Tensor                 # [n, P] uint8 or int16 bins
    n_bins: List[int]                # per predictor
    thresholds: List[Optional[np.ndarray]]   # numeric predictors: bin b is x <= thr[b]
    categorical: List[bool]
    B: int                           # max bins over predictors

    @property
    def bin_bytes(self) -> int:
        return self.Xb.element_size()

    def cat_flags(self) -> torch.Tensor:
        """Device copy of ``categorical`` (made once: a host list -> device tensor per level
        is a blocking copy)."""
        cf = getattr(self, "_cat_dev", None)
        if cf is None or cf.device != self.Xb.device:
            cf = torch.tensor(self.categorical, device=self.Xb.device)
            object.__setattr__(self, "_cat_dev", cf)
        return cf


def _quantile_thresholds(col: np.ndarray, max_bins: int) -> np.ndarray:
    u = np.unique(col)
    if len(u) <= max_bins:
        return u[:-1].astype(np.float64)
    qs = np.quantile(col, np.arange(1, max_bins) / max_bins, method="lower")
    thr = np.unique(qs)
    # never put the maximum as a threshold (nothing could go right of it)
    return thr[thr < u[-1]].astype(np.float64)


def _row_stride(P: int, dtype) -> int:
    """Row pitch (elements) of the binned matrix: byte rows padded to the next power of two up
    to 128 bytes, then to a multiple of 128, so that no row straddles a 128-byte cache line.
    The level histograms read each row of a node through the permutation -- 100-byte rows at
    arbitrary offsets touched 1.8 lines each on average, padded rows touch one."""
    if dtype != torch.uint8 or P <= 0:
        return max(P, 1)
    if P >= 128:
        return (P + 127) // 128 * 128
    s = 1
    while s < P:
        s *= 2
    return s


def bin_features(X, categorical: Sequence[bool], arities: Sequence[int], max_bins: int,
                 device, seed: int = 0, sample_size: Optional[int] = None,
                 threshold_source=None) -> BinnedData:
    """``X``: float64 [n, P] predictors (categorical as encodings).  Returns device bins.

    ``threshold_source``: the rows the split thresholds are computed from (default ``X``);
    ranks that bin disjoint slices of one data set pass the full data so that every rank
    gets identical bins.
    """
    on_device = isinstance(X, torch.Tensor)
    if not on_device:
        X = np.asarray(X, dtype=np.float64)
    n, P = X.shape
    src = X if threshold_source is None else threshold_source
    if not isinstance(src, torch.Tensor):
        src = np.asarray(src, dtype=np.float64)
    rng = np.random.default_rng(seed)
    ns = sample_size or max(10000, max_bins * max_bins)
    if len(src) <= ns:
        sample = src
    else:
        pick = np.sort(rng.choice(len(src), ns, replace=False))
        sample = src[torch.from_numpy(pick).to(src.device)] if isinstance(src, torch.Tensor) \
            else src[pick]
    if isinstance(sample, torch.Tensor):
        sample = sample.to(torch.float64).cpu().numpy()
    thresholds: List[Optional[np.ndarray]] = []
    n_bins: List[int] = []
    for f in range(P):
        if categorical[f]:
            thresholds.append(None)
            n_bins.append(max(1, int(arities[f])))
        else:
            thr = _quantile_thresholds(sample[:, f], max_bins)
            thresholds.append(thr)
            n_bins.append(len(thr) + 1)
    B = max(n_bins) if n_bins else 1
    dtype = torch.uint8 if B <= 256 else torch.int16
    Xb = torch.empty((n, _row_stride(P, dtype)), dtype=dtype, device=device)[:, :P]
    for f in range(P):
        col = X[:, f].to(device, torch.float64).contiguous() if on_device else \
            torch.from_numpy(np.ascontiguousarray(X[:, f])).to(device)
        if categorical[f]:
            b = col.to(torch.int64)
        else:
            thr = torch.from_numpy(thresholds[f]).to(device)
            # number of thresholds strictly below x: x <= thr[b] <=> bin <= b
            b = torch.searchsorted(thr, col, right=False) if len(thr) else \
                torch.zeros(n, dtype=torch.int64, device=device)
        Xb[:, f] = b.to(dtype)
    return BinnedData(Xb, n_bins, thresholds, list(categorical), B)


# ---------------------------------------------------------------- impurity

def _impurity(stats: torch.Tensor, kind: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """(impurity, weight) of label statistics [..., S]."""
    if kind == "variance":
        w = stats[..., 0]
        safe = w.clamp_min(1e-30)
        mean = stats[..., 1] / safe
        imp = (stats[..., 2] / safe - mean * mean).clamp_min(0)
        return imp, w
    w = stats.sum(-1)
    p = stats / w.clamp_min(1e-30).unsqueeze(-1)
    if kind == "gini":
        imp = 1.0 - (p * p).sum(-1)
    else:   # entropy (log base 2, as MLlib)
        imp = -(p * torch.log2(p.clamp_min(1e-30))).sum(-1)
    return imp, w


@dataclass
class LevelSplits:
    feat: torch.Tensor       # [T, N] predictor index or -1 (leaf)
    bin: torch.Tensor        # [T, N] numeric: last bin going left; -1 categorical
    cat_left: Optional[torch.Tensor]   # [T, N, B] uint8
    totals: torch.Tensor     # [T, N, S] label statistics of the node (weighted)
    gain: torch.Tensor       # [T, N]


def _choose_splits(hist: torch.Tensor, feats: torch.Tensor, data: BinnedData, kind: str,
                   force_leaf: bool) -> LevelSplits:
    T, N, Fs, B, S = hist.shape
    dev = hist.device
    if kind == "variance":
        hist = hist.double()        # cumsum / E[y^2] - mean^2 in fp64 (MLlib's aggregator)
    totals = hist[:, :, 0].sum(2)                                   # [T, N, S]
    parent_imp, w = _impurity(totals, kind)                         # [T, N]
    if B < 2:
        none = torch.full((T, N), -1, dtype=torch.int64, device=dev)
        return LevelSplits(none, none.clone(), None, totals, torch.zeros((T, N), device=dev))
    any_cat = any(data.categorical)                                 # host: no device sync
    cat_flag = data.cat_flags()[feats]                              # [T, N, Fs]
    h = hist
    order = None
    if any_cat:
        # categorical bins ordered by label centroid (regression: mean; classification:
        # share of the node's majority class); empty bins last
        if kind == "variance":
            cen = h[..., 1] / h[..., 0].clamp_min(1e-30)
            empty = h[..., 0] <= 0
        else:
            maj = totals.argmax(-1)                                 # [T, N]
            cnt = h.sum(-1)
            sel = h.gather(-1, maj[:, :, None, None, None].expand(T, N, Fs, B, 1))[..., 0]
            cen = sel / cnt.clamp_min(1e-30)
            empty = cnt <= 0
        cen = torch.where(empty, torch.full_like(cen, float("inf")), cen)
        ident = torch.arange(B, device=dev).expand(T, N, Fs, B)
        order = torch.where(cat_flag[..., None], torch.argsort(cen, dim=-1, stable=True), ident)
        h = h.gather(3, order[..., None].expand(T, N, Fs, B, S))
    left = torch.cumsum(h, dim=3)[:, :, :, :-1]                     # split after position k
    right = totals[:, :, None, None, :] - left
    imp_l, w_l = _impurity(left, kind)
    imp_r, w_r = _impurity(right, kind)
    wt = w[:, :, None, None].clamp_min(1e-30)
    gain = parent_imp[:, :, None, None] - (w_l * imp_l + w_r * imp_r) / wt
    valid = (w_l >= 1.0) & (w_r >= 1.0)
    gain = torch.where(valid, gain, torch.full_like(gain, float("-inf")))
    flat = gain.reshape(T, N, Fs * (B - 1))
    best, arg = flat.max(-1)
    j = arg // (B - 1)
    k = arg % (B - 1)
    leaf = (best <= 1e-12) | (w < 2.0) | (parent_imp <= 1e-12) | torch.isinf(best)
    if force_leaf:
        leaf = torch.ones_like(leaf)
    feat = torch.where(leaf, torch.full_like(j, -1), feats.gather(2, j[..., None])[..., 0])
    is_cat = cat_flag.gather(2, j[..., None])[..., 0] & ~leaf
    sbin = torch.where(is_cat | leaf, torch.full_like(k, -1), k)
    cat_left = None
    if any_cat:
        # left set = the first k+1 categories in centroid order
        o = order.gather(2, j[:, :, None, None].expand(T, N, 1, B))[:, :, 0]   # [T, N, B]
        pos_in_order = torch.empty_like(o)
        pos_in_order.scatter_(2, o, torch.arange(B, device=dev).expand(T, N, B))
        cat_left = ((pos_in_order <= k[..., None]) & is_cat[..., None]).to(torch.uint8)
    return LevelSplits(feat, sbin, cat_left, totals, torch.where(leaf, torch.zeros_like(best),
                                                                 best))


_KIND = {"gini": 0, "entropy": 1, "variance": 2}


def _check_split_err(err: torch.Tensor, depth: int, ctx) -> None:
    """Raise when the split search met a non-finite histogram entry (synchronises).  Bootstrap
    counts, label counts and label sums are finite by construction, so a NaN / inf there means
    the level's (all-reduced) statistics are corrupt; trees grown from them would be silently
    wrong."""
    if int(err.item()):
        err.zero_()
        raise RuntimeError("RDF level %d: non-finite split statistics on rank %d%s"
                           % (depth, ctx.rank, " (after the all-reduce)" if ctx.is_distributed
                              else ""))


def _split_kernel_ok(data: BinnedData, S: int) -> bool:
    return S <= 32 and (not any(data.categorical) or 64 * data.B * 2 <= 64 * 1024)


def _choose_splits_kernel(hist: torch.Tensor, feats: torch.Tensor, data: BinnedData, kind: str,
                          force_leaf: bool, err: Optional[torch.Tensor] = None) -> LevelSplits:
    """:func:`_choose_splits` as one HIP kernel (``rdf_best_split``: a wave per node, a lane
    per candidate feature, fp64 prefix sums and gains) instead of ~25 tensor ops over
    [T, N, Fs, B, S] temporaries.  ``err`` (int32 [1], optional) is set to 1 when a node's
    histogram holds a non-finite value (see :func:`_check_split_err`)."""
    T, N, Fs, B, S = hist.shape
    dev = hist.device
    lib = native.require_kernels()
    h = hist.contiguous()
    fe = feats.contiguous()
    cat = data.cat_flags().to(torch.uint8) if any(data.categorical) else None
    feat = torch.empty((T, N), dtype=torch.int32, device=dev)
    sbin = torch.empty((T, N), dtype=torch.int32, device=dev)
    tot = torch.empty((T, N, S), dtype=torch.float64, device=dev)
    gain = torch.empty((T, N), dtype=torch.float32, device=dev)
    cl = torch.empty((T, N, B), dtype=torch.uint8, device=dev) if cat is not None else None
    rc = lib.oryx_rdf_best_split(h.data_ptr(), fe.data_ptr(),
                                 cat.data_ptr() if cat is not None else None, T, N, Fs, B, S,
                                 _KIND[kind], int(bool(force_leaf)), feat.data_ptr(),
                                 sbin.data_ptr(), tot.data_ptr(), gain.data_ptr(),
                                 cl.data_ptr() if cl is not None else None,
                                 err.data_ptr() if err is not None else None,
                                 native.stream_ptr(dev))
    native.check(rc, "oryx_rdf_best_split")
    return LevelSplits(feat.long(), sbin.long(), cl, tot, gain)


# ---------------------------------------------------------------- histogram / route

def _histogram(data: BinnedData, label, y, S, cls, weight, node_of, lo, nodes, feats, B):
    T = node_of.shape[0]
    Fs = feats.shape[2]
    dev = node_of.device
    hist = torch.zeros((T, nodes, Fs, B, S), dtype=torch.float32, device=dev)
    n, P = data.Xb.shape
    if dev.type == "cuda":
        lib = native.require_kernels()
        rc = lib.oryx_rdf_histogram(
            data.Xb.data_ptr(), data.bin_bytes, n, data.Xb.stride(0),
            label.data_ptr() if cls else None, None if cls else y.data_ptr(), S, int(cls),
            weight.data_ptr() if weight is not None else None, T, node_of.data_ptr(), lo,
            nodes, feats.contiguous().data_ptr(), Fs, B, hist.data_ptr(),
            native.stream_ptr(dev))
        native.check(rc, "oryx_rdf_histogram")
        return hist
    flat = hist.view(-1)
    for t in range(T):
        nd = node_of[t] - lo
        m = (nd >= 0) & (nd < nodes)
        if weight is not None:
            m &= weight[t] > 0
        rows = torch.nonzero(m).flatten()
        if rows.numel() == 0:
            continue
        nd = nd[rows].long()
        w = weight[t][rows].float() if weight is not None else torch.ones(rows.numel())
        fsel = feats[t][nd]                                          # [m, Fs]
        bins = data.Xb[rows[:, None], fsel].long()                   # [m, Fs]
        jj = torch.arange(Fs)[None, :]
        base = ((((t * nodes + nd[:, None]) * Fs + jj) * B + bins) * S)   # [m, Fs]
        if cls:
            idx = base + label[rows].long()[:, None]
            flat.index_add_(0, idx.flatten(), w[:, None].expand(-1, Fs).flatten())
        else:
            yy = y[rows].float()
            for s_, v in enumerate((w, w * yy, w * yy * yy)):
                flat.index_add_(0, (base + s_).flatten(), v[:, None].expand(-1, Fs).flatten())
    return hist


_PIECE = int(os.environ.get("ORYX_RDF_PIECE", "16384"))   # rows per histogram workgroup
_SORT_MAX_KEYS = 16384


class RowGroups:
    """Rows of every tree grouped by their open node at the current level (GPU path): a
    permutation of the flattened [T][n] row space plus per-(tree, node) counts/offsets."""

    def __init__(self, perm: Optional[torch.Tensor], counts: np.ndarray, width: int, n: int,
                 visits: Optional[np.ndarray] = None):
        self.perm = perm                      # int32 [T*n] (None: identity, one node per tree)
        self.counts = counts                  # int64 [T, width]: rows with weight > 0
        self.width = width
        self.n = n
        # int64 [T, width]: every row at the node, bootstrap weight 0 included (the PMML
        # recordCount / importance input that routing would otherwise count)
        self.visits = visits
        flat = counts.reshape(-1)
        self.offsets = (np.cumsum(flat) - flat).reshape(counts.shape)

    @staticmethod
    def root(T: int, n: int) -> "RowGroups":
        g = RowGroups(None, np.full((T, 1), n, dtype=np.int64), 1, n,
                      np.full((T, 1), n, dtype=np.int64))
        g.offsets = (np.arange(T, dtype=np.int64) * n)[:, None]
        return g

    @staticmethod
    def from_nodes(node_of: torch.Tensor, width: int,
                   weight: Optional[torch.Tensor] = None) -> Optional["RowGroups"]:
        finish = RowGroups.launch_from_nodes(node_of, width, weight)
        return finish() if finish is not None else None

    @staticmethod
    def launch_from_nodes(node_of: torch.Tensor, width: int,
                          weight: Optional[torch.Tensor] = None,
                          keys: Optional[torch.Tensor] = None):
        """Queue the level's counting sort on the device and return ``finish()`` (which waits
        for the counts and builds the RowGroups), or None when the key space is too wide; the
        host can do other work between the two."""
        """Counting sort of the rows by (tree, node); None when the key space is too wide.
        Rows a tree's bootstrap left out (weight 0) only count as node visits: they get a
        second key per node after all live keys, and rows that reached a leaf a last, unused
        key, so one sort yields both the live groups and the visit counts."""
        T, n = node_of.shape
        k = 2 * T * width + 1
        if k > _SORT_MAX_KEYS or T * n >= (1 << 31):
            return None
        dev = node_of.device
        lib = native.require_kernels()
        if keys is None:       # (given: written by the fused route, rdf_route_rows<KEYS>)
            keys = torch.empty(T * n, dtype=torch.int32, device=dev)
            w = weight.contiguous() if weight is not None else None
            rc = lib.oryx_rdf_sort_keys(node_of.contiguous().data_ptr(),
                                        w.data_ptr() if w is not None else None, T, n, width,
                                        keys.data_ptr(), native.stream_ptr(dev))
            native.check(rc, "oryx_rdf_sort_keys")
        perm = torch.empty(T * n, dtype=torch.int32, device=dev)
        counts = torch.empty(k, dtype=torch.int64, device=dev)
        ws = torch.empty(int(lib.oryx_kmeans_sorted_ws_bytes(T * n, k)), dtype=torch.uint8,
                         device=dev)
        rc = lib.oryx_counting_sort(keys.data_ptr(), T * n, k, perm.data_ptr(),
                                    counts.data_ptr(), ws.data_ptr(), native.stream_ptr(dev))
        native.check(rc, "oryx_counting_sort")

        def finish() -> "RowGroups":
            c = counts.cpu().numpy()[:-1]
            live = c[:T * width].reshape(T, width)
            return RowGroups(perm, live, width, n, live + c[T * width:].reshape(T, width))

        def device():
            """(perm, live counts [T*width], visits [T, width]) left on the device."""
            live = counts[:T * width]
            return perm, live, (live + counts[T * width:2 * T * width]).view(T, width)
        finish.device = device
        return finish

    def pieces(self, lo: int, hi: int, dev):
        """(tree, node - lo, begin, end) of every PIECE-row slice of nodes [lo, hi)."""
        cnt = self.counts[:, lo:hi]
        off = self.offsets[:, lo:hi]
        npc = (cnt + _PIECE - 1) // _PIECE
        tot = int(npc.sum())
        if tot == 0:
            return None
        T, W = cnt.shape
        t_idx = np.repeat(np.repeat(np.arange(T), W), npc.reshape(-1))
        n_idx = np.repeat(np.tile(np.arange(W), T), npc.reshape(-1))
        first = np.repeat(np.cumsum(npc.reshape(-1)) - npc.reshape(-1), npc.reshape(-1))
        k = np.arange(tot) - first
        begin = np.repeat(off.reshape(-1), npc.reshape(-1)) + k * _PIECE
        end = np.minimum(begin + _PIECE, np.repeat((off + cnt).reshape(-1), npc.reshape(-1)))
        to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a.astype(dt))).to(dev)
        return (to(t_idx, np.int32), to(n_idx, np.int32), to(begin, np.int64),
                to(end, np.int64), tot)


def _histogram_groups(data: BinnedData, label, y, S, cls, weight, groups: RowGroups, lo, nodes,
                      feats, B, T):
    """Level histogram of node slots [lo, lo + nodes) from grouped rows (GPU)."""
    Fs = feats.shape[2]
    dev = data.Xb.device
    hist = torch.zeros((T, nodes, Fs, B, S), dtype=torch.float32, device=dev)
    pc = groups.pieces(lo, lo + nodes, dev)
    if pc is None:
        return hist
    pt, pn, pb, pe, tot = pc
    n, P = data.Xb.shape
    lib = native.require_kernels()
    fe = feats.contiguous()
    rc = lib.oryx_rdf_histogram_pieces(
        data.Xb.data_ptr(), data.bin_bytes, n, data.Xb.stride(0), P,
        label.data_ptr() if cls else None,
        None if cls else y.data_ptr(), S, int(cls),
        weight.data_ptr() if weight is not None else None,
        groups.perm.data_ptr() if groups.perm is not None else None,
        pt.data_ptr(), pn.data_ptr(), pb.data_ptr(), pe.data_ptr(), tot, nodes, fe.data_ptr(),
        Fs, B, hist.data_ptr(), None, native.stream_ptr(dev))
    native.check(rc, "oryx_rdf_histogram_pieces")
    return hist


def _route(data: BinnedData, node_of, nodes, split: LevelSplits, child_base, B,
           count_visits: bool = True):
    """Move every open row one level down; returns the per-node visit counts (None on the
    GPU when ``count_visits`` is off: the grouped path already has them)."""
    T, n = node_of.shape
    dev = node_of.device
    visits = torch.zeros((T, nodes), dtype=torch.int64, device=dev) \
        if count_visits or dev.type != "cuda" else None
    if dev.type == "cuda":
        lib = native.require_kernels()
        # keep every converted operand alive until the launch: a temporary freed mid-call
        # could be recycled (and overwritten) by the next conversion before the kernel runs
        cl = split.cat_left.contiguous() if split.cat_left is not None else None
        sf = split.feat.int().contiguous()
        sb = split.bin.int().contiguous()
        cb = child_base.int().contiguous()
        rc = lib.oryx_rdf_route(data.Xb.data_ptr(), data.bin_bytes, n, data.Xb.stride(0),
                                data.Xb.shape[1], T,
                                node_of.data_ptr(), nodes, sf.data_ptr(), sb.data_ptr(),
                                cl.data_ptr() if cl is not None else None, B, cb.data_ptr(),
                                visits.data_ptr() if visits is not None else None,
                                native.stream_ptr(dev))
        native.check(rc, "oryx_rdf_route")
        return visits
    for t in range(T):
        nd = node_of[t]
        act = nd >= 0
        rows = torch.nonzero(act).flatten()
        ndr = nd[rows].long()
        visits[t] += torch.bincount(ndr, minlength=nodes)
        f = split.feat[t][ndr]
        leafm = f < 0
        fb = data.Xb[rows, f.clamp_min(0)].long()
        if split.cat_left is not None:
            catm = split.bin[t][ndr] < 0
            go_left_cat = split.cat_left[t][ndr, fb] > 0
            right = torch.where(catm, ~go_left_cat, fb > split.bin[t][ndr])
        else:
            right = fb > split.bin[t][ndr]
        new = child_base[t][ndr] + right.long()
        new = torch.where(leafm, torch.full_like(new, -1), new)
        node_of[t][rows] = new.to(node_of.dtype)
    return visits


# ---------------------------------------------------------------- training

@dataclass(slots=True)
class TrainedNode:
    id: str
    count: int = 0                  # unweighted training examples reaching the node
    stats: Optional[np.ndarray] = None     # weighted label statistics
    feature: int = -1               # predictor index, -1 = leaf
    bin: int = -1
    cat_left: Optional[np.ndarray] = None  # categorical: encodings going left
    left: Optional["TrainedNode"] = None
    right: Optional["TrainedNode"] = None


@dataclass
class TrainedForest:
    roots: List[TrainedNode]
    predictor_counts: np.ndarray    # visits of decision nodes, by predictor (importances)
    classification: bool


def _feature_subset_size(P: int, num_trees: int, classification: bool) -> int:
    if num_trees == 1:
        return P
    if classification:
        return min(P, max(1, int(math.ceil(math.sqrt(P)))))
    return min(P, max(1, int(math.ceil(P / 3.0))))


def train_forest(data: BinnedData, target: torch.Tensor, num_classes: int, num_trees: int,
                 max_depth: int, impurity: str, seed: int = 0,
                 ctx: Optional[dist.DistContext] = None,
                 feature_subset: Optional[int] = None,
                 timings: Optional[dict] = None) -> TrainedForest:
    """``target``: int class encodings (``num_classes`` > 0) or float values (regression).
    ``timings``: seconds per phase are added to it (``prep`` -- targets and bootstrap
    weights, ``levels`` -- the level loop with the overlapped host node builds, ``tail`` --
    the last level's node build), each closed by a device synchronize."""
    t_mark = [time.perf_counter()]

    def lap(name):
        if timings is None:
            return
        if data.Xb.device.type == "cuda":
            torch.cuda.synchronize(data.Xb.device)
        t = time.perf_counter()
        timings[name] = timings.get(name, 0.0) + t - t_mark[0]
        t_mark[0] = t
    classification = num_classes > 0
    kind = impurity if classification else "variance"
    if classification and kind not in ("gini", "entropy"):
        raise ValueError("impurity must be gini or entropy for classification")
    dev = data.Xb.device
    n, P = data.Xb.shape
    T = int(num_trees)
    B = data.B
    S = num_classes if classification else 3
    ctx = ctx or dist.DistContext(device=dev)
    g = torch.Generator(device="cpu")
    g.manual_seed(seed & ((1 << 62) - 1))
    label = target.to(dev, torch.int32).contiguous() if classification else None
    y = None
    y_shift = 0.0
    if not classification:
        # regression statistics (sum w, sum wy, sum wy^2) are accumulated in fp32 on the
        # device: centre the targets on their global mean first so that E[y^2] - mean^2 does
        # not cancel for targets with a large offset (the split search then runs in fp64)
        yd = target.to(dev, torch.float64)
        s = torch.stack([yd.sum(), torch.tensor(float(n), dtype=torch.float64, device=dev)])
        if ctx.is_distributed:
            dist.all_reduce_sum(s, ctx)
        y_shift = float(s[0] / s[1].clamp_min(1.0))
        y = (yd - y_shift).to(torch.float32).contiguous()
    if T > 1 and dev.type == "cuda":
        # one fused pass (rdf_poisson_weights: hashed uniforms through the Poisson(1) inverse
        # CDF, uint8 out) instead of rand + bucketize + cast over T x n
        weight = torch.empty((T, n), dtype=torch.uint8, device=dev)
        native.check(native.require_kernels().oryx_rdf_poisson_weights(
            (seed * 31 + ctx.rank + 7) & ((1 << 64) - 1), T * n, weight.data_ptr(),
            native.stream_ptr(dev)), "oryx_rdf_poisson_weights")
    elif T > 1:
        gd = torch.Generator(device=dev)
        gd.manual_seed((seed * 31 + ctx.rank + 7) & ((1 << 62) - 1))
        # Poisson(1) bootstrap counts by inverse CDF of one uniform per (tree, row): same
        # distribution as torch.poisson (the rejection sampler), a fraction of its time
        k = torch.arange(24, dtype=torch.float64)
        cdf = torch.cumsum(torch.exp(-1.0 - torch.lgamma(k + 1.0)), 0)[:-1].to(torch.float32)
        u = torch.rand((T, n), generator=gd, device=dev)
        weight = torch.bucketize(u, cdf.to(dev), right=True).to(torch.uint8)
    else:
        weight = None
    Fs = feature_subset or _feature_subset_size(P, T, classification)
    if dev.type == "cuda" and _GROUPED and _DEVICE_LOOP and T * (1 << max_depth) <= 8191 and \
            n * T < (1 << 31) and _split_kernel_ok(data, S):
        lap("prep")
        return _train_device(data, label, y, y_shift, S, classification, kind, weight, T, Fs,
                             max_depth, seed, ctx, lap)
    lap("prep")
    node_of = torch.zeros((T, n), dtype=torch.int32, device=dev)
    roots = [TrainedNode("r") for _ in range(T)]
    level_nodes: List[List[Optional[TrainedNode]]] = [[r] for r in roots]
    predictor_counts = np.zeros(P, dtype=np.float64)
    nodes = 1
    groups = RowGroups.root(T, n) if dev.type == "cuda" and _GROUPED else None

    def sample_feats(width: int) -> torch.Tensor:
        # Fs smallest of P uniforms per node, in order: the same subsets as a full argsort
        # prefix, at a third of the host time
        if Fs < P:
            f = torch.topk(torch.rand((T, width, P), generator=g), Fs, dim=-1, largest=False,
                           sorted=True).indices
        else:
            f = torch.arange(P).expand(T, width, P)
        return f.to(torch.int32).to(dev).contiguous()

    def build_level(level_nodes, feat_h, bin_h, tot_h, vis_h, cat_h, width_next):
        new_level: List[List[Optional[TrainedNode]]] = []
        next_nodes = 0
        for t in range(T):
            row: List[Optional[TrainedNode]] = []
            for slot, node in enumerate(level_nodes[t]):
                if node is None:
                    continue
                node.count = int(vis_h[t, slot])
                node.stats = tot_h[t, slot]
                f = int(feat_h[t, slot])
                if f >= 0:
                    node.feature = f
                    node.bin = int(bin_h[t, slot])
                    if node.bin < 0:
                        node.cat_left = np.nonzero(cat_h[t, slot])[0]
                    node.left = TrainedNode(node.id + "-")
                    node.right = TrainedNode(node.id + "+")
                    row.extend([node.left, node.right])
                    predictor_counts[f] += node.count
            new_level.append(row)
            next_nodes = max(next_nodes, len(row))
        assert next_nodes == width_next, (next_nodes, width_next)
        return new_level

    # The host tree of level d is built after level d + 1's device work is queued (the
    # GPU builds histograms while Python allocates nodes); next-level feature subsets are
    # drawn while the device runs the level's counting sort.
    pending = None
    feats = sample_feats(nodes)
    for depth in range(max_depth + 1):
        faults.point("rdf.level", depth=depth, rank=ctx.rank)
        watchdog.heartbeat("rdf.level")
        # histogram in node chunks that fit the budget
        chunk = max(1, _HIST_BUDGET // max(1, T * Fs * B * S))
        splits = []
        nonfinite = torch.zeros((), dtype=torch.bool, device=dev)
        for lo in range(0, nodes, chunk):
            hi = min(nodes, lo + chunk)
            if groups is not None:
                hist = _histogram_groups(data, label, y, S, classification, weight, groups, lo,
                                         hi - lo, feats[:, lo:hi], B, T)
            else:
                hist = _histogram(data, label, y, S, classification, weight, node_of, lo,
                                  hi - lo, feats[:, lo:hi], B)
            if ctx.is_distributed:
                dist.all_reduce_sum(hist, ctx)
                # see _check_split_err: read with the level's one host transfer below
                nonfinite = nonfinite | ~torch.isfinite(hist).all()
            splits.append(_choose_splits(hist, feats[:, lo:hi], data, kind,
                                         force_leaf=depth == max_depth))
        split = LevelSplits(
            torch.cat([s.feat for s in splits], 1), torch.cat([s.bin for s in splits], 1),
            None if all(s.cat_left is None for s in splits) else torch.cat(
                [s.cat_left if s.cat_left is not None else
                 torch.zeros((T, s.feat.shape[1], B), dtype=torch.uint8, device=dev)
                 for s in splits], 1),
            torch.cat([s.totals for s in splits], 1), torch.cat([s.gain for s in splits], 1))
        is_split = split.feat >= 0
        rank = torch.cumsum(is_split.int(), 1) - is_split.int()
        child_base = torch.where(is_split, 2 * rank, torch.full_like(rank, -1))
        if groups is not None and groups.visits is not None:
            _route(data, node_of, nodes, split, child_base, B, count_visits=False)
            visits = torch.from_numpy(np.ascontiguousarray(groups.visits[:, :nodes])).to(dev)
        else:
            visits = _route(data, node_of, nodes, split, child_base, B)
        if ctx.is_distributed:
            dist.all_reduce_sum(visits, ctx)
        if pending is not None:
            level_nodes = build_level(*pending)
            pending = None
        # one device -> host transfer (one sync) for everything the host tree needs
        parts = [split.feat.double().reshape(T, -1), split.bin.double().reshape(T, -1),
                 split.totals.double().reshape(T, -1), visits.double().reshape(T, -1)]
        if split.cat_left is not None:
            parts.append(split.cat_left.double().reshape(T, -1))
        host = torch.cat(parts, 1).cpu().numpy()
        if ctx.is_distributed:
            dist.check_collectives(ctx)      # see _train_device
            _check_split_err(nonfinite.int().reshape(1), depth, ctx)
        w = [p_.shape[1] for p_ in parts]
        cut = np.cumsum([0] + w)
        feat_h = host[:, cut[0]:cut[1]].astype(np.int64)
        bin_h = host[:, cut[1]:cut[2]].astype(np.int64)
        tot_h = host[:, cut[2]:cut[3]].reshape(split.totals.shape)
        if y_shift:
            # un-centre the node statistics: sum w(y'+m)^2 and sum w(y'+m)
            w_, s1 = tot_h[..., 0].copy(), tot_h[..., 1].copy()
            tot_h[..., 2] += 2.0 * y_shift * s1 + y_shift * y_shift * w_
            tot_h[..., 1] += y_shift * w_
        vis_h = host[:, cut[3]:cut[4]].astype(np.int64)
        cat_h = host[:, cut[4]:cut[5]].reshape(split.cat_left.shape).astype(np.uint8) \
            if split.cat_left is not None else None
        # next level's width from the split flags (padding slots of narrower trees are leaves),
        # so its counting sort is queued on the device before anything else on the host
        width_next = int(2 * (feat_h >= 0).sum(1).max()) if feat_h.size else 0
        finish_groups = None
        if groups is not None and width_next > 0:
            finish_groups = RowGroups.launch_from_nodes(node_of, width_next, weight)
        pending = (level_nodes, feat_h, bin_h, tot_h, vis_h, cat_h, width_next)
        nodes = width_next
        if nodes == 0:
            break
        feats = sample_feats(nodes)
        if groups is not None:
            groups = finish_groups() if finish_groups is not None else None
    if pending is not None:
        build_level(*pending)
    watchdog.get().end_heartbeats()
    lap("levels")
    return TrainedForest(roots, predictor_counts, classification)


_DEVICE_LOOP = os.environ.get("ORYX_RDF_DEVICE_LOOP", "1") != "0"
# device pieces ordered by first row (trees over the same rows on one XCD); 0: slot order
_ROW_ORDER = os.environ.get("ORYX_RDF_ROW_ORDER", "1") != "0"


def _totals_ok(width: int, S: int) -> bool:
    """The last level's node totals fit rdf_node_totals' LDS (width x (S + 1) words)."""
    return width * (S + 1) * 4 <= 64 * 1024


def _train_device(data: BinnedData, label, y, y_shift: float, S: int, classification: bool,
                  kind: str, weight, T: int, Fs: int, max_depth: int, seed: int,
                  ctx: dist.DistContext, lap=None) -> TrainedForest:
    """The level loop with no host round trip inside it (GPU, forests whose widest level fits
    the counting sort's key space).  Level d has 2^d node slots per tree (slots past a tree's
    real nodes stay empty: no rows, so no pieces, and they come out as leaves); per level the
    device runs: feature subsets (device RNG), the piece list from the previous level's
    counting sort (``rdf_expand_pieces``), the grouped histogram (grid = an upper bound on
    the pieces, surplus workgroups retire on the device-side count), the split search
    (``rdf_best_split``), child numbering, routing and the next level's counting sort.  Each
    level's splits / totals / visits go to pinned host memory asynchronously with an event;
    the host builds level d's nodes while the device is already working on later levels."""
    dev = data.Xb.device
    n, P = data.Xb.shape
    B = data.B
    lib = native.require_kernels()
    stream = native.stream_ptr(dev)
    gf = torch.Generator(device=dev)
    gf.manual_seed((seed * 977 + 13) & ((1 << 62) - 1))
    node_of = torch.zeros((T, n), dtype=torch.int32, device=dev)
    roots = [TrainedNode("r") for _ in range(T)]
    level_nodes: List[List[Optional[TrainedNode]]] = [[r] for r in roots]
    predictor_counts = np.zeros(P, dtype=np.float64)
    # root: every row of a tree is one group (identity permutation)
    counts = torch.full((T,), n, dtype=torch.int64, device=dev)
    visits = torch.full((T, 1), n, dtype=torch.int64, device=dev)
    perm = None
    pending = []
    any_cat = any(data.categorical)
    split_err = torch.zeros(1, dtype=torch.int32, device=dev)

    def sample_feats(width: int) -> torch.Tensor:
        if Fs < P:
            r = torch.rand((T, width, P), generator=gf, device=dev)
            return torch.topk(r, Fs, dim=-1, largest=False, sorted=True).indices \
                .to(torch.int32).contiguous()
        return torch.arange(P, dtype=torch.int32, device=dev).expand(T, width, P).contiguous()

    def build(lv) -> None:
        nonlocal level_nodes
        lv["event"].synchronize()
        tot_h = lv["tot"].numpy().copy()
        if y_shift:
            w_, s1 = tot_h[..., 0].copy(), tot_h[..., 1].copy()
            tot_h[..., 2] += 2.0 * y_shift * s1 + y_shift * y_shift * w_
            tot_h[..., 1] += y_shift * w_
        # Python lists (scalar access on numpy arrays costs more than the node itself)
        feat_l = lv["feat"].numpy().tolist()
        bin_l = lv["bin"].numpy().tolist()
        vis_l = lv["vis"].numpy().tolist()
        cat_h = lv["cat"].numpy() if lv["cat"] is not None else None
        np.add.at(predictor_counts, lv["feat"].numpy()[lv["feat"].numpy() >= 0],
                  lv["vis"].numpy()[lv["feat"].numpy() >= 0])
        # label statistics stay numpy row views (not containers the cyclic GC tracks: as
        # Python lists, ~10^4 more tracked objects per forest made the collector's passes
        # over the live trees cost more than the build itself)
        tot_l = tot_h
        new_level: List[List[Optional[TrainedNode]]] = []
        TN = TrainedNode
        for t in range(T):
            row: List[Optional[TrainedNode]] = []
            app = row.append
            for slot, (node, f, b, c, st) in enumerate(zip(level_nodes[t], feat_l[t], bin_l[t],
                                                          vis_l[t], tot_l[t])):
                node.count = c
                node.stats = st
                if f >= 0:
                    node.feature = f
                    node.bin = b
                    if b < 0:
                        node.cat_left = np.nonzero(cat_h[t, slot])[0]
                    nid = node.id
                    node.left = left = TN(nid + "-")
                    node.right = right = TN(nid + "+")
                    app(left)
                    app(right)
            new_level.append(row)
        level_nodes = new_level

    def to_host(t: torch.Tensor) -> torch.Tensor:
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        return h

    W = 1
    for depth in range(max_depth + 1):
        faults.point("rdf.level", depth=depth, rank=ctx.rank)
        watchdog.heartbeat("rdf.level")
        last = depth == max_depth and _totals_ok(W, S)
        feats = sample_feats(W) if not last else None
        chunk = max(1, _HIST_BUDGET // max(1, T * Fs * B * S))
        parts = []
        if last:
            # last level: every node becomes a leaf, so only its label totals (and visits) are
            # needed -- one coalesced pass over node_of / weights / labels, no bin-matrix
            # reads and no counting sort before it
            tot = torch.zeros((T, W, 1, 1, S), dtype=torch.float32, device=dev)
            visits = torch.zeros((T, W), dtype=torch.int64, device=dev)
            native.check(lib.oryx_rdf_node_totals(
                node_of.data_ptr(), weight.data_ptr() if weight is not None else None,
                label.data_ptr() if classification else None,
                None if classification else y.data_ptr(), S, int(classification), T, n, W,
                tot.data_ptr(), visits.data_ptr(), stream), "oryx_rdf_node_totals")
            if ctx.is_distributed:
                dist.all_reduce_sum(tot, ctx)
            parts.append(_choose_splits_kernel(
                tot, torch.zeros((T, W, 1), dtype=torch.int32, device=dev), data, kind,
                force_leaf=True, err=split_err))
        for lo in range(0, W if not last else 0, chunk):
            hi = min(W, lo + chunk)
            max_pieces = (T * n + _PIECE - 1) // _PIECE + T * (hi - lo)
            ptree = torch.empty(max_pieces, dtype=torch.int32, device=dev)
            pnode = torch.empty(max_pieces, dtype=torch.int32, device=dev)
            pbeg = torch.empty(max_pieces, dtype=torch.int64, device=dev)
            pend = torch.empty(max_pieces, dtype=torch.int64, device=dev)
            n_live = torch.empty(1, dtype=torch.int32, device=dev)
            native.check(lib.oryx_rdf_expand_pieces(
                counts.data_ptr(), T, W, lo, hi, _PIECE, max_pieces, ptree.data_ptr(),
                pnode.data_ptr(), pbeg.data_ptr(), pend.data_ptr(), n_live.data_ptr(), stream),
                "oryx_rdf_expand_pieces")
            # pieces in order of their first row (trees interleaved): the workgroups that run
            # together read the same rows, which then come from L2 / MALL instead of HBM
            if _ROW_ORDER:
                live = torch.arange(max_pieces, device=dev) < n_live
                first = pbeg.clamp(0, T * n - 1)
                row0 = (perm[first].long() if perm is not None else first) % n
                key = torch.where(live, row0 * T + ptree.long().clamp(0, T - 1),
                                  torch.full_like(row0, 1 << 62))
                order = torch.argsort(key)
                ptree, pnode = ptree[order].contiguous(), pnode[order].contiguous()
                pbeg, pend = pbeg[order].contiguous(), pend[order].contiguous()
            fe = feats[:, lo:hi].contiguous()
            hist = torch.zeros((T, hi - lo, Fs, B, S), dtype=torch.float32, device=dev)
            native.check(lib.oryx_rdf_histogram_pieces(
                data.Xb.data_ptr(), data.bin_bytes, n, data.Xb.stride(0), P,
                label.data_ptr() if classification else None,
                None if classification else y.data_ptr(), S, int(classification),
                weight.data_ptr() if weight is not None else None,
                perm.data_ptr() if perm is not None else None, ptree.data_ptr(),
                pnode.data_ptr(), pbeg.data_ptr(), pend.data_ptr(), max_pieces, hi - lo,
                fe.data_ptr(), Fs, B, hist.data_ptr(), n_live.data_ptr(), stream),
                "oryx_rdf_histogram_pieces")
            if ctx.is_distributed:
                dist.all_reduce_sum(hist, ctx)
            parts.append(_choose_splits_kernel(hist, fe, data, kind,
                                               force_leaf=depth == max_depth, err=split_err))
            del hist
        if len(parts) == 1:
            split = parts[0]
        else:
            split = LevelSplits(torch.cat([q.feat for q in parts], 1),
                                torch.cat([q.bin for q in parts], 1),
                                torch.cat([q.cat_left for q in parts], 1) if any_cat else None,
                                torch.cat([q.totals for q in parts], 1),
                                torch.cat([q.gain for q in parts], 1))
        is_split = split.feat >= 0
        rank = torch.cumsum(is_split.int(), 1) - is_split.int()
        child_base = torch.where(is_split, 2 * rank, torch.full_like(rank, -1))
        # sparse level state: children are numbered densely per tree, so the next level
        # needs 2 * (most splits in any tree) slots, not 2^(depth + 1) -- one small host read
        # per level sizes every later histogram, split search and all-reduce to the live
        # nodes (deep levels of a forest are mostly leaves)
        # (the split search's error flag comes back with the same read)
        live_err = torch.stack([is_split.sum(1).max().to(torch.int64),
                                split_err[0].to(torch.int64)]).tolist()
        live = int(live_err[0]) if depth < max_depth else 0
        if live_err[1]:
            _check_split_err(split_err, depth, ctx)
        if ctx.is_distributed:
            # the split search above consumed this level's all-reduced histograms: a one-shot
            # all-reduce whose peer never arrived must fail the forest here, not grow trees
            # from NaN statistics (the host already waited on the device for `live`)
            dist.check_collectives(ctx)
        keys = None
        # the next level is the last one and takes its totals straight from node_of
        next_last = depth + 1 == max_depth and live > 0 and _totals_ok(2 * live, S)
        if live > 0:
            W2 = 2 * live
            if next_last:
                _route(data, node_of, W, split, child_base, B, count_visits=False)
            elif 2 * T * W2 + 1 <= _SORT_MAX_KEYS and T * n < (1 << 31):
                # route + the next level's counting-sort keys in one pass
                keys = torch.empty(T * n, dtype=torch.int32, device=dev)
                cl = split.cat_left.contiguous() if split.cat_left is not None else None
                sf = split.feat.int().contiguous()
                sb = split.bin.int().contiguous()
                cb = child_base.int().contiguous()
                native.check(lib.oryx_rdf_route_keys(
                    data.Xb.data_ptr(), data.bin_bytes, n, data.Xb.stride(0), P, T,
                    node_of.data_ptr(), W, sf.data_ptr(), sb.data_ptr(),
                    cl.data_ptr() if cl is not None else None, B, cb.data_ptr(),
                    weight.data_ptr() if weight is not None else None, W2, keys.data_ptr(),
                    stream), "oryx_rdf_route_keys")
            else:
                _route(data, node_of, W, split, child_base, B, count_visits=False)
        vis = visits
        if ctx.is_distributed:
            vis = vis.clone()
            dist.all_reduce_sum(vis, ctx)
        lv = {"feat": to_host(split.feat.int()), "bin": to_host(split.bin.int()),
              "tot": to_host(split.totals), "vis": to_host(vis),
              "cat": to_host(split.cat_left) if split.cat_left is not None else None,
              "event": torch.cuda.Event()}
        lv["event"].record(torch.cuda.current_stream(dev))
        if live > 0:
            # next level: 2 * live slots, rows grouped by (tree, node) with one counting sort
            if next_last:
                perm = counts = visits = None
            else:
                finish = RowGroups.launch_from_nodes(node_of, W2, weight, keys=keys)
                perm, counts, visits = finish.device()
            W = W2
        # the previous level's nodes are built while this level's work runs
        while pending:
            build(pending.pop(0))
        pending.append(lv)
        if live == 0:
            break
    if lap is not None:
        lap("levels")
    while pending:
        build(pending.pop(0))
    if lap is not None:
        lap("tail")
    watchdog.get().end_heartbeats()
    return TrainedForest(roots, predictor_counts, classification)


# ---------------------------------------------------------------- scoring (flattened)

@dataclass
class FlatForest:
    roots: torch.Tensor
    feat: torch.Tensor
    thr: torch.Tensor
    cat_off: torch.Tensor
    cat_bits: torch.Tensor
    cat_len: torch.Tensor
    left: torch.Tensor
    right: torch.Tensor
    leaf_value: torch.Tensor         # [nodes, C] probabilities or [nodes, 1] means
    weights: torch.Tensor
    nodes: list                      # node objects by flat index (terminal lookups)


def flatten_forest(forest, device, num_classes: int) -> FlatForest:
    """Flatten a :class:`~oryx_amd.models.rdf.tree.DecisionForest` for device scoring."""
    from ..models.rdf.tree import CategoricalDecision
    feat, thr, cat_off, cat_len, left, right, vals, objs = [], [], [], [], [], [], [], []
    bits: List[int] = []
    roots = []
    for tree in forest.get_trees():
        base = len(feat)
        order = []
        stack = [tree.get_root()]
        while stack:
            nd = stack.pop()
            order.append(nd)
            if not nd.is_terminal():
                stack.append(nd.right)
                stack.append(nd.left)
        index = {id(nd): base + i for i, nd in enumerate(order)}
        roots.append(base)
        for nd in order:
            objs.append(nd)
            if nd.is_terminal():
                feat.append(-1)
                thr.append(0.0)
                cat_off.append(-1)
                cat_len.append(0)
                left.append(-1)
                right.append(-1)
                p = nd.get_prediction()
                if num_classes > 0:
                    vals.append(np.asarray(p.get_category_probabilities(), dtype=np.float64))
                else:
                    vals.append(np.array([p.get_prediction()], dtype=np.float64))
            else:
                d = nd.decision
                feat.append(d.get_feature_number())
                left.append(index[id(nd.left)])
                right.append(index[id(nd.right)])
                if isinstance(d, CategoricalDecision):
                    ln = (max(d.active) + 1) if d.active else 0
                    cat_off.append(len(bits))
                    cat_len.append(ln)
                    bits.extend(1 if e in d.active else 0 for e in range(ln))
                    thr.append(0.0)
                else:
                    cat_off.append(-1)
                    cat_len.append(0)
                    thr.append(d.get_threshold())
                vals.append(np.zeros(max(1, num_classes), dtype=np.float64))
    width = max(1, num_classes)
    leaf_value = np.zeros((len(vals), width), dtype=np.float64)
    for i, v in enumerate(vals):
        leaf_value[i, :len(v)] = v
    it = lambda a: torch.tensor(a, dtype=torch.int32, device=device)
    return FlatForest(it(roots), it(feat), torch.tensor(thr, dtype=torch.float64, device=device),
                      it(cat_off), torch.tensor(bits + [0], dtype=torch.uint8, device=device),
                      it(cat_len), it(left), it(right),
                      torch.from_numpy(leaf_value).to(device),
                      torch.from_numpy(np.asarray(forest.get_weights(), dtype=np.float64))
                      .to(device), objs)


def forest_vote(flat: FlatForest, X: torch.Tensor) -> torch.Tensor:
    """Weighted vote of the forest per example: [n, C] mean class probabilities
    (classification) or [n, 1] weighted mean prediction (regression).  GPU: one fused
    traversal + vote kernel (``rdf_forest_vote``); CPU: leaves then a gather."""
    X = X.to(torch.float64).contiguous()
    n, F = X.shape
    T = flat.roots.numel()
    C = int(flat.leaf_value.shape[1])
    dev = X.device
    if dev.type == "cuda":
        lib = native.require_kernels()
        out = torch.empty((n, C), dtype=torch.float64, device=dev)
        lv = flat.leaf_value.contiguous()
        wt = flat.weights.to(torch.float64).contiguous()
        rc = lib.oryx_rdf_forest_vote(X.data_ptr(), n, F, T, flat.roots.data_ptr(),
                                      flat.feat.data_ptr(), flat.thr.data_ptr(),
                                      flat.cat_off.data_ptr(), flat.cat_bits.data_ptr(),
                                      flat.cat_len.data_ptr(), flat.left.data_ptr(),
                                      flat.right.data_ptr(), lv.data_ptr(), C, wt.data_ptr(),
                                      out.data_ptr(), native.stream_ptr(dev))
        native.check(rc, "oryx_rdf_forest_vote")
        return out
    leaves = forest_leaves(flat, X)
    vals = flat.leaf_value[leaves]                                    # [n, T, C]
    w = flat.weights[None, :, None]
    return (vals * w).sum(1) / flat.weights.sum()


def forest_leaves(flat: FlatForest, X: torch.Tensor) -> torch.Tensor:
    """Leaf flat-index [n, T] of every example in every tree (X: float64 [n, F])."""
    X = X.to(torch.float64).contiguous()
    n, F = X.shape
    T = flat.roots.numel()
    dev = X.device
    if dev.type == "cuda":
        lib = native.require_kernels()
        out = torch.empty((n, T), dtype=torch.int32, device=dev)
        rc = lib.oryx_rdf_forest_leaf(X.data_ptr(), n, F, T, flat.roots.data_ptr(),
                                      flat.feat.data_ptr(), flat.thr.data_ptr(),
                                      flat.cat_off.data_ptr(), flat.cat_bits.data_ptr(),
                                      flat.cat_len.data_ptr(), flat.left.data_ptr(),
                                      flat.right.data_ptr(), out.data_ptr(),
                                      native.stream_ptr(dev))
        native.check(rc, "oryx_rdf_forest_leaf")
        return out.long()
    node = flat.roots.long()[None, :].expand(n, T).clone()
    rows = torch.arange(n)[:, None].expand(n, T)
    for _ in range(4096):
        f = flat.feat.long()[node]
        active = f >= 0
        if not bool(active.any()):
            break
        x = X[rows, f.clamp_min(0)]
        co = flat.cat_off.long()[node]
        enc = x.long()
        in_range = (enc >= 0) & (enc < flat.cat_len.long()[node])
        bit = flat.cat_bits.long()[(co + enc.clamp_min(0)).clamp(0, flat.cat_bits.numel() - 1)]
        pos = torch.where(co >= 0, in_range & (bit > 0), x >= flat.thr[node])
        nxt = torch.where(pos, flat.right.long()[node], flat.left.long()[node])
        node = torch.where(active, nxt, node)
    return node
