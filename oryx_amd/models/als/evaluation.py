"""ALS evaluation on device: RMSE and per-user AUC.

``Evaluation.rmse`` / ``areaUnderCurve`` (``[mllib]/als/Evaluation.java:49-136``):

* RMSE over test pairs whose user and item are in the model (the join drops the rest);
* AUC: for each test user, sample about as many negative items (from the distinct test
  items, excluding the user's positives) as positives, then the fraction of
  (positive, negative) pairs with positive score > negative score, averaged over users.
  The negative sampling runs for all users at once on the device (rounds of uniform draws,
  positives rejected by a binary search in the sorted positive keys); the pairwise count is
  one device sort per evaluation: scores are ordered within each user (positives before
  negatives on ties) and a segmented running count of negatives gives, for each positive,
  how many negatives score strictly lower.
"""

from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch

from ...ops import als as als_ops
from ...utils import rng

__all__ = ["rmse", "area_under_curve"]


def _pairs_dot(X, Y, u, i):
    kp = X.shape[1]
    if X.device.type == "cuda" and kp % 16 == 0:
        return als_ops.pair_dots(X.contiguous(), Y.contiguous(), u, i)
    return (X[u] * Y[i]).sum(1)


def _dev_index(a, dev) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.to(dev, torch.int64)
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(dev)


def _dev_values(a, dev) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.to(dev, torch.float64)
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)


def squared_error_parts(X: torch.Tensor, Y: torch.Tensor, u, i, r,
                        device=None) -> Tuple[float, int]:
    """(sum of squared errors, count) over the pairs with known IDs (rows >= 0); ``u`` /
    ``i`` / ``r`` numpy arrays or device tensors."""
    dev = X.device
    uu, ii, rr = _dev_index(u, dev), _dev_index(i, dev), _dev_values(r, dev)
    ok = (uu >= 0) & (ii >= 0)
    uu, ii, rr = uu[ok], ii[ok], rr[ok]
    if uu.numel() == 0:
        return 0.0, 0
    pred = (X[uu].double() * Y[ii].double()).sum(1)
    return float(((pred - rr) ** 2).sum().item()), int(uu.numel())


def rmse(X: torch.Tensor, Y: torch.Tensor, u, i, r, device=None) -> float:
    se, n = squared_error_parts(X, Y, u, i, r)
    return math.sqrt(se / n) if n else float("nan")


def area_under_curve(X: torch.Tensor, Y: torch.Tensor, u, i, device=None, seed=None) -> float:
    tot, cnt = auc_parts(X, Y, u, i, None, device=device, seed=seed)
    return tot / cnt if cnt else float("nan")


def _seg_offsets(counts: torch.Tensor) -> torch.Tensor:
    return torch.cumsum(counts, 0) - counts


def sample_negatives(users: torch.Tensor, n_pos: torch.Tensor, pos_keys: torch.Tensor,
                     stride: int, universe: torch.Tensor, gen: torch.Generator
                     ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per user, up to ``n_pos`` negative items drawn uniformly (with replacement) from
    ``universe``, rejecting the user's positives (``pos_keys``: sorted ``user * stride +
    item``), with at most ``len(universe)`` attempts per user -- the sampling loop of
    ``Evaluation.java:94-106`` run for all users at once on the device.  Draws happen in
    rounds: each round gives every unfinished user a block of attempts, keeps the accepted
    draws up to the user's remaining need and charges only the attempts a sequential loop
    would have made (up to the last accepted draw it needed), so the sample has the
    sequential loop's distribution."""
    dev = users.device
    n_items = int(universe.numel())
    need = n_pos.clone()
    left = torch.full_like(need, n_items)
    out_u, out_i = [], []
    while True:
        act = (need > 0) & (left > 0)
        if not bool(act.any()):
            break
        au, an, al = users[act], need[act], left[act]
        # about 1.3x the remaining need (most users reject few draws), at least 16
        m = torch.minimum(al, an + (an * 3 + 9) // 10 + 16)
        M = int(m.sum())
        seg = torch.repeat_interleave(torch.arange(au.numel(), device=dev), m)
        draw = torch.randint(0, n_items, (M,), device=dev, generator=gen)
        item = universe[draw]
        key = au[seg] * stride + item
        if pos_keys.numel():
            at = torch.searchsorted(pos_keys, key).clamp_max(pos_keys.numel() - 1)
            acc = pos_keys[at] != key
        else:
            acc = torch.ones(M, dtype=torch.bool, device=dev)
        start = _seg_offsets(m)
        cum = torch.cumsum(acc.to(torch.int64), 0)
        before = (cum - acc.to(torch.int64))[start]           # accepted before each segment
        rank = cum - before[seg]                               # 1-based among accepted
        take = acc & (rank <= an[seg])
        got = torch.zeros_like(an).index_add_(0, seg, take.to(torch.int64))
        # attempts a sequential loop makes: through the need-th acceptance, else all m
        pos = torch.arange(M, device=dev) - start[seg] + 1
        last = torch.where(take & (rank == an[seg]), pos, torch.full_like(pos, 1 << 62))
        used = torch.full_like(an, 1 << 62).scatter_reduce_(0, seg, last, "amin")
        used = torch.where(used == (1 << 62), m, used)
        out_u.append(au[seg[take]])
        out_i.append(item[take])
        need[act] = an - got
        left[act] = al - used
    if not out_u:
        e = torch.zeros(0, dtype=torch.int64, device=dev)
        return e, e
    return torch.cat(out_u), torch.cat(out_i)


def auc_parts(X: torch.Tensor, Y: torch.Tensor, u, i, all_items=None, device=None,
              seed=None) -> Tuple[float, int]:
    """(sum of per-user AUCs, number of users) -- the mean over users is the reference's AUC
    (``[mllib]/als/Evaluation.java:70-136``); ``all_items`` is the negative-sampling universe
    (default: the distinct items of these pairs; sharded callers pass the global set).
    ``u`` / ``i``: row indices into X / Y (numpy or device tensors; rows < 0 are dropped).
    Everything runs on X's device: negative sampling (:func:`sample_negatives`), the pair
    scores (``pair_dots``) and the per-user pairwise count."""
    dev = X.device
    uu, ii = _dev_index(u, dev), _dev_index(i, dev)
    ok = (uu >= 0) & (ii >= 0)
    uu, ii = uu[ok], ii[ok]
    if uu.numel() == 0:
        return 0.0, 0
    if seed is None:
        seed = int(rng.get_random().generator.integers(0, 1 << 62))
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed) & ((1 << 62) - 1))
    universe = torch.unique(ii) if all_items is None else _dev_index(all_items, dev)
    stride = int(Y.shape[0]) + 1
    # positives per user, users ascending
    order = torch.argsort(uu, stable=True)
    u_s, i_s = uu[order], ii[order]
    users, counts = torch.unique_consecutive(u_s, return_counts=True)
    pos_keys = torch.sort(u_s * stride + i_s).values
    nu, ni = sample_negatives(users, counts, pos_keys, stride, universe, gen)
    if nu.numel() == 0:
        return 0.0, 0
    tu = torch.cat([u_s, nu])
    ti = torch.cat([i_s, ni])
    is_pos = torch.cat([torch.ones(u_s.numel(), dtype=torch.bool, device=dev),
                        torch.zeros(nu.numel(), dtype=torch.bool, device=dev)])
    scores = _pairs_dot(X.float(), Y.float(), tu, ti).double()
    return _pairwise_auc(tu, is_pos, scores)


def _pairwise_auc(tu: torch.Tensor, is_pos: torch.Tensor, scores: torch.Tensor
                  ) -> Tuple[float, int]:
    dev = tu.device
    # sort by (user, score, positives-first on ties)
    o = torch.argsort(-is_pos.to(torch.int64), stable=True)
    o = o[torch.argsort(scores[o], stable=True)]
    o = o[torch.argsort(tu[o], stable=True)]
    su, sp = tu[o], is_pos[o]
    neg = (~sp).to(torch.int64)
    cum_neg = torch.cumsum(neg, 0)
    # segment start offsets
    seg_start = torch.ones_like(su, dtype=torch.bool)
    seg_start[1:] = su[1:] != su[:-1]
    seg_id = torch.cumsum(seg_start.to(torch.int64), 0) - 1
    base = (cum_neg - neg)[seg_start]                 # negatives before each segment
    below = cum_neg - neg - base[seg_id]               # negatives strictly before position
    n_seg = int(seg_id.max().item()) + 1
    correct = torch.zeros(n_seg, dtype=torch.float64, device=dev)
    correct.index_add_(0, seg_id[sp], below[sp].double())
    n_pos = torch.zeros(n_seg, dtype=torch.float64, device=dev).index_add_(
        0, seg_id, sp.double())
    n_neg = torch.zeros(n_seg, dtype=torch.float64, device=dev).index_add_(
        0, seg_id, (~sp).double())
    valid = (n_pos > 0) & (n_neg > 0)
    auc_u = correct[valid] / (n_pos[valid] * n_neg[valid])
    return float(auc_u.sum().item()), int(auc_u.numel())


def auc_parts_reference(X: torch.Tensor, Y: torch.Tensor, u: np.ndarray, i: np.ndarray,
                        all_items: Optional[np.ndarray] = None, seed=None) -> Tuple[float, int]:
    """The sequential host loop of ``Evaluation.java:94-106`` (one draw at a time per user,
    a hash set of positives) -- the model :func:`auc_parts` is tested against."""
    ok = (u >= 0) & (i >= 0)
    u, i = u[ok], i[ok]
    if len(u) == 0:
        return 0.0, 0
    dev = X.device
    gen = rng.get_random().generator if seed is None else np.random.default_rng(seed)
    if all_items is None:
        all_items = np.unique(i)
    n_items = len(all_items)
    order = np.argsort(u, kind="stable")
    u_s, i_s = u[order], i[order]
    users, counts = np.unique(u_s, return_counts=True)
    stride = int(Y.shape[0]) + 1
    pos_key = set((u_s.astype(np.int64) * stride + i_s).tolist())
    neg_u, neg_i = [], []
    for user, n_pos in zip(users.tolist(), counts.tolist()):
        got = attempts = 0
        while attempts < n_items and got < n_pos:
            item = int(all_items[int(gen.integers(0, n_items))])
            attempts += 1
            if user * stride + item not in pos_key:
                neg_u.append(user)
                neg_i.append(item)
                got += 1
    if not neg_u:
        return 0.0, 0
    tu = torch.from_numpy(np.concatenate([u_s, np.asarray(neg_u, dtype=np.int64)])).to(dev)
    ti = torch.from_numpy(np.concatenate([i_s, np.asarray(neg_i, dtype=np.int64)])).to(dev)
    is_pos = torch.cat([torch.ones(len(u_s), dtype=torch.bool),
                        torch.zeros(len(neg_u), dtype=torch.bool)]).to(dev)
    scores = _pairs_dot(X.float(), Y.float(), tu, ti).double()
    return _pairwise_auc(tu, is_pos, scores)
