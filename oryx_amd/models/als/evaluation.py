"""ALS evaluation on device: RMSE and per-user AUC.

``Evaluation.rmse`` / ``areaUnderCurve`` (``[mllib]/als/Evaluation.java:49-136``):

* RMSE over test pairs whose user and item are in the model (the join drops the rest);
* AUC: for each test user, sample about as many negative items (from the distinct test
  items, excluding the user's positives) as positives, then the fraction of
  (positive, negative) pairs with positive score > negative score, averaged over users.
  The pairwise count is one device sort per evaluation: scores are ordered within each user
  (positives before negatives on ties) and a segmented running count of negatives gives, for
  each positive, how many negatives score strictly lower.
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


def rmse(X: torch.Tensor, Y: torch.Tensor, u: np.ndarray, i: np.ndarray, r: np.ndarray,
         device=None) -> float:
    ok = (u >= 0) & (i >= 0)
    if not ok.any():
        return float("nan")
    dev = X.device
    uu = torch.from_numpy(u[ok]).to(dev)
    ii = torch.from_numpy(i[ok]).to(dev)
    rr = torch.from_numpy(r[ok].astype(np.float64)).to(dev)
    pred = (X[uu].double() * Y[ii].double()).sum(1)
    return float(torch.sqrt(((pred - rr) ** 2).mean()).item())


def squared_error_parts(X: torch.Tensor, Y: torch.Tensor, u: np.ndarray, i: np.ndarray,
                        r: np.ndarray, device=None) -> Tuple[float, int]:
    """(sum of squared errors, count) over the pairs with known IDs (sharded RMSE)."""
    ok = (u >= 0) & (i >= 0)
    if not ok.any():
        return 0.0, 0
    dev = X.device
    uu = torch.from_numpy(u[ok]).to(dev)
    ii = torch.from_numpy(i[ok]).to(dev)
    rr = torch.from_numpy(r[ok].astype(np.float64)).to(dev)
    pred = (X[uu].double() * Y[ii].double()).sum(1)
    return float(((pred - rr) ** 2).sum().item()), int(ok.sum())


def area_under_curve(X: torch.Tensor, Y: torch.Tensor, u: np.ndarray, i: np.ndarray,
                     device=None, seed=None) -> float:
    tot, cnt = auc_parts(X, Y, u, i, None, device=device, seed=seed)
    return tot / cnt if cnt else float("nan")


def auc_parts(X: torch.Tensor, Y: torch.Tensor, u: np.ndarray, i: np.ndarray,
              all_items: Optional[np.ndarray], device=None, seed=None) -> Tuple[float, int]:
    """(sum of per-user AUCs, number of users) -- the mean over users is the reference's AUC
    (``[mllib]/als/Evaluation.java:70-136``); ``all_items`` is the negative-sampling universe
    (default: the distinct items of these pairs; sharded callers pass the global set)."""
    ok = (u >= 0) & (i >= 0)
    u, i = u[ok], i[ok]
    if len(u) == 0:
        return 0.0, 0
    dev = X.device
    gen = rng.get_random().generator if seed is None else np.random.default_rng(seed)
    if all_items is None:
        all_items = np.unique(i)
    n_items = len(all_items)
    # positives per user
    order = np.argsort(u, kind="stable")
    u_s, i_s = u[order], i[order]
    users, starts, counts = np.unique(u_s, return_index=True, return_counts=True)
    pos_key = set((u_s.astype(np.int64) * (int(Y.shape[0]) + 1) + i_s).tolist())
    # negatives: for each user up to n_pos draws (at most n_items attempts), rejecting positives
    neg_u, neg_i = [], []
    draws = gen.integers(0, n_items, size=int(min(counts.sum(), 1 << 26) * 1 + 1))
    cursor = 0
    stride = int(Y.shape[0]) + 1
    for user, n_pos in zip(users.tolist(), counts.tolist()):
        got = 0
        attempts = 0
        while attempts < n_items and got < n_pos:
            if cursor >= len(draws):
                draws = gen.integers(0, n_items, size=len(draws))
                cursor = 0
            item = int(all_items[draws[cursor]])
            cursor += 1
            attempts += 1
            if user * stride + item not in pos_key:
                neg_u.append(user)
                neg_i.append(item)
                got += 1
    if not neg_u:
        return 0.0, 0
    nu = np.asarray(neg_u, dtype=np.int64)
    ni = np.asarray(neg_i, dtype=np.int64)
    tu = torch.from_numpy(np.concatenate([u_s, nu])).to(dev)
    ti = torch.from_numpy(np.concatenate([i_s, ni])).to(dev)
    is_pos = torch.cat([torch.ones(len(u_s), dtype=torch.bool),
                        torch.zeros(len(nu), dtype=torch.bool)]).to(dev)
    scores = _pairs_dot(X.float(), Y.float(), tu, ti).double()
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
