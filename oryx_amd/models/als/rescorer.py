"""Rescorer plug-in SPI for the ALS serving endpoints.

``Rescorer`` / ``RescorerProvider`` / ``AbstractRescorerProvider`` / ``MultiRescorer`` /
``MultiRescorerProvider`` (``[app-api]/Rescorer.java:24-41``, ``RescorerProvider.java:48-110``,
``AbstractRescorerProvider.java:26-68``, ``MultiRescorer.java:31-90``,
``MultiRescorerProvider.java:30-142``).  Providers are named by class in
``oryx.als.rescorer-provider-class`` (comma-separated -> composed).

GPU note: rescoring is arbitrary host code, so -- like ``TopNConsumer.accept``
(``[serving-app]/als/model/TopNConsumer.java:55-74``) -- EVERY candidate item's raw score is
filtered and rescored: the GPU scores all candidates in one pass, and the host applies
:meth:`Rescorer.is_filtered_many` / :meth:`Rescorer.rescore_many` to the whole candidate
array.  Their defaults call the per-item methods; a rescorer that overrides them with
vectorised versions (numpy over the arrays) makes rescored requests as fast as plain ones.
"""

from __future__ import annotations

import abc
import collections
import math
import threading
from typing import List, Optional, Sequence

import numpy as np

from ...utils import lang

__all__ = ["Rescorer", "RescorerProvider", "AbstractRescorerProvider", "MultiRescorer",
           "MultiRescorerProvider", "load_rescorer_providers", "ItemFilterRescorer",
           "ItemFilterRescorerProvider"]


class Rescorer(abc.ABC):
    @abc.abstractmethod
    def rescore(self, id_: str, original_score: float) -> float: ...

    @abc.abstractmethod
    def is_filtered(self, id_: str) -> bool: ...

    # -- array forms (an extension of the reference SPI; override for vectorised rescorers)
    def is_filtered_many(self, ids: Sequence[str]) -> np.ndarray:
        """``is_filtered`` of every ID (bool array)."""
        return np.fromiter((bool(self.is_filtered(i)) for i in ids), dtype=bool,
                           count=len(ids))

    def rescore_many(self, ids: Sequence[str], scores: np.ndarray) -> np.ndarray:
        """``rescore`` of every (ID, score) pair (float64 array; NaN drops the item)."""
        return np.fromiter((float(self.rescore(i, float(v))) for i, v in zip(ids, scores)),
                           dtype=np.float64, count=len(ids))

    # -- device form (an extension: rescoring without leaving the GPU)
    def rescore_device(self, rows, scores, store):
        """Optional: the filtered + rescored scores of candidate items on the device --
        ``rows`` (int64 store rows) and ``scores`` (fp32 raw scores) are device tensors of
        the candidates, ``store`` the item :class:`~oryx_amd.models.als.common.FeatureVectors`
        (``store.row_mask(ids)`` / ``store.id_array()`` map IDs to rows).  Return a float
        tensor like ``scores`` where NaN or -inf drops the item, or None when this rescorer
        has no device form (the host forms then run over every candidate)."""
        return None


class RescorerProvider(abc.ABC):
    @abc.abstractmethod
    def get_recommend_rescorer(self, user_ids: List[str], args: List[str]
                               ) -> Optional[Rescorer]: ...

    @abc.abstractmethod
    def get_recommend_to_anonymous_rescorer(self, item_ids: List[str], args: List[str]
                                            ) -> Optional[Rescorer]: ...

    @abc.abstractmethod
    def get_most_popular_items_rescorer(self, args: List[str]) -> Optional[Rescorer]: ...

    @abc.abstractmethod
    def get_most_active_users_rescorer(self, args: List[str]) -> Optional[Rescorer]: ...

    @abc.abstractmethod
    def get_most_similar_items_rescorer(self, args: List[str]) -> Optional[Rescorer]: ...


class AbstractRescorerProvider(RescorerProvider):
    def get_recommend_rescorer(self, user_ids, args):
        return None

    def get_recommend_to_anonymous_rescorer(self, item_ids, args):
        return None

    def get_most_popular_items_rescorer(self, args):
        return None

    def get_most_active_users_rescorer(self, args):
        return None

    def get_most_similar_items_rescorer(self, args):
        return None


class MultiRescorer(Rescorer):
    def __init__(self, rescorers: Sequence[Rescorer]):
        self.rescorers = list(rescorers)

    @staticmethod
    def of(*rescorers) -> Rescorer:
        if len(rescorers) == 1 and isinstance(rescorers[0], (list, tuple)):
            rescorers = tuple(rescorers[0])
        if not rescorers:
            raise ValueError("rescorers is null or empty")
        expanded = []
        for r in rescorers:
            if isinstance(r, MultiRescorer):
                expanded.extend(r.rescorers)
            else:
                expanded.append(r)
        return MultiRescorer(expanded)

    def rescore(self, id_, value):
        for r in self.rescorers:
            value = r.rescore(id_, value)
            if math.isnan(value):
                return float("nan")
        return value

    def is_filtered(self, id_):
        return any(r.is_filtered(id_) for r in self.rescorers)

    def is_filtered_many(self, ids):
        out = np.zeros(len(ids), dtype=bool)
        for r in self.rescorers:
            out |= np.asarray(r.is_filtered_many(ids), dtype=bool)
        return out

    def rescore_many(self, ids, scores):
        v = np.asarray(scores, dtype=np.float64)
        for r in self.rescorers:
            # an item that went NaN stays NaN (the per-item form stops at the first NaN)
            nan = np.isnan(v)
            v = np.where(nan, np.nan, np.asarray(r.rescore_many(ids, v), dtype=np.float64))
        return v

    def rescore_device(self, rows, scores, store):
        import torch
        v = scores
        for r in self.rescorers:
            nv = r.rescore_device(rows, v, store)
            if nv is None:
                return None
            v = torch.where(torch.isnan(v), v, nv)
        return v


class ItemFilterRescorer(Rescorer):
    """Drops a set of item IDs and multiplies every other score by ``factor`` -- the
    per-item and array forms and a device form (a cached row mask) give the same results."""

    def __init__(self, excluded: Sequence[str], factor: float = 1.0):
        self.excluded = frozenset(excluded)
        self.factor = float(factor)
        self._mask = None          # (store id, store version, device mask)

    def rescore(self, id_, value):
        return float("nan") if id_ in self.excluded else value * self.factor

    def is_filtered(self, id_):
        return id_ in self.excluded

    def is_filtered_many(self, ids):
        ex = self.excluded
        return np.fromiter((i in ex for i in ids), dtype=bool, count=len(ids))

    def rescore_many(self, ids, scores):
        v = np.asarray(scores, dtype=np.float64) * self.factor
        v[self.is_filtered_many(ids)] = np.nan
        return v

    def rescore_device(self, rows, scores, store):
        import torch
        key = (id(store), store.id_version)
        if self._mask is None or self._mask[0] != key[0] or self._mask[1] != key[1]:
            self._mask = key + (store.row_mask(self.excluded, rows.device),)
        m = self._mask[2]
        hit = m[rows.clamp(max=m.numel() - 1)] & (rows < m.numel())
        out = scores * self.factor
        return torch.where(hit, torch.full_like(out, float("nan")), out)


class ItemFilterRescorerProvider(AbstractRescorerProvider):
    """An example provider (``oryx.als.rescorer-provider-class``): ``rescorerParams`` values
    ``exclude:<id>`` drop items and ``factor:<x>`` scales scores, for /recommend and
    /similarity; ``ORYX_EXAMPLE_RESCORER_EXCLUDE_MOD`` (bench_serving.py) additionally drops
    every item whose numeric ID suffix is divisible by the given modulus."""

    def __init__(self):
        # rescorers by request arguments, reused across requests so that their device row
        # masks are built once per store ID layout, not per request
        self._cache: "collections.OrderedDict" = collections.OrderedDict()
        self._cache_lock = threading.Lock()

    def _parse(self, args) -> Optional[Rescorer]:
        import os
        key = (tuple(args or ()), os.environ.get("ORYX_EXAMPLE_RESCORER_EXCLUDE_MOD"))
        with self._cache_lock:
            if key in self._cache:
                self._cache.move_to_end(key)
                return self._cache[key]
        r = self._build(args)
        with self._cache_lock:
            self._cache[key] = r
            while len(self._cache) > 64:
                self._cache.popitem(last=False)
        return r

    @staticmethod
    def _build(args) -> Optional[Rescorer]:
        import os
        excl, factor = [], 1.0
        for a in args or []:
            if a.startswith("exclude:"):
                excl.append(a[len("exclude:"):])
            elif a.startswith("factor:"):
                factor = float(a[len("factor:"):])
        mod = os.environ.get("ORYX_EXAMPLE_RESCORER_EXCLUDE_MOD")
        if mod:
            return _ModExcludeRescorer(int(mod), factor, excl)
        if not excl and factor == 1.0:
            return None
        return ItemFilterRescorer(excl, factor)

    def get_recommend_rescorer(self, user_ids, args):
        return self._parse(args)

    def get_most_similar_items_rescorer(self, args):
        return self._parse(args)


class _ModExcludeRescorer(ItemFilterRescorer):
    """Drops items whose trailing digits are divisible by ``mod`` (plus explicit IDs)."""

    def __init__(self, mod: int, factor: float, excl: Sequence[str]):
        super().__init__(excl, factor)
        self.mod = mod

    def _dropped(self, id_) -> bool:
        if id_ in self.excluded:
            return True
        digits = id_[len(id_.rstrip("0123456789")):][-18:]    # as RowMap.key_suffixes
        return bool(digits) and int(digits) % self.mod == 0

    def rescore(self, id_, value):
        return float("nan") if self._dropped(id_) else value * self.factor

    def is_filtered(self, id_):
        return self._dropped(id_)

    def is_filtered_many(self, ids):
        return np.fromiter((self._dropped(i) for i in ids), dtype=bool, count=len(ids))

    def rescore_device(self, rows, scores, store):
        import torch
        key = (id(store), store.id_version)
        if self._mask is None or self._mask[0] != key[0] or self._mask[1] != key[1]:
            # every row's numeric ID suffix in one native pass over the store's id map
            suf = store.key_suffixes()
            drop = (suf >= 0) & (suf % self.mod == 0)
            if self.excluded:
                drop[store.host_rows(self.excluded)] = True
            self._mask = key + (torch.from_numpy(drop).to(rows.device),)
        m = self._mask[2]
        hit = m[rows.clamp(max=max(m.numel() - 1, 0))] & (rows < m.numel())
        out = scores * self.factor
        return torch.where(hit, torch.full_like(out, float("nan")), out)


def _build(rescorers):
    rescorers = [r for r in rescorers if r is not None]
    if not rescorers:
        return None
    if len(rescorers) == 1:
        return rescorers[0]
    return MultiRescorer.of(rescorers)


class MultiRescorerProvider(AbstractRescorerProvider):
    def __init__(self, providers: Sequence[RescorerProvider]):
        self.providers = list(providers)

    @staticmethod
    def of(*providers) -> RescorerProvider:
        if len(providers) == 1 and isinstance(providers[0], (list, tuple)):
            providers = tuple(providers[0])
        if not providers:
            raise ValueError("providers is null or empty")
        expanded = []
        for p in providers:
            if isinstance(p, MultiRescorerProvider):
                expanded.extend(p.providers)
            else:
                expanded.append(p)
        return MultiRescorerProvider(expanded)

    def get_recommend_rescorer(self, user_ids, args):
        return _build(p.get_recommend_rescorer(user_ids, args) for p in self.providers)

    def get_recommend_to_anonymous_rescorer(self, item_ids, args):
        return _build(p.get_recommend_to_anonymous_rescorer(item_ids, args)
                      for p in self.providers)

    def get_most_popular_items_rescorer(self, args):
        return _build(p.get_most_popular_items_rescorer(args) for p in self.providers)

    def get_most_active_users_rescorer(self, args):
        return _build(p.get_most_active_users_rescorer(args) for p in self.providers)

    def get_most_similar_items_rescorer(self, args):
        return _build(p.get_most_similar_items_rescorer(args) for p in self.providers)


def load_rescorer_providers(class_names: Optional[str]) -> Optional[RescorerProvider]:
    """``ALSServingModelManager.loadRescorerProviders``: comma-separated class names."""
    if not class_names:
        return None
    names = [n.strip() for n in class_names.split(",") if n.strip()]
    providers = [lang.load_instance_of(n, RescorerProvider) for n in names]
    if len(providers) == 1:
        return providers[0]
    return MultiRescorerProvider.of(providers)
