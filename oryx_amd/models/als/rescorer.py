"""Rescorer plug-in SPI for the ALS serving endpoints.

``Rescorer`` / ``RescorerProvider`` / ``AbstractRescorerProvider`` / ``MultiRescorer`` /
``MultiRescorerProvider`` (``[app-api]/Rescorer.java:24-41``, ``RescorerProvider.java:48-110``,
``AbstractRescorerProvider.java:26-68``, ``MultiRescorer.java:31-90``,
``MultiRescorerProvider.java:30-142``).  Providers are named by class in
``oryx.als.rescorer-provider-class`` (comma-separated -> composed).

GPU note: rescoring is arbitrary host code, so the serving model scores every item on the
GPU, takes a candidate pool of the best raw scores (all items for catalogues up to
``RESCORE_FULL_POOL`` items, which is exact), and applies filter + rescore on that pool.
"""

from __future__ import annotations

import abc
import math
from typing import List, Optional, Sequence

from ...utils import lang

__all__ = ["Rescorer", "RescorerProvider", "AbstractRescorerProvider", "MultiRescorer",
           "MultiRescorerProvider", "load_rescorer_providers"]


class Rescorer(abc.ABC):
    @abc.abstractmethod
    def rescore(self, id_: str, original_score: float) -> float: ...

    @abc.abstractmethod
    def is_filtered(self, id_: str) -> bool: ...


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
