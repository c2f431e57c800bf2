"""Input schema and categorical value encodings shared by the k-means and RDF apps.

Behavioural equivalents of ``InputSchema`` (``[app-common]/schema/InputSchema.java:49-275``)
and ``CategoricalValueEncodings`` (``[app-common]/schema/CategoricalValueEncodings.java:32-100``):

* feature names come from ``oryx.input-schema.feature-names`` or, when empty,
  ``num-features`` generates ``"0".."n-1"``; names must be unique;
* active = all - id - ignored; exactly one of ``numeric-features`` / ``categorical-features``
  may be given (the other is the complement within the active set);
* the optional target must be active; predictors are the active non-target features, numbered
  in feature order (the feature <-> predictor index bijection).

Encodings map each categorical feature's distinct values to 0..n-1 in insertion order.
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Mapping, Optional, Sequence

from ..utils import config as cfg

__all__ = ["InputSchema", "CategoricalValueEncodings"]


class InputSchema:
    def __init__(self, config):
        names = list(config.get_string_list("oryx.input-schema.feature-names"))
        if not names:
            n = config.get_int("oryx.input-schema.num-features")
            if n <= 0:
                raise ValueError("Neither feature-names nor num-features is set")
            names = [str(i) for i in range(n)]
        if len(set(names)) != len(names):
            raise ValueError("Feature names must be unique: %s" % names)
        self.feature_names: List[str] = names
        self.id_features = frozenset(config.get_string_list("oryx.input-schema.id-features"))
        if not self.id_features <= set(names):
            raise ValueError("Unknown ID features %s" % sorted(self.id_features - set(names)))
        ignored = frozenset(config.get_string_list("oryx.input-schema.ignored-features"))
        if not ignored <= set(names):
            raise ValueError("Unknown ignored features %s" % sorted(ignored - set(names)))
        active = set(names) - self.id_features - ignored
        self.active_features = frozenset(active)
        numeric = cfg.get_optional_string_list(config, "oryx.input-schema.numeric-features")
        categorical = cfg.get_optional_string_list(config,
                                                   "oryx.input-schema.categorical-features")
        if numeric is None:
            if categorical is None:
                raise ValueError("Neither numeric-features nor categorical-features was set")
            cat = frozenset(categorical)
            if not cat <= active:
                raise ValueError("Active features %s not contained in categorical features %s"
                                 % (sorted(active), sorted(cat)))
            self.categorical_features = cat
            self.numeric_features = frozenset(active - cat)
        else:
            num = frozenset(numeric)
            if not num <= active:
                raise ValueError("Active features %s not contained in numeric features %s"
                                 % (sorted(active), sorted(num)))
            self.numeric_features = num
            self.categorical_features = frozenset(active - num)
        self.target_feature: Optional[str] = cfg.get_optional_string(
            config, "oryx.input-schema.target-feature")
        if self.target_feature is not None and self.target_feature not in active:
            raise ValueError("Target feature is not known, an ID, or ignored: %s"
                             % self.target_feature)
        self.target_feature_index = (-1 if self.target_feature is None
                                     else names.index(self.target_feature))
        self._all_to_pred: Dict[int, int] = {}
        self._pred_to_all: Dict[int, int] = {}
        p = 0
        for f in range(len(names)):
            if self.is_active(f) and not self.is_target(f):
                self._all_to_pred[f] = p
                self._pred_to_all[p] = f
                p += 1
        # vectorised helpers: predictor -> feature index order, active numeric mask
        self.predictor_feature_indices: List[int] = [self._pred_to_all[i] for i in range(p)]

    # --- accessors (accept a feature name or an index)
    def _name(self, f) -> str:
        return self.feature_names[f] if isinstance(f, int) else f

    def get_feature_names(self) -> List[str]:
        return self.feature_names

    def get_num_features(self) -> int:
        return len(self.feature_names)

    def get_num_predictors(self) -> int:
        return len(self.active_features) - (1 if self.has_target() else 0)

    def is_id(self, f) -> bool:
        return self._name(f) in self.id_features

    def is_active(self, f) -> bool:
        return self._name(f) in self.active_features

    def is_numeric(self, f) -> bool:
        return self._name(f) in self.numeric_features

    def is_categorical(self, f) -> bool:
        return self._name(f) in self.categorical_features

    def is_target(self, f) -> bool:
        if isinstance(f, int):
            return self.target_feature_index == f
        return f == self.target_feature

    def has_target(self) -> bool:
        return self.target_feature is not None

    def get_target_feature(self) -> str:
        if self.target_feature is None:
            raise ValueError("no target feature")
        return self.target_feature

    def get_target_feature_index(self) -> int:
        if self.target_feature_index < 0:
            raise ValueError("no target feature")
        return self.target_feature_index

    def is_classification(self) -> bool:
        return self.is_categorical(self.get_target_feature())

    def feature_to_predictor_index(self, feature_index: int) -> int:
        try:
            return self._all_to_pred[feature_index]
        except KeyError:
            raise ValueError("No predictor for feature %s" % feature_index) from None

    def predictor_to_feature_index(self, predictor_index: int) -> int:
        try:
            return self._pred_to_all[predictor_index]
        except KeyError:
            raise ValueError("No feature for predictor %s" % predictor_index) from None

    def __repr__(self):
        return "InputSchema[featureNames:%s...]" % self.feature_names


class CategoricalValueEncodings:
    """feature index -> (value -> encoding) and inverse, encodings in insertion order."""

    def __init__(self, distinct_values: Mapping[int, Iterable[str]]):
        self._v2e: Dict[int, Dict[str, int]] = {}
        self._e2v: Dict[int, List[str]] = {}
        for idx, values in distinct_values.items():
            m: Dict[str, int] = {}
            inv: List[str] = []
            for v in values:
                if v in m:
                    raise ValueError("duplicate value %r for feature %d" % (v, idx))
                m[v] = len(inv)
                inv.append(v)
            self._v2e[int(idx)] = m
            self._e2v[int(idx)] = inv

    def _check(self, index: int) -> None:
        if index < 0:
            raise ValueError("negative index")
        if index not in self._v2e:
            raise KeyError("No values for index %d" % index)

    def get_value_encoding_map(self, index: int) -> Dict[str, int]:
        self._check(index)
        return self._v2e[index]

    def get_encoding_value_map(self, index: int) -> Dict[int, str]:
        self._check(index)
        return dict(enumerate(self._e2v[index]))

    def values_in_order(self, index: int) -> List[str]:
        self._check(index)
        return self._e2v[index]

    def get_value_count(self, index: int) -> int:
        self._check(index)
        return len(self._e2v[index])

    def get_category_counts(self) -> Dict[int, int]:
        return {k: len(v) for k, v in self._e2v.items()}

    def indices(self) -> List[int]:
        return sorted(self._v2e)

    def __repr__(self):
        return repr(self._v2e)
