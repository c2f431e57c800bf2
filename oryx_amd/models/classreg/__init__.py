"""Classification / regression shared types: features, examples, predictions, voting.

Equivalents of ``[app-common]/classreg/example/*`` (``Example``, ``NumericFeature``,
``CategoricalFeature``, ``FeatureType``, ``ExampleUtils.dataToExample``
``ExampleUtils.java:42-71``) and ``[app-common]/classreg/predict/*`` (``CategoricalPrediction``
``CategoricalPrediction.java:32-134``, ``NumericPrediction`` ``NumericPrediction.java:28-79``,
``WeightedPrediction.voteOnFeature`` ``WeightedPrediction.java:44-94``).
"""

from __future__ import annotations

import enum
import threading
from typing import List, Optional, Sequence

import numpy as np

from ...utils import text
from ..schema import CategoricalValueEncodings, InputSchema

__all__ = ["FeatureType", "NumericFeature", "CategoricalFeature", "Example", "data_to_example",
           "Prediction", "CategoricalPrediction", "NumericPrediction", "vote_on_feature"]


class FeatureType(enum.Enum):
    NUMERIC = "NUMERIC"
    CATEGORICAL = "CATEGORICAL"


class NumericFeature:
    __slots__ = ("value",)
    feature_type = FeatureType.NUMERIC

    def __init__(self, value: float):
        self.value = float(value)

    @staticmethod
    def for_value(value: float) -> "NumericFeature":
        return NumericFeature(value)

    def get_value(self) -> float:
        return self.value

    def __eq__(self, o):
        return isinstance(o, NumericFeature) and o.value == self.value

    def __hash__(self):
        return hash(self.value)

    def __repr__(self):
        return text.java_double_str(self.value)


class CategoricalFeature:
    __slots__ = ("encoding",)
    feature_type = FeatureType.CATEGORICAL
    _CACHE = {}

    def __init__(self, encoding: int):
        if encoding < 0:
            raise ValueError("negative encoding")
        self.encoding = int(encoding)

    @classmethod
    def for_encoding(cls, encoding: int) -> "CategoricalFeature":
        f = cls._CACHE.get(encoding)
        if f is None:
            f = cls._CACHE[encoding] = CategoricalFeature(encoding)
        return f

    def get_encoding(self) -> int:
        return self.encoding

    def __eq__(self, o):
        return isinstance(o, CategoricalFeature) and o.encoding == self.encoding

    def __hash__(self):
        return self.encoding

    def __repr__(self):
        return ":%d" % self.encoding


class Example:
    """Features indexed by FEATURE index (not predictor index); ``None`` = missing/inactive."""

    __slots__ = ("features", "target")

    def __init__(self, target, *features):
        if len(features) == 1 and isinstance(features[0], (list, tuple)):
            features = tuple(features[0])
        self.features = tuple(features)
        self.target = target

    def get_feature(self, i: int):
        return self.features[i]

    def get_target(self):
        return self.target

    def __eq__(self, o):
        return isinstance(o, Example) and o.features == self.features and o.target == self.target

    def __hash__(self):
        return hash((self.features, self.target))

    def __repr__(self):
        s = "[" + ", ".join(repr(f) if f is not None else "null" for f in self.features) + "]"
        return s if self.target is None else s + " -> " + repr(self.target)


def _parse_double(tok: str) -> float:
    from ..kmeans.common import _parse_double as pd
    return pd(tok)


def data_to_example(data: Sequence[str], schema: InputSchema,
                    encodings: CategoricalValueEncodings) -> Example:
    features = [None] * len(data)
    target = None
    for fi, tok in enumerate(data):
        is_target = schema.is_target(fi)
        feature = None
        if is_target and tok == "":
            feature = None
        elif schema.is_numeric(fi):
            feature = NumericFeature.for_value(_parse_double(tok))
        elif schema.is_categorical(fi):
            enc = encodings.get_value_encoding_map(fi).get(tok)
            if enc is None:
                raise ValueError("Unknown value %r for feature %d" % (tok, fi))
            feature = CategoricalFeature.for_encoding(enc)
        if is_target:
            target = feature
        else:
            features[fi] = feature
    return Example(target, features)


# ---------------------------------------------------------------- predictions

class Prediction:
    feature_type: FeatureType

    def __init__(self, count: int):
        self.count = int(count)
        self._lock = threading.Lock()

    def get_count(self) -> int:
        return self.count


class CategoricalPrediction(Prediction):
    feature_type = FeatureType.CATEGORICAL

    def __init__(self, category_counts):
        counts = np.asarray(category_counts, dtype=np.float64).copy()
        super().__init__(int(round(float(counts.sum()))))
        self.category_counts = counts
        self._recompute()

    def _recompute(self) -> None:
        total = float(self.category_counts.sum())
        if len(self.category_counts) == 0:
            raise ValueError("no categories")
        self.max_category = int(np.argmax(self.category_counts))   # first max wins
        self.category_probabilities = self.category_counts / total

    def get_category_counts(self) -> np.ndarray:
        return self.category_counts

    def get_category_probabilities(self) -> np.ndarray:
        return self.category_probabilities

    def get_most_probable_category_encoding(self) -> int:
        return self.max_category

    def update_example(self, train: Example) -> None:
        self.update(train.get_target().get_encoding(), 1)

    def update(self, encoding: int, count: int) -> None:
        with self._lock:
            self.category_counts[encoding] += count
            self.count += int(count)
            self._recompute()

    def __eq__(self, o):
        return isinstance(o, CategoricalPrediction) and \
            np.array_equal(o.category_counts, self.category_counts)

    def __hash__(self):
        return hash(tuple(self.category_counts.tolist()))

    def __repr__(self):
        return ":[" + ", ".join(text.java_double_str(float(p))
                                for p in self.category_probabilities) + "]"


class NumericPrediction(Prediction):
    feature_type = FeatureType.NUMERIC

    def __init__(self, prediction: float, initial_count: int):
        super().__init__(initial_count)
        self.prediction = float(prediction)

    def get_prediction(self) -> float:
        return self.prediction

    def update_example(self, train: Example) -> None:
        self.update(train.get_target().get_value(), 1)

    def update(self, new_prediction: float, new_count: int) -> None:
        with self._lock:
            total = self.count + int(new_count)
            frac = float(new_count) / total
            self.count = total
            self.prediction += frac * (float(new_prediction) - self.prediction)

    def __eq__(self, o):
        return isinstance(o, NumericPrediction) and o.prediction == self.prediction

    def __hash__(self):
        return hash(self.prediction)

    def __repr__(self):
        return text.java_double_str(self.prediction)


def vote_on_feature(predictions: Sequence[Prediction], weights: Sequence[float]) -> Prediction:
    if not predictions:
        raise ValueError("No predictions")
    if len(predictions) != len(weights):
        raise ValueError("%d predictions but %d weights?" % (len(predictions), len(weights)))
    first = predictions[0]
    if first.feature_type is FeatureType.NUMERIC:
        w = np.asarray(weights, dtype=np.float64)
        vals = np.array([p.get_prediction() for p in predictions], dtype=np.float64)
        total = float(w.sum())
        mean = float((vals * w).sum() / total) if total > 0 else float("nan")
        return NumericPrediction(mean, len(predictions))
    acc = None
    total = 0.0
    for p, wt in zip(predictions, weights):
        probs = p.get_category_probabilities()
        acc = probs * wt if acc is None else acc + probs * wt
        total += wt
    return CategoricalPrediction(acc / total)
