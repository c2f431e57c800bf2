"""Decision trees and forests (the serving/speed-side model of the RDF app).

Equivalents of ``[app-common]/rdf/decision/{NumericDecision,CategoricalDecision}.java``
(``NumericDecision.java:29-82``: ``x >= threshold``, default on missing;
``CategoricalDecision.java:32-104``: encoding in the active set) and
``[app-common]/rdf/tree/{TreeNode,TerminalNode,DecisionNode,DecisionTree,DecisionForest,
TreePath}.java`` (``DecisionTree.findTerminal`` ``:53-64``: right if the decision is positive;
``findByID`` ``:66-84`` walks ``+``/``-`` suffixes; ``DecisionForest.predict`` = weighted vote).

The serving side keeps this pointer tree for single-example ``/predict`` and speed-layer
``UP`` updates (leaf lookup by ID); bulk scoring (evaluation, the speed layer's batch) uses the
flattened arrays of :meth:`DecisionForest.flatten` on the device (:mod:`oryx_amd.ops.rdf`).
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from ...utils import text
from ..classreg import (CategoricalPrediction, Example, FeatureType, NumericPrediction,
                        Prediction, vote_on_feature)

__all__ = ["NumericDecision", "CategoricalDecision", "TerminalNode", "DecisionNode",
           "DecisionTree", "DecisionForest", "TreePath"]


class NumericDecision:
    feature_type = FeatureType.NUMERIC

    def __init__(self, feature_number: int, threshold: float, default_decision: bool):
        self.feature_number = int(feature_number)
        self.threshold = float(threshold)
        self.default_decision = bool(default_decision)

    def get_feature_number(self) -> int:
        return self.feature_number

    def get_threshold(self) -> float:
        return self.threshold

    def get_default_decision(self) -> bool:
        return self.default_decision

    def get_type(self) -> FeatureType:
        return FeatureType.NUMERIC

    def is_positive(self, example: Example) -> bool:
        f = example.get_feature(self.feature_number)
        return self.default_decision if f is None else f.get_value() >= self.threshold

    def __eq__(self, o):
        return isinstance(o, NumericDecision) and o.feature_number == self.feature_number \
            and o.threshold == self.threshold

    def __hash__(self):
        return hash((self.feature_number, self.threshold))

    def __repr__(self):
        return "(#%d >= %s)" % (self.feature_number, text.java_double_str(self.threshold))


class CategoricalDecision:
    feature_type = FeatureType.CATEGORICAL

    def __init__(self, feature_number: int, active_category_encodings, default_decision: bool):
        self.feature_number = int(feature_number)
        self.active = frozenset(int(e) for e in active_category_encodings)
        self.default_decision = bool(default_decision)

    def get_feature_number(self) -> int:
        return self.feature_number

    def get_active_category_encodings(self) -> frozenset:
        return self.active

    def get_default_decision(self) -> bool:
        return self.default_decision

    def get_type(self) -> FeatureType:
        return FeatureType.CATEGORICAL

    def is_positive(self, example: Example) -> bool:
        f = example.get_feature(self.feature_number)
        if f is None:
            return self.default_decision
        return f.get_encoding() in self.active

    def __eq__(self, o):
        return isinstance(o, CategoricalDecision) and o.feature_number == self.feature_number \
            and o.active == self.active

    def __hash__(self):
        return hash((self.feature_number, self.active))

    def __repr__(self):
        return "(#%d ∈ [%s])" % (self.feature_number,
                                      ",".join(str(e) for e in sorted(self.active)))


class TerminalNode:
    def __init__(self, id_: str, prediction: Prediction):
        if id_ is None:
            raise ValueError("null id")
        self.id = id_
        self.prediction = prediction

    def get_id(self) -> str:
        return self.id

    def is_terminal(self) -> bool:
        return True

    def get_prediction(self) -> Prediction:
        return self.prediction

    def get_count(self) -> int:
        return self.prediction.get_count()

    def update(self, train: Example) -> None:
        self.prediction.update_example(train)

    def __eq__(self, o):
        return isinstance(o, TerminalNode) and o.prediction == self.prediction

    def __hash__(self):
        return hash(self.prediction)

    def __repr__(self):
        return "[ %r ]" % (self.prediction,)


class DecisionNode:
    def __init__(self, id_: str, decision, left, right):
        if id_ is None:
            raise ValueError("null id")
        self.id = id_
        self.decision = decision
        self.left = left
        self.right = right

    def get_id(self) -> str:
        return self.id

    def is_terminal(self) -> bool:
        return False

    def get_decision(self):
        return self.decision

    def get_left(self):
        return self.left

    def get_right(self):
        return self.right

    def __eq__(self, o):
        return isinstance(o, DecisionNode) and o.decision == self.decision and \
            o.left == self.left and o.right == self.right

    def __hash__(self):
        return hash(self.decision) ^ hash(self.left) ^ hash(self.right)

    def __repr__(self):
        return repr(self.decision)


class TreePath:
    """Left/right path bits (``[app-common]/rdf/tree/TreePath.java:25-102``)."""

    __slots__ = ("bits", "length")

    def __init__(self, bits: int = 0, length: int = 0):
        if not 0 <= length <= 64:
            raise ValueError("bad path length")
        self.bits = bits
        self.length = length

    def is_left_at(self, i: int) -> bool:
        if not 0 <= i < self.length:
            raise IndexError(i)
        return not (self.bits >> (63 - i)) & 1

    def extend_left(self) -> "TreePath":
        return TreePath(self.bits, self.length + 1)

    def extend_right(self) -> "TreePath":
        return TreePath(self.bits | (1 << (63 - self.length)), self.length + 1)

    def __eq__(self, o):
        return isinstance(o, TreePath) and o.bits == self.bits and o.length == self.length

    def __hash__(self):
        return hash((self.bits, self.length))

    def __repr__(self):
        return "".join("0" if self.is_left_at(i) else "1" for i in range(self.length))

    def _key(self):
        # left < right at the first difference; a prefix sorts before its right extensions
        # and after its left extensions
        out = []
        for i in range(64):
            if i < self.length:
                out.append(0 if self.is_left_at(i) else 2)
            else:
                out.append(1)
                break
        return out

    def __lt__(self, o):
        return self._key() < o._key()


TreePath.EMPTY = TreePath()


class DecisionTree:
    def __init__(self, root):
        if root is None:
            raise ValueError("null root")
        self.root = root

    def get_root(self):
        return self.root

    def predict(self, test: Example) -> Prediction:
        return self.find_terminal(test).get_prediction()

    def find_terminal(self, example: Example) -> TerminalNode:
        node = self.root
        while not node.is_terminal():
            node = node.right if node.decision.is_positive(example) else node.left
        return node

    def find_by_id(self, id_: str):
        node = self.root
        while id_ != node.id:
            if node.is_terminal():
                raise ValueError("No node with ID " + id_)
            if not id_.startswith(node.id):
                raise ValueError("Node ID %s is not a prefix of %s" % (node.id, id_))
            c = id_[len(node.id)]
            if c == "+":
                node = node.right
            elif c == "-":
                node = node.left
            else:
                raise ValueError("bad node id " + id_)
        return node

    def update(self, train: Example) -> None:
        self.find_terminal(train).update(train)

    def nodes(self):
        """All nodes, preorder (positive/right child first, as in the PMML)."""
        stack = [self.root]
        while stack:
            n = stack.pop()
            yield n
            if not n.is_terminal():
                stack.append(n.left)
                stack.append(n.right)

    def __repr__(self):
        out = []
        stack: List[Tuple[object, TreePath]] = [(self.root, TreePath.EMPTY)]
        while stack:
            node, path = stack.pop()
            for i in range(path.length):
                if i == path.length - 1:
                    out.append(" +-")
                else:
                    out.append(" | " if path.is_left_at(i) else "   ")
            out.append(repr(node) + "\n")
            if not node.is_terminal():
                stack.append((node.right, path.extend_right()))
                stack.append((node.left, path.extend_left()))
        return "".join(out)


class DecisionForest:
    def __init__(self, trees: Sequence[DecisionTree], weights: Sequence[float],
                 feature_importances: Optional[Sequence[float]]):
        self.trees = list(trees)
        self.weights = np.asarray(weights, dtype=np.float64)
        self.feature_importances = (None if feature_importances is None
                                    else np.asarray(feature_importances, dtype=np.float64))
        self._flat = None

    def get_trees(self) -> List[DecisionTree]:
        return self.trees

    def get_weights(self) -> np.ndarray:
        return self.weights

    def get_feature_importances(self) -> Optional[np.ndarray]:
        return self.feature_importances

    def predict(self, test: Example) -> Prediction:
        return vote_on_feature([t.predict(test) for t in self.trees], self.weights)

    def update(self, train: Example) -> None:
        for t in self.trees:
            t.update(train)

    def __repr__(self):
        return "".join(repr(t) + "\n" for t in self.trees)
