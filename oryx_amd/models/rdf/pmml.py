"""RDF PMML codec: TreeModel / MiningModel <-> :class:`DecisionForest`.

Reading is ``RDFPMMLUtils.read`` / ``translateFromPMML`` (``[app-common]/rdf/RDFPMMLUtils.java:
116-278``): the child with the ``True`` predicate is the negative (left) child, the other
carries a ``SimplePredicate`` (``greaterOrEqual``, or ``greaterThan`` implemented as ``>=`` the
threshold + 1 ulp) or a ``SimpleSetPredicate`` (``isIn`` / ``isNotIn``); the default child
gives the missing-value decision; leaves carry ``ScoreDistribution`` record counts
(classification) or a ``score`` + ``recordCount`` (regression).  ``validate_pmml_vs_schema``
is ``RDFPMMLUtils.validatePMMLVsSchema`` (``:62-114``).

Writing follows ``RDFUpdate.rdfModelToPMML`` / ``toTreeModel`` / ``buildPredicate``
(``[mllib]/rdf/RDFUpdate.java:369-550``): node IDs ``r``, ``r+``, ``r-``; the positive (right)
child comes first; ``isNotIn`` of the left categories or ``greaterThan`` the threshold; default
child = the child that saw more training examples; one ``Segment`` (weight 1) per tree in a
``MiningModel`` (weighted majority vote / weighted average) when there is more than one tree;
extensions ``maxDepth``, ``maxSplitCandidates``, ``impurity``.  Divergences (deliberate):
regression leaves carry the real mean (the reference truncates it to an int); classification
leaves carry the true per-class counts (the reference spreads MLlib's single probability).
"""

from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ...utils import pmml as pm
from ...utils import text
from .. import app_pmml
from ..classreg import CategoricalPrediction, NumericPrediction
from ..schema import CategoricalValueEncodings, InputSchema
from .tree import (CategoricalDecision, DecisionForest, DecisionNode, DecisionTree,
                   NumericDecision, TerminalNode)

__all__ = ["validate_pmml_vs_schema", "read", "forest_to_pmml", "TreeSpecNode"]


def _model(pmml: pm.PMMLDoc) -> ET.Element:
    models = pmml.models()
    if len(models) != 1:
        raise ValueError("Should have exactly one model, but had %d" % len(models))
    return models[0]


def validate_pmml_vs_schema(pmml: pm.PMMLDoc, schema: InputSchema) -> None:
    model = _model(pmml)
    fn = model.get("functionName")
    if schema.is_classification():
        if fn != "classification":
            raise ValueError("Expected classification function type but got %s" % fn)
    elif fn != "regression":
        raise ValueError("Expected regression function type but got %s" % fn)
    dd = pmml.find("DataDictionary")
    if dd is None or schema.feature_names != app_pmml.feature_names_of(dd):
        raise ValueError("Feature names in schema don't match names in PMML")
    ms = model.find(pm.q("MiningSchema"))
    if ms is None or schema.feature_names != app_pmml.feature_names_of(ms):
        raise ValueError("Feature names in schema don't match MiningSchema")
    pmml_idx = app_pmml.find_target_index(ms)
    if schema.has_target():
        if pmml_idx is None or pmml_idx != schema.get_target_feature_index():
            raise ValueError("Configured schema expects target at index %s, but PMML has target "
                             "at index %s" % (schema.get_target_feature_index(), pmml_idx))
    elif pmml_idx is not None:
        raise ValueError("PMML has a target but the schema does not")


def _java_ulp(x: float) -> float:
    return math.ulp(x)


def _predicate(node: ET.Element) -> Optional[ET.Element]:
    for tag in ("True", "SimplePredicate", "SimpleSetPredicate", "False"):
        p = node.find(pm.q(tag))
        if p is not None:
            return p
    return None


def _translate(node: ET.Element, encodings: CategoricalValueEncodings, names: List[str],
               target_index: int):
    id_ = node.get("id")
    children = node.findall(pm.q("Node"))
    if not children:
        dists = node.findall(pm.q("ScoreDistribution"))
        if dists:
            target_enc = encodings.get_value_encoding_map(target_index)
            counts = np.zeros(len(target_enc), dtype=np.float64)
            for d in dists:
                counts[target_enc[d.get("value")]] = float(d.get("recordCount"))
            pred = CategoricalPrediction(counts)
        else:
            pred = NumericPrediction(float(node.get("score")),
                                     int(round(float(node.get("recordCount") or 0))))
        return TerminalNode(id_, pred)
    if len(children) != 2:
        raise ValueError("expected 2 children")
    c1, c2 = children
    if _predicate(c1).tag == pm.q("True"):
        neg, pos = c1, c2
    else:
        if _predicate(c2).tag != pm.q("True"):
            raise ValueError("one child must have a True predicate")
        neg, pos = c2, c1
    pred = _predicate(pos)
    default_decision = pos.get("id") == node.get("defaultChild")
    if pred.tag == pm.q("SimplePredicate"):
        op = pred.get("operator")
        if op not in ("greaterOrEqual", "greaterThan"):
            raise ValueError("unsupported operator " + str(op))
        thr = float(pred.get("value"))
        if op == "greaterThan":
            thr += _java_ulp(thr)
        decision = NumericDecision(names.index(pred.get("field")), thr, default_decision)
    elif pred.tag == pm.q("SimpleSetPredicate"):
        op = pred.get("booleanOperator")
        if op not in ("isIn", "isNotIn"):
            raise ValueError("unsupported set operator " + str(op))
        fnum = names.index(pred.get("field"))
        venc = encodings.get_value_encoding_map(fnum)
        arr = pred.find(pm.q("Array"))
        cats = text.parse_pmml_delimited(arr.text or "")
        if op == "isIn":
            active = {venc[c] for c in cats}
        else:
            active = set(venc.values()) - {venc[c] for c in cats}
        decision = CategoricalDecision(fnum, active, default_decision)
    else:
        raise ValueError("unsupported predicate " + pred.tag)
    return DecisionNode(id_, decision, _translate(neg, encodings, names, target_index),
                        _translate(pos, encodings, names, target_index))


def read(pmml: pm.PMMLDoc) -> Tuple[DecisionForest, CategoricalValueEncodings]:
    dd = pmml.find("DataDictionary")
    names = app_pmml.feature_names_of(dd)
    encodings = app_pmml.build_categorical_value_encodings(dd)
    model = _model(pmml)
    ms = model.find(pm.q("MiningSchema"))
    target_index = app_pmml.find_target_index(ms)
    if target_index is None:
        raise ValueError("no target in MiningSchema")
    trees, weights = [], []
    if model.tag == pm.q("MiningModel"):
        seg = model.find(pm.q("Segmentation"))
        method = seg.get("multipleModelMethod")
        if method not in ("weightedAverage", "weightedMajorityVote"):
            raise ValueError("unsupported multipleModelMethod " + str(method))
        segments = seg.findall(pm.q("Segment"))
        if not segments:
            raise ValueError("no segments")
        for s in segments:
            if s.find(pm.q("True")) is None:
                raise ValueError("segment predicate must be True")
            weights.append(float(s.get("weight", "1")))
            tm = s.find(pm.q("TreeModel"))
            trees.append(DecisionTree(_translate(tm.find(pm.q("Node")), encodings, names,
                                                 target_index)))
    else:
        trees.append(DecisionTree(_translate(model.find(pm.q("Node")), encodings, names,
                                             target_index)))
        weights.append(1.0)
    importances = np.zeros(len(names), dtype=np.float64)
    for i, f in enumerate(ms.findall(pm.q("MiningField"))):
        imp = f.get("importance")
        if imp is not None:
            importances[i] = float(imp)
    return DecisionForest(trees, weights, importances), encodings


# ---------------------------------------------------------------- writing

class TreeSpecNode:
    """A trained node: leaf (``class_counts`` or ``mean``) or split on ``feature`` (feature
    index) by ``threshold`` (numeric: left = x <= threshold) or ``left_categories``."""

    __slots__ = ("id", "count", "class_counts", "mean", "feature", "threshold",
                 "left_categories", "default_right", "left", "right")

    def __init__(self, id_: str, count: float):
        self.id = id_
        self.count = count
        self.class_counts = None
        self.mean = None
        self.feature = None
        self.threshold = None
        self.left_categories = None
        self.default_right = False
        self.left = None
        self.right = None

    @property
    def is_leaf(self) -> bool:
        return self.feature is None


def _tree_model(root: TreeSpecNode, schema: InputSchema, encodings: CategoricalValueEncodings,
                classification: bool) -> ET.Element:
    tm = ET.Element(pm.q("TreeModel"), {
        "functionName": "classification" if classification else "regression",
        "splitCharacteristic": "binarySplit", "missingValueStrategy": "defaultChild"})
    names = schema.feature_names
    target_values = (encodings.values_in_order(schema.get_target_feature_index())
                     if classification else None)

    def emit(parent: ET.Element, n: TreeSpecNode, predicate: Optional[ET.Element]):
        el = pm.sub(parent, "Node", {"id": n.id, "recordCount": float(n.count)})
        if predicate is None:
            pm.sub(el, "True")
        else:
            el.append(predicate)
        if n.is_leaf:
            if classification:
                counts = np.asarray(n.class_counts, dtype=np.float64)
                total = float(counts.sum())
                for enc, value in enumerate(target_values):
                    c = float(counts[enc]) if enc < len(counts) else 0.0
                    if c > 0.0:
                        pm.sub(el, "ScoreDistribution", {
                            "value": value, "recordCount": c,
                            "confidence": c / total if total > 0 else 0.0})
            else:
                el.set("score", text.java_double_str(float(n.mean)))
            return
        el.set("defaultChild", n.id + ("+" if n.default_right else "-"))
        fname = names[n.feature]
        if n.left_categories is not None:
            fenc = encodings.values_in_order(n.feature)
            neg_values = [fenc[e] for e in sorted(n.left_categories)]
            pred = ET.Element(pm.q("SimpleSetPredicate"),
                              {"field": fname, "booleanOperator": "isNotIn"})
            arr = pm.sub(pred, "Array", {"type": "string", "n": str(len(neg_values))})
            arr.text = text.join_pmml_delimited(neg_values)
        else:
            pred = ET.Element(pm.q("SimplePredicate"), {
                "field": fname, "operator": "greaterThan",
                "value": text.java_double_str(float(n.threshold))})
        # the positive (right) child carries the predicate and is evaluated first
        emit(el, n.right, pred)
        emit(el, n.left, None)

    # the root's own (absent) predicate is True
    emit(tm, root, None)
    return tm


def forest_to_pmml(roots: Sequence[TreeSpecNode], schema: InputSchema,
                   encodings: CategoricalValueEncodings, importances: Sequence[float],
                   max_depth: int, max_split_candidates: int, impurity: str) -> pm.PMMLDoc:
    classification = schema.is_classification()
    fn = "classification" if classification else "regression"
    if len(roots) == 1:
        model = _tree_model(roots[0], schema, encodings, classification)
        model.insert(0, app_pmml.build_mining_schema(schema, importances))
    else:
        model = ET.Element(pm.q("MiningModel"), {"functionName": fn})
        model.append(app_pmml.build_mining_schema(schema, importances))
        seg = pm.sub(model, "Segmentation", {
            "multipleModelMethod": "weightedMajorityVote" if classification
            else "weightedAverage"})
        for i, r in enumerate(roots):
            s = pm.sub(seg, "Segment", {"id": str(i), "weight": 1.0})
            pm.sub(s, "True")
            s.append(_tree_model(r, schema, encodings, classification))
    doc = pm.build_skeleton_pmml()
    doc.add(app_pmml.build_data_dictionary(schema, encodings))
    doc.add(model)
    doc.add_extension("maxDepth", max_depth)
    doc.add_extension("maxSplitCandidates", max_split_candidates)
    doc.add_extension("impurity", impurity)
    return doc
