"""App-level PMML helpers: MiningSchema and DataDictionary from an :class:`InputSchema`.

Equivalent of the schema-related half of ``AppPMMLUtils``
(``[app-common]/pmml/AppPMMLUtils.java:126-254``): ``buildMiningSchema`` (with optional
per-predictor importances), ``getFeatureNames`` (MiningSchema / DataDictionary),
``findTargetIndex``, ``buildDataDictionary`` (categorical values listed in encoding order) and
``buildCategoricalValueEncodings`` (the inverse).
"""

from __future__ import annotations

import xml.etree.ElementTree as ET
from typing import List, Optional, Sequence

from ..utils import pmml as pm
from .schema import CategoricalValueEncodings, InputSchema

__all__ = ["build_mining_schema", "build_data_dictionary", "feature_names_of",
           "find_target_index", "build_categorical_value_encodings"]


def build_mining_schema(schema: InputSchema, importances: Optional[Sequence[float]] = None
                        ) -> ET.Element:
    if importances is not None and len(importances) != schema.get_num_predictors():
        raise ValueError("importances length != number of predictors")
    ms = ET.Element(pm.q("MiningSchema"))
    for fi, name in enumerate(schema.feature_names):
        attrs = {"name": name}
        if schema.is_numeric(name):
            attrs["optype"] = "continuous"
            usage = "active"
        elif schema.is_categorical(name):
            attrs["optype"] = "categorical"
            usage = "active"
        else:
            usage = "supplementary"
        if schema.has_target() and schema.is_target(name):
            usage = "predicted"
        attrs["usageType"] = usage
        if usage == "active" and importances is not None:
            attrs["importance"] = float(importances[schema.feature_to_predictor_index(fi)])
        pm.sub(ms, "MiningField", attrs)
    return ms


def feature_names_of(element: ET.Element) -> List[str]:
    """Field names of a MiningSchema or DataDictionary, in order."""
    tag = element.tag.split("}")[-1]
    child = "MiningField" if tag == "MiningSchema" else "DataField"
    names = [f.get("name") for f in element.findall(pm.q(child))]
    if tag == "DataDictionary" and not names:
        raise ValueError("No fields in DataDictionary")
    return names


def find_target_index(mining_schema: ET.Element) -> Optional[int]:
    for i, f in enumerate(mining_schema.findall(pm.q("MiningField"))):
        if f.get("usageType") == "predicted":
            return i
    return None


def build_data_dictionary(schema: InputSchema,
                          encodings: Optional[CategoricalValueEncodings]) -> ET.Element:
    dd = ET.Element(pm.q("DataDictionary"), {"numberOfFields": str(schema.get_num_features())})
    for fi, name in enumerate(schema.feature_names):
        attrs = {"name": name}
        if schema.is_numeric(name):
            attrs["optype"] = "continuous"
            attrs["dataType"] = "double"
        elif schema.is_categorical(name):
            attrs["optype"] = "categorical"
            attrs["dataType"] = "string"
        field = pm.sub(dd, "DataField", attrs)
        if schema.is_categorical(name) and encodings is not None:
            for v in encodings.values_in_order(fi):
                pm.sub(field, "Value", {"value": v})
    return dd


def build_categorical_value_encodings(dictionary: ET.Element) -> CategoricalValueEncodings:
    index_to_values = {}
    for fi, field in enumerate(dictionary.findall(pm.q("DataField"))):
        values = [v.get("value") for v in field.findall(pm.q("Value"))]
        if values:
            index_to_values[fi] = values
    return CategoricalValueEncodings(index_to_values)
