"""RDF speed layer: route new examples to their leaves, emit per-leaf statistics.

Equivalent of ``RDFSpeedModel`` / ``RDFSpeedModelManager``
(``[speed-app]/rdf/RDFSpeedModel.java:28-58``, ``RDFSpeedModelManager.java:70-151``):
``MODEL``/``MODEL-REF`` loads forest + encodings (validated against the schema), ``UP`` is
ignored; ``build_updates`` finds every example's terminal node in every tree (one batched
device traversal over the flattened forest) and groups targets by (tree, node):
classification -> ``[treeID,"nodeID",{"encoding":count,...}]``, regression ->
``[treeID,"nodeID",mean,count]``.
"""

from __future__ import annotations

import json
import logging
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ...api import Dataset, SpeedModel, SpeedModelManager
from ...ops import rdf as rdf_ops
from ...utils import pmml as pmmlu, text
from ..schema import InputSchema
from . import pmml as rdf_pmml
from .batch import parse_examples

__all__ = ["RDFSpeedModel", "RDFSpeedModelManager"]

log = logging.getLogger(__name__)


def _device():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class RDFSpeedModel(SpeedModel):
    def __init__(self, forest, encodings):
        if forest is None or encodings is None:
            raise ValueError("forest and encodings are required")
        self.forest = forest
        self.encodings = encodings
        self._flat = None

    def get_forest(self):
        return self.forest

    def get_encodings(self):
        return self.encodings

    def flat(self, device, num_classes):
        if self._flat is None:
            self._flat = rdf_ops.flatten_forest(self.forest, device, num_classes)
        return self._flat

    def get_fraction_loaded(self) -> float:
        return 1.0

    def __repr__(self):
        return "RDFSpeedModel[numTrees:%d]" % len(self.forest.get_trees())


class RDFSpeedModelManager(SpeedModelManager):
    def __init__(self, config):
        self.input_schema = InputSchema(config)
        self.model: Optional[RDFSpeedModel] = None
        self.device = _device()

    def consume(self, updates, context=None) -> None:
        for km in updates:
            if km.key is None:
                raise ValueError("Bad message: %r" % (km,))
            if km.key == "UP":
                continue
            if km.key in ("MODEL", "MODEL-REF"):
                log.info("Loading new model")
                pmml = pmmlu.read_pmml_from_update_key_message(km.key, km.message)
                rdf_pmml.validate_pmml_vs_schema(pmml, self.input_schema)
                forest, encodings = rdf_pmml.read(pmml)
                self.model = RDFSpeedModel(forest, encodings)
                log.info("New model loaded: %s", self.model)
            else:
                raise ValueError("Bad message: %r" % (km,))

    def build_updates(self, new_data: Dataset) -> List[str]:
        model = self.model
        if model is None:
            return []
        schema = self.input_schema
        rows = [text.parse_input_line(v) for v in new_data.values()]
        if not rows:
            return []
        _, target, full = parse_examples(rows, schema, model.encodings, require_target=False)
        C = model.encodings.get_value_count(schema.get_target_feature_index()) \
            if schema.is_classification() else 0
        flat = model.flat(self.device, C)
        leaves = rdf_ops.forest_leaves(flat, torch.from_numpy(full).to(self.device)).cpu() \
            .numpy()                                             # [n, T]
        has_target = ~np.isnan(target)
        groups: Dict[Tuple[int, str], list] = {}
        for e in np.nonzero(has_target)[0].tolist():
            for t in range(leaves.shape[1]):
                node = flat.nodes[int(leaves[e, t])]
                groups.setdefault((t, node.get_id()), []).append(target[e])
        out = []
        for (t, node_id), vals in groups.items():
            if schema.is_classification():
                counts: Dict[str, int] = {}
                for v in vals:
                    k = str(int(v))
                    counts[k] = counts.get(k, 0) + 1
                out.append(json.dumps([t, node_id, counts], separators=(",", ":")))
            else:
                arr = np.asarray(vals, dtype=np.float64)
                out.append(json.dumps([t, node_id, float(arr.mean()), int(len(arr))],
                                      separators=(",", ":")))
        return out

    def close(self) -> None:
        pass
