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
        leaves = leaves[has_target]                               # [m, T] flat node indices
        tv = target[has_target]
        if leaves.size == 0:
            return []
        # flat nodes are laid out tree by tree from each root index
        roots = flat.roots.cpu().numpy().astype(np.int64)
        flat_leaf = leaves.ravel().astype(np.int64)
        vals = np.broadcast_to(tv[:, None], leaves.shape).ravel()
        out = []
        if schema.is_classification():
            # one pass over (leaf, class) pairs: counts per leaf per class
            cls = vals.astype(np.int64)
            nc = int(cls.max()) + 1
            keys, counts = np.unique(flat_leaf * nc + cls, return_counts=True)
            leaf_k, cls_k = keys // nc, keys % nc
            bounds = np.flatnonzero(np.diff(leaf_k)) + 1
            for seg_l, seg_c, seg_n in zip(np.split(leaf_k, bounds), np.split(cls_k, bounds),
                                           np.split(counts, bounds)):
                leaf = int(seg_l[0])
                t = int(np.searchsorted(roots, leaf, side="right")) - 1
                cmap = {str(int(c)): int(k) for c, k in zip(seg_c, seg_n)}
                out.append(json.dumps([t, flat.nodes[leaf].get_id(), cmap],
                                      separators=(",", ":")))
        else:
            keys, inv, counts = np.unique(flat_leaf, return_inverse=True, return_counts=True)
            sums = np.bincount(inv, weights=vals, minlength=len(keys))
            trees = np.searchsorted(roots, keys, side="right") - 1
            for j, leaf in enumerate(keys.tolist()):
                out.append(json.dumps([int(trees[j]), flat.nodes[leaf].get_id(),
                                       float(sums[j] / counts[j]), int(counts[j])],
                                      separators=(",", ":")))
        return out

    def close(self) -> None:
        pass
