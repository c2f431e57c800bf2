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

from ... import ingest
from ...api import Dataset, SpeedModel, SpeedModelManager
from ...ops import rdf as rdf_ops
from ...utils import pmml as pmmlu, text
from ..schema import InputSchema
from . import pmml as rdf_pmml
from .batch import parse_csv_block, parse_examples

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
            # per flat node: its tree and its ID as JSON text (the update messages' fields)
            roots = self._flat.roots.cpu().numpy().astype(np.int64)
            n = len(self._flat.nodes)
            self.tree_of = np.searchsorted(roots, np.arange(n), side="right") - 1
            self.id_blob, self.id_ends = ingest.strings_blob(
                [json.dumps(nd.get_id()) for nd in self._flat.nodes])
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
        # milliseconds per phase of the last micro-batch on the GPU path (parse: text ->
        # encoded host rows; leaves: upload + forest traversal; counts_format: per-leaf counts
        # or sums, results to the host, the UP messages)
        self.last_phase_ms: dict = {}

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
        import time
        t0 = time.perf_counter()
        schema = self.input_schema
        values = new_data.values()
        if not len(values):
            return []
        C = model.encodings.get_value_count(schema.get_target_feature_index()) \
            if schema.is_classification() else 0
        if self.device.type == "cuda":
            self.last_phase_ms = {}
            got = self._parse_device(values, model)
            if got is not None:
                t1 = time.perf_counter()
                flat = model.flat(self.device, C)
                self.last_phase_ms["flat"] = (time.perf_counter() - t1) * 1e3
                self.last_phase_ms["parse"] = (t1 - t0) * 1e3
                return self._updates_device(model, flat, got[0], got[1], C)
        parsed = parse_csv_block(values, schema, model.encodings)
        if parsed is None:
            rows = [text.parse_input_line(v) for v in values]
            parsed = parse_examples(rows, schema, model.encodings, require_target=False)
        _, target, full = parsed
        flat = model.flat(self.device, C)
        if self.device.type == "cuda":
            self.last_phase_ms = {"parse": (time.perf_counter() - t0) * 1e3}
            return self._updates_device(model, flat, full, target, C)
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
        # node ids of the touched leaves, looked up once per distinct leaf
        if schema.is_classification():
            # one pass over (leaf, class) pairs: counts per leaf per class
            cls = vals.astype(np.int64)
            nc = int(cls.max()) + 1
            keys, counts = np.unique(flat_leaf * nc + cls, return_counts=True)
            leaf_k, cls_k = keys // nc, keys % nc
            starts = np.flatnonzero(np.r_[True, np.diff(leaf_k) != 0])
            ends = np.r_[starts[1:], len(leaf_k)]
            trees = (np.searchsorted(roots, leaf_k[starts], side="right") - 1).tolist()
            leaf_l, cls_l, cnt_l = leaf_k.tolist(), cls_k.tolist(), counts.tolist()
            for j, (a, b) in enumerate(zip(starts.tolist(), ends.tolist())):
                cmap = ",".join('"%d":%d' % (cls_l[q], cnt_l[q]) for q in range(a, b))
                out.append('[%d,%s,{%s}]' % (trees[j], json.dumps(flat.nodes[leaf_l[a]].get_id()),
                                             cmap))
        else:
            keys, inv, counts = np.unique(flat_leaf, return_inverse=True, return_counts=True)
            sums = np.bincount(inv, weights=vals, minlength=len(keys))
            trees = (np.searchsorted(roots, keys, side="right") - 1).tolist()
            means = (sums / counts).tolist()
            for j, leaf in enumerate(keys.tolist()):
                out.append(json.dumps([trees[j], flat.nodes[leaf].get_id(), means[j],
                                       int(counts[j])], separators=(",", ":")))
        return out

    def _parse_device(self, values, model):
        """(full fp64 [n, F], target [n]) of a TextLines micro-batch parsed on the device
        (``features.parse_features``: the CSV kernel, categorical spans encoded on the host)
        with the categorical codes mapped to the model's encodings -- the matrix the host path
        (``parse_csv_block``) builds, without the host parse of every value and the upload
        (2.0 of a 4.1 ms interval at 10k x 100 features).  None when the host path should take
        the batch: not a TextLines buffer, no device parser, a category the model does not know
        or an empty predictor (the general path's cases)."""
        from ...textlines import TextLines
        from ..features import _device_ok, parse_features
        schema = self.input_schema
        if not isinstance(values, TextLines) or not _device_ok(schema, self.device):
            return None
        import time
        t0 = time.perf_counter()
        blk = parse_features(values, schema, self.device, torch.float64)
        full = blk.full.to(self.device, torch.float64)
        self.last_phase_ms["parse_text"] = (time.perf_counter() - t0) * 1e3
        if full.shape[0] != len(values):
            return None                      # (an empty line the parser skipped)
        for f, vs in (blk.values or {}).items():
            m = model.encodings.get_value_encoding_map(f)
            codes = [m.get(v) for v in vs]
            if any(c is None for c in codes):
                return None
            lut = torch.tensor([float(c) for c in codes] + [float("nan")], dtype=torch.float64,
                               device=self.device)
            col = full[:, f]
            idx = torch.where(torch.isnan(col), len(vs), torch.nan_to_num(col).to(torch.int64))
            full[:, f] = lut[idx]
        F = schema.get_num_features()
        unused = [f for f in range(F) if not schema.is_numeric(f) and
                  not schema.is_categorical(f)]
        if unused:
            full[:, unused] = 0.0
        num_pred = [f for f in range(F) if schema.is_numeric(f) and not schema.is_target(f)]
        if num_pred and bool(torch.isnan(full[:, num_pred]).any()):
            return None
        if schema.has_target():
            target = full[:, schema.get_target_feature_index()]
        else:
            target = torch.full((full.shape[0],), float("nan"), dtype=torch.float64,
                                device=self.device)
        return full, target

    def _updates_device(self, model, flat, full, target, C: int):
        """Leaves by the traversal kernel, per-(leaf, class) counts (or per-leaf sums) by one
        bincount on the device, the touched leaves' messages formatted natively
        (``ingest.format_leaf_updates``): one MessageBlock."""
        import time
        t0 = time.perf_counter()
        ph = self.last_phase_ms
        dev = self.device
        X = full if torch.is_tensor(full) else torch.from_numpy(np.ascontiguousarray(full)).to(dev)
        leaves = rdf_ops.forest_leaves(flat, X)                      # [n, T] int64
        tv = target if torch.is_tensor(target) else \
            torch.from_numpy(np.ascontiguousarray(target)).to(dev)
        ok = ~torch.isnan(tv)
        leaves, tv = leaves[ok], tv[ok]
        if leaves.numel() == 0:
            return []
        t1 = time.perf_counter()
        ph["leaves"] = (t1 - t0) * 1e3
        n_nodes = len(flat.nodes)
        T = leaves.shape[1]
        if C > 0:
            cls = tv.to(torch.int64).clamp(0, C - 1)
            key = (leaves * C + cls[:, None]).reshape(-1)
            cnt = torch.bincount(key, minlength=n_nodes * C).view(n_nodes, C)
            touched = torch.nonzero(cnt.sum(1)).flatten()
            # one copy to the host: [node, class counts...] rows
            packed = torch.cat([touched[:, None], cnt[touched]], 1).cpu().numpy()
            t_h = np.ascontiguousarray(packed[:, 0])
            c_h = np.ascontiguousarray(packed[:, 1:])
            out = ingest.format_leaf_updates(model.tree_of[t_h], model.id_blob,
                                             model.id_ends, t_h, c_h, C)
            ph["counts_format"] = (time.perf_counter() - t1) * 1e3
            return out
        flat_leaf = leaves.reshape(-1)
        vals = tv[:, None].expand(-1, T).reshape(-1)
        cnt = torch.bincount(flat_leaf, minlength=n_nodes)
        sums = torch.zeros(n_nodes, dtype=torch.float64, device=dev).index_add_(0, flat_leaf,
                                                                                vals)
        touched = torch.nonzero(cnt).flatten()
        # one copy to the host: [node, count, mean] rows (integers exact in fp64)
        nt = cnt[touched]
        packed = torch.stack([touched.to(torch.float64), nt.to(torch.float64),
                              sums[touched] / nt.to(torch.float64)], 1).cpu().numpy()
        t_h = packed[:, 0].astype(np.int64)
        n_h = packed[:, 1].astype(np.int64)
        m_h = np.ascontiguousarray(packed[:, 2])
        out = ingest.format_leaf_updates(model.tree_of[t_h], model.id_blob, model.id_ends,
                                         t_h, n_h, 0, m_h)
        ph["counts_format"] = (time.perf_counter() - t1) * 1e3
        return out

    def close(self) -> None:
        pass
