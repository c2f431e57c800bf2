"""k-means speed layer: assign new points, running-mean update of the touched clusters.

Equivalent of ``KMeansSpeedModel`` / ``KMeansSpeedModelManager``
(``[speed-app]/kmeans/KMeansSpeedModel.java:31-63``,
``[speed-app]/kmeans/KMeansSpeedModelManager.java:58-125``):

* ``consume``: ``MODEL``/``MODEL-REF`` -> validate against the schema and load the clusters;
  ``UP`` is ignored (the layer hears its own updates);
* ``build_updates``: the interval's points are assigned in one batched device pass, the
  per-cluster (sum, count) reduced with ``index_add``, and each touched cluster is updated with
  ``ClusterInfo.update(mean, count)``; output ``[clusterID,[center...],count]`` per cluster, in
  ascending cluster position.
"""

from __future__ import annotations

import logging
from typing import List, Optional

import numpy as np
import torch

from ... import ingest, native
from ...api import Dataset, SpeedModel, SpeedModelManager
from ...utils import pmml as pmmlu, text
from ..features import parse_features
from ..schema import InputSchema
from .common import ClusterSet, parse_feature_matrix, read_clusters, validate_pmml_vs_schema

__all__ = ["KMeansSpeedModel", "KMeansSpeedModelManager"]

log = logging.getLogger(__name__)


def _default_device():
    return torch.device("cuda") if torch.cuda.is_available() else None


class KMeansSpeedModel(SpeedModel):
    def __init__(self, clusters, device=None):
        self.clusters = ClusterSet(clusters, device if device is not None else _default_device())

    def get_cluster(self, index: int):
        return self.clusters.get(index)

    def set_cluster(self, index: int, info) -> None:
        self.clusters.set(index, info)

    def closest_cluster(self, vector):
        return self.clusters.nearest(vector)[0]

    def get_fraction_loaded(self) -> float:
        return 1.0

    def __repr__(self):
        return "KMeansSpeedModel[numClusters=%d]" % len(self.clusters)


class KMeansSpeedModelManager(SpeedModelManager):
    def __init__(self, config):
        self.input_schema = InputSchema(config)
        self.model: Optional[KMeansSpeedModel] = None
        self.last_phase_ms: dict = {}

    def consume(self, updates, context=None) -> None:
        for km in updates:
            key, message = km.key, km.message
            if key is None:
                raise ValueError("Bad message: %r" % (km,))
            if key == "UP":
                continue
            if key in ("MODEL", "MODEL-REF"):
                log.info("Loading new model")
                pmml = pmmlu.read_pmml_from_update_key_message(key, message)
                validate_pmml_vs_schema(pmml, self.input_schema)
                self.model = KMeansSpeedModel(read_clusters(pmml))
                log.info("New model loaded: %s", self.model)
            else:
                raise ValueError("Bad message: %r" % (km,))

    def build_updates(self, new_data: Dataset) -> List[str]:
        model = self.model
        if model is None:
            return []
        cs = model.clusters
        if (cs.device is not None and cs.device.type == "cuda" and native.kernels_available()
                and 0 < self.input_schema.get_num_predictors() <= 1024):
            return self._build_updates_device(new_data)
        x = parse_feature_matrix(new_data.values(), self.input_schema)
        if len(x) == 0:
            return []
        idx, _ = model.clusters.nearest_batch(x)
        k = len(model.clusters)
        sums = np.zeros((k, x.shape[1]), dtype=np.float64)
        np.add.at(sums, idx, x)
        counts = np.bincount(idx, minlength=k)
        out = []
        for pos in np.nonzero(counts)[0].tolist():
            info = model.get_cluster(pos)
            info.update(sums[pos] / counts[pos], int(counts[pos]))
            model.set_cluster(pos, info)
            out.append(text.join_json([info.id, [float(v) for v in info.center], info.count]))
        return out

    def _build_updates_device(self, new_data: Dataset):
        """The GPU path: the micro-batch parsed natively straight to a device fp64 matrix
        (models/features.parse_features), nearest clusters by the exact fp64 kernel,
        per-cluster sums / counts by index_add / bincount, the running means of the touched
        clusters (ClusterInfo.update's formula, vectorised), and the messages formatted
        natively (ingest.format_cluster_updates: the same bytes as text.join_json) in one
        MessageBlock."""
        import time
        from ...textlines import TextLines
        t0 = time.perf_counter()
        cs = self.model.clusters
        lines = new_data.values()
        if not isinstance(lines, TextLines):
            lines = TextLines.from_strings([str(v) for v in lines])
        if len(lines) == 0:
            return []
        block = parse_features(lines, self.input_schema, cs.device, torch.float64)
        x = block.predictors(self.input_schema)
        if x.shape[0] == 0:
            return []
        t1 = time.perf_counter()
        idx, _ = cs.nearest_batch_device(x)
        centers, _, counts = cs.device_state()
        k, d = centers.shape
        sums = torch.zeros((k, d), dtype=torch.float64, device=x.device)
        sums.index_add_(0, idx, x.to(torch.float64))
        n_new = torch.bincount(idx, minlength=k)
        touched = torch.nonzero(n_new).flatten()
        nt = n_new[touched]
        total = nt + counts[touched]
        c = centers[touched]
        mean = sums[touched] / nt[:, None].to(torch.float64)
        frac = nt.to(torch.float64) / total.to(torch.float64)
        new_c = c + frac[:, None] * (mean - c)
        # one copy to the host: [position, center..., count] rows (integers exact in fp64)
        packed = torch.cat([touched.to(torch.float64)[:, None], new_c,
                            total.to(torch.float64)[:, None]], 1).cpu().numpy()
        pos_h = packed[:, 0].astype(np.int64)
        new_h = np.ascontiguousarray(packed[:, 1:d + 1])
        tot_h = packed[:, d + 1].astype(np.int64)
        t2 = time.perf_counter()
        cs.set_many(pos_h.tolist(), new_h, tot_h.tolist(),
                    device_update=(touched, new_c, total))
        ids = np.array([cs.clusters[p].id for p in pos_h.tolist()], dtype=np.int64)
        t3 = time.perf_counter()
        out = ingest.format_cluster_updates(ids, new_h, tot_h, device_centers=new_c)
        # milliseconds per phase of the last micro-batch (parse: text -> device matrix;
        # assign_update: nearest clusters, sums, running means, results to the host;
        # set: the model's host / device state; format: the UP messages)
        self.last_phase_ms = {"parse": (t1 - t0) * 1e3, "assign_update": (t2 - t1) * 1e3,
                              "set": (t3 - t2) * 1e3,
                              "format": (time.perf_counter() - t3) * 1e3}
        return out

    def close(self) -> None:
        pass
