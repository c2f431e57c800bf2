"""k-means serving model and manager.

Equivalent of ``KMeansServingModel`` (``[serving-app]/kmeans/model/KMeansServingModel.java:34-87``)
and ``KMeansServingModelManager.consume``
(``[serving-app]/kmeans/model/KMeansServingModelManager.java:61-96``): ``MODEL``/``MODEL-REF``
replaces the cluster list (validated against the input schema); ``UP``
``[clusterID,[center],count]`` replaces the cluster at that position.  Single queries scan the
host float64 centers; batches go through :meth:`ClusterSet.nearest_batch` on the device.
"""

from __future__ import annotations

import logging
from typing import List, Optional, Sequence

import numpy as np
import torch

from ...api import AbstractServingModelManager, ServingModel
from ...utils import pmml as pmmlu, text
from ..schema import InputSchema
from .common import (ClusterInfo, ClusterSet, features_from_tokens, read_clusters,
                     validate_pmml_vs_schema)

__all__ = ["KMeansServingModel", "KMeansServingModelManager"]

log = logging.getLogger(__name__)


def _default_device():
    return torch.device("cuda") if torch.cuda.is_available() else None


class KMeansServingModel(ServingModel):
    def __init__(self, clusters: List[ClusterInfo], input_schema: InputSchema, device=None):
        if clusters is None or input_schema is None:
            raise ValueError("clusters and schema are required")
        self.clusters = ClusterSet(clusters, device if device is not None else _default_device())
        self.input_schema = input_schema

    def _features(self, datum: Sequence[str]) -> np.ndarray:
        if len(datum) != self.input_schema.get_num_features():
            raise ValueError("Wrong number of features")
        return features_from_tokens(datum, self.input_schema)

    def nearest_cluster_id(self, datum: Sequence[str]) -> int:
        return self.closest_cluster(self._features(datum))[0].id

    def nearest_cluster_ids(self, data: Sequence[Sequence[str]]) -> List[int]:
        x = np.stack([self._features(d) for d in data])
        pos, _ = self.clusters.nearest_batch(x)
        return [self.clusters.get(int(p)).id for p in pos]

    def get_num_clusters(self) -> int:
        return len(self.clusters)

    def get_cluster(self, index: int) -> ClusterInfo:
        return self.clusters.get(index)

    def get_input_schema(self) -> InputSchema:
        return self.input_schema

    def closest_cluster(self, vector):
        return self.clusters.nearest(vector)

    def update(self, cluster_id: int, center, count: int) -> None:
        self.clusters.set(cluster_id, ClusterInfo(cluster_id, center, count))

    def get_fraction_loaded(self) -> float:
        return 1.0

    def __repr__(self):
        return "KMeansServingModel[clusters:%d]" % len(self.clusters)


class KMeansServingModelManager(AbstractServingModelManager):
    def __init__(self, config):
        super().__init__(config)
        self.input_schema = InputSchema(config)
        self.model: Optional[KMeansServingModel] = None

    def consume(self, updates, context=None) -> None:
        for km in updates:
            key, message = km.key, km.message
            if key is None:
                raise ValueError("Bad message: %r" % (km,))
            if key == "UP":
                if self.model is None:
                    continue
                update = text.read_json(message)
                self.model.update(int(update[0]), np.asarray(update[1], dtype=np.float64),
                                  int(update[2]))
            elif key in ("MODEL", "MODEL-REF"):
                log.info("Loading new model")
                pmml = pmmlu.read_pmml_from_update_key_message(key, message)
                validate_pmml_vs_schema(pmml, self.input_schema)
                self.model = KMeansServingModel(read_clusters(pmml), self.input_schema)
                log.info("New model: %s", self.model)
            else:
                raise ValueError("Bad message: %r" % (km,))

    def get_model(self) -> Optional[KMeansServingModel]:
        return self.model
