"""k-means batch-layer update: parse -> GPU k-means -> PMML ClusteringModel -> publish.

Equivalent of ``KMeansUpdate`` (``[mllib]/kmeans/KMeansUpdate.java:68-232``):

* config: ``oryx.kmeans.{initialization-strategy, evaluation-strategy, runs, iterations}`` and
  hyperparameter ``oryx.kmeans.hyperparams.k``; the input schema must have no target and no
  categorical features (unsupervised, numeric only);
* ``build_model``: records -> predictor matrix (active features) -> :func:`kmeans_train`
  (k-means|| or random init, Lloyd on the MFMA assignment kernel, best of ``runs``) -> cluster
  sizes -> PMML ``ClusteringModel`` (center-based, squared Euclidean) + DataDictionary;
* ``evaluate``: train + test points scored with the configured strategy (higher is better).

Divergence (deliberate): a cluster that ends up empty is re-seeded at the farthest point
during Lloyd, so every published cluster has size >= 1 (MLlib can return an empty cluster,
which the reference's ``fetchClusterCountsFromModel`` then fails on).
"""

from __future__ import annotations

import logging
import time
from typing import List

import numpy as np
import torch

from ...ml import hyperparams as hp
from ...ml.mlupdate import MLUpdate
from ...ops import kmeans as km_ops
from ...parallel import dist
from ...utils import rng
from ..schema import InputSchema
from . import evaluation
from .common import parse_feature_matrix, read_clusters, validate_pmml_vs_schema, \
    clustering_model_pmml

__all__ = ["KMeansUpdate"]

log = logging.getLogger(__name__)

_INIT_STRATEGIES = ("k-means||", "random")


class KMeansUpdate(MLUpdate):
    sharded_data = True

    def __init__(self, config):
        super().__init__(config)
        self.initialization_strategy = config.get_string("oryx.kmeans.initialization-strategy")
        self.evaluation_strategy = config.get_string("oryx.kmeans.evaluation-strategy")
        self.number_of_runs = config.get_int("oryx.kmeans.runs")
        self.max_iterations = config.get_int("oryx.kmeans.iterations")
        self.hyper_param_values = [hp.from_config(config, "oryx.kmeans.hyperparams.k")]
        self.input_schema = InputSchema(config)
        from ...utils import config as cfg
        self.precision = cfg.get_optional_string(config, "oryx.gpu.dtype") or "fp32"
        if self.max_iterations <= 0 or self.number_of_runs <= 0:
            raise ValueError("iterations and runs must be > 0")
        if self.initialization_strategy not in _INIT_STRATEGIES:
            raise ValueError("Unknown initialization strategy " + self.initialization_strategy)
        if self.evaluation_strategy not in evaluation.EVAL_STRATEGIES:
            raise ValueError("Unknown evaluation strategy " + self.evaluation_strategy)
        if self.input_schema.has_target():
            raise ValueError("k-means does not use a target feature")
        for i in range(self.input_schema.get_num_features()):
            if self.input_schema.is_categorical(i):
                raise ValueError("k-means supports only numeric features")

    def get_hyper_parameter_values(self):
        return self.hyper_param_values

    def _ctx(self, context) -> dist.DistContext:
        if isinstance(context, dist.DistContext):
            return context
        c = getattr(context, "dist", None)
        return c if c is not None else dist.get_context()

    def _sharded(self, ctx) -> bool:
        return ctx.is_distributed and self.dist_ctx is not None and self.dist_ctx.is_distributed

    def build_model(self, context, train_data, hyper_parameters, candidate_path):
        k = int(hyper_parameters[0])
        if k <= 1:
            raise ValueError("k must be > 1")
        ctx = self._ctx(context)
        x = parse_feature_matrix(list(train_data), self.input_schema)
        sharded = self._sharded(ctx)
        if sharded:
            from ...parallel import shuffle
            if sum(shuffle.all_gather_int(len(x), ctx)) == 0:
                return None
            if len(x) == 0:
                x = np.zeros((0, self.input_schema.get_num_predictors()), dtype=np.float64)
        elif len(x) == 0:
            return None
        t0 = time.perf_counter()
        # sharded: this rank's share of the records; otherwise every rank parsed everything
        # and takes a disjoint slice
        rows = x if sharded else x[ctx.rank::ctx.world_size]
        local = torch.from_numpy(rows.astype(np.float32)).to(ctx.device)
        res = km_ops.kmeans_train(local, k, self.max_iterations, self.number_of_runs,
                                  self.initialization_strategy, seed=rng.next_seed(),
                                  ctx=ctx, precision=self.precision)
        centers = res.centers.double().cpu().numpy()
        sizes = res.counts.cpu().numpy()
        log.info("k-means k=%d on %d points x %d: cost %.6g, %d iterations, %.3fs", k, len(x),
                 x.shape[1], res.cost, res.iterations, time.perf_counter() - t0)
        if not ctx.is_main and not sharded:
            return None
        return clustering_model_pmml(self.input_schema, centers, sizes)

    def evaluate(self, context, model, model_parent_path, test_data, train_data):
        validate_pmml_vs_schema(model, self.input_schema)
        x = parse_feature_matrix(list(train_data) + list(test_data), self.input_schema)
        clusters = read_clusters(model)
        ctx = self._ctx(context)
        if self._sharded(ctx):
            if len(x) == 0:
                x = np.zeros((0, len(clusters[0].center)), dtype=np.float64)
            ev = evaluation.evaluate_sharded(self.evaluation_strategy, clusters, x, ctx,
                                             device=ctx.device)
        else:
            ev = evaluation.evaluate(self.evaluation_strategy, clusters, x, device=ctx.device)
        log.info("k-means eval (%s): %s", self.evaluation_strategy, ev)
        return ev
