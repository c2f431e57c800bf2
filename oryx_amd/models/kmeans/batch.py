"""k-means batch-layer update: parse -> GPU k-means -> PMML ClusteringModel -> publish.

Equivalent of ``KMeansUpdate`` (``[mllib]/kmeans/KMeansUpdate.java:68-232``):

* config: ``oryx.kmeans.{initialization-strategy, evaluation-strategy, runs, iterations}`` and
  hyperparameter ``oryx.kmeans.hyperparams.k``; the input schema must have no target and no
  categorical features (unsupervised, numeric only);
* ``build_model``: records -> predictor matrix (active features) -> :func:`kmeans_train`
  (k-means|| or random init, Lloyd on the MFMA assignment kernel, best of ``runs``) -> cluster
  sizes -> PMML ``ClusteringModel`` (center-based, squared Euclidean) + DataDictionary;
* ``evaluate``: train + test points scored with the configured strategy (higher is better).

Records are parsed natively straight to a device float32 matrix, and past part files' parses
stay resident on the device across generations (:mod:`oryx_amd.models.features`).

Divergence (deliberate, ``oryx.kmeans.reseed-empty-clusters``, default true): a cluster that
ends up empty is re-seeded at the farthest point during Lloyd, so every published cluster has
size >= 1.  MLlib keeps an empty cluster's old center (false here), and the reference's
``fetchClusterCountsFromModel`` + ``pmmlClusteringModel`` then fail on the missing count
(``KMeansUpdate.java:127-130``, ``:192-221``); with false this update publishes it with size 0.
"""

from __future__ import annotations

import logging
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from ...ml import hyperparams as hp
from ...ml.mlupdate import MLUpdate
from ...ops import kmeans as km_ops
from ...parallel import dist
from ...textlines import concat_lines
from ...utils import rng
from ..features import FeatureHistory, parse_features
from ..schema import InputSchema
from . import evaluation
from .common import ClusterInfo, read_clusters, validate_pmml_vs_schema, clustering_model_pmml

__all__ = ["KMeansUpdate"]

log = logging.getLogger(__name__)

_INIT_STRATEGIES = ("k-means||", "random")


class KMeansUpdate(MLUpdate):
    sharded_data = True
    # the interval is saved as several part files when large; FeatureHistory adopts each
    # from the interval's parse (models/features.py)
    split_interval_files = True

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
        rs = cfg.get_optional_bool(config, "oryx.kmeans.reseed-empty-clusters")
        self.reseed_empty = True if rs is None else bool(rs)
        rh = cfg.get_optional_bool(config, "oryx.kmeans.resident-history")
        self.resident_history = True if rh is None else bool(rh)
        self.history: Optional[FeatureHistory] = None
        self.phase_seconds: Dict[str, float] = {}
        # the "train" phase broken down (kmeans_train's timings; accumulates like the above)
        self.train_phases: Dict[str, float] = {}
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

    def warm_up(self, context) -> None:
        """Start-up warm-up (``BatchLayer.warm_up``): k-means on a few thousand random points
        of the schema's dimension with every configured k, on this rank's device (the assign
        / accumulate / k-means|| kernels of those shapes load here).  Local."""
        ctx = self._ctx(context)
        dev = ctx.device
        if dev.type != "cuda":
            return
        d = self.input_schema.get_num_predictors()
        ks = sorted({int(round(float(v))) for v in
                     self.hyper_param_values[0].get_trial_values(max(1, self.candidates))})
        local = dist.DistContext(device=dev)
        g = torch.Generator(device=dev).manual_seed(1)
        for k in ks:
            if k <= 1:
                continue
            x = torch.randn((max(4096, 4 * k), d), device=dev, generator=g)
            km_ops.kmeans_train(x, k, 2, 1, self.initialization_strategy, seed=1, ctx=local,
                                precision=self.precision, reseed_empty=self.reseed_empty)
        torch.cuda.synchronize(dev)

    def _ctx(self, context) -> dist.DistContext:
        if isinstance(context, dist.DistContext):
            return context
        c = getattr(context, "dist", None)
        return c if c is not None else dist.get_context()

    def _sharded(self, ctx) -> bool:
        return ctx.is_distributed and self.dist_ctx is not None and self.dist_ctx.is_distributed

    def _history_for(self, device) -> Optional[FeatureHistory]:
        if not self.resident_history:
            return None
        dev = torch.device(device) if device is not None else torch.device("cpu")
        if self.history is None or self.history.device != dev:
            self.history = FeatureHistory(dev)
        return self.history

    def _points(self, lines, ctx) -> torch.Tensor:
        """This rank's records -> predictor matrix, float64 on the device: the evaluation
        metrics score the parsed values in double precision as the reference does
        (KMeansUpdate.java:139-178); training takes a float32 copy."""
        tp = time.perf_counter()
        blk = parse_features(lines, self.input_schema, ctx.device, torch.float64,
                             history=self._history_for(ctx.device))
        x = blk.predictors(self.input_schema).contiguous()
        self.phase_seconds["parse"] = self.phase_seconds.get("parse", 0.0) + \
            time.perf_counter() - tp
        return x

    def build_model(self, context, train_data, hyper_parameters, candidate_path):
        k = int(hyper_parameters[0])
        if k <= 1:
            raise ValueError("k must be > 1")
        ctx = self._ctx(context)
        x64 = self._points(train_data, ctx)
        # the evaluation of this candidate scores train + test points: it takes these parsed
        # rows instead of re-joining and re-reading the training text
        self._train_points = (train_data, x64)
        sharded = self._sharded(ctx)
        n = int(x64.shape[0])
        if sharded:
            from ...parallel import shuffle
            if sum(shuffle.all_gather_int(n, ctx)) == 0:
                return None
        elif n == 0:
            return None
        # train in float32 on points shifted by the (global) mean: k-means is translation
        # invariant, and the fp32 distance expansion |x|^2 - 2 x.c + |c|^2 loses everything to
        # cancellation when features carry a large common offset; the shift comes back on the
        # centers in float64
        t0 = time.perf_counter()
        s = torch.stack([x64.sum(0), torch.full((x64.shape[1],), float(n), dtype=torch.float64,
                                                 device=x64.device)])
        if sharded:
            dist.all_reduce_sum(s, ctx)
        shift = s[0] / s[1].clamp_min(1.0)
        # shifted and narrowed in row slices: (x64 - shift) whole would be another float64
        # copy of the matrix (25.6 GB at 12.5M x 256) on top of the parse and the result
        x = torch.empty(x64.shape, dtype=torch.float32, device=x64.device)
        step = max(1, (1 << 27) // max(1, x64.shape[1]))
        for lo in range(0, n, step):
            x[lo:lo + step] = (x64[lo:lo + step] - shift).float()
        tm = self.train_phases
        if x.device.type == "cuda":
            torch.cuda.synchronize(x.device)
        tm["shift"] = tm.get("shift", 0.0) + time.perf_counter() - t0
        # sharded: this rank's share of the records; otherwise every rank parsed everything
        # and takes a disjoint slice
        local = x if sharded else x[ctx.rank::ctx.world_size].contiguous()
        res = km_ops.kmeans_train(local, k, self.max_iterations, self.number_of_runs,
                                  self.initialization_strategy, seed=rng.next_seed(),
                                  ctx=ctx, precision=self.precision,
                                  reseed_empty=self.reseed_empty, timings=tm)
        centers = (res.centers.double() + shift).cpu().numpy()
        sizes = res.counts.cpu().numpy()
        self.phase_seconds["train"] = self.phase_seconds.get("train", 0.0) + \
            time.perf_counter() - t0
        log.info("k-means k=%d on %d points x %d: cost %.6g, %d iterations, %.3fs", k, n,
                 x.shape[1], res.cost, res.iterations, time.perf_counter() - t0)
        if not ctx.is_main and not sharded:
            return None
        tp = time.perf_counter()
        pmml = clustering_model_pmml(self.input_schema, centers, sizes)
        # the evaluation of this candidate takes the clusters as built instead of parsing them
        # back out of the PMML (its real arrays are shortest round-trip decimals: the same
        # doubles)
        try:
            self._built_clusters = (pmml, [ClusterInfo(i, centers[i].tolist(), int(sizes[i]))
                                           for i in range(len(centers))])
        except ValueError:               # (e.g. an empty cluster: the PMML path decides)
            self._built_clusters = None
        self.phase_seconds["pmml"] = self.phase_seconds.get("pmml", 0.0) + \
            time.perf_counter() - tp
        return pmml

    def evaluate(self, context, model, model_parent_path, test_data, train_data):
        validate_pmml_vs_schema(model, self.input_schema)
        ctx = self._ctx(context)
        cached = getattr(self, "_train_points", None)
        self._train_points = None
        if cached is not None and cached[0] is train_data:
            # rows in the order of concat_lines([train, test]): the training rows, then the
            # test rows (the evaluation sums over points, so a rank's row order is immaterial)
            x = cached[1]
            if test_data is not None and len(test_data):
                x = torch.cat([x, self._points(test_data, ctx)])
        else:
            x = self._points(concat_lines([train_data, test_data]), ctx)
        tp = time.perf_counter()
        built = getattr(self, "_built_clusters", None)
        self._built_clusters = None
        clusters = built[1] if built is not None and built[0] is model else read_clusters(model)
        if self._sharded(ctx):
            ev = evaluation.evaluate_sharded(self.evaluation_strategy, clusters, x, ctx,
                                             device=ctx.device)
        else:
            ev = evaluation.evaluate(self.evaluation_strategy, clusters, x, device=ctx.device)
        self.phase_seconds["eval"] = self.phase_seconds.get("eval", 0.0) + \
            time.perf_counter() - tp
        log.info("k-means eval (%s): %s", self.evaluation_strategy, ev)
        return ev
