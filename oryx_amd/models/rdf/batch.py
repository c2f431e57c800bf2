"""RDF batch-layer update: parse -> encode -> GPU random forest -> PMML -> publish.

Equivalent of ``RDFUpdate`` (``[mllib]/rdf/RDFUpdate.java:97-558``) and ``Evaluation``
(``[mllib]/rdf/Evaluation.java:32-53``):

* config ``oryx.rdf.num-trees`` and hyperparameters ``max-split-candidates``, ``max-depth``,
  ``impurity``; the input schema must have a target (categorical -> classification);
* categorical values are encoded in order of first appearance over the training data;
* training: :func:`oryx_amd.ops.rdf.train_forest` (HIP histogram + routing kernels);
* PMML: TreeModel (one tree) or MiningModel with one segment per tree; node record counts
  and feature importances (share of decision-node visits per predictor) come from pushing all
  training examples through the trees, as the reference does;
* evaluation: accuracy (classification) or -RMSE (regression) of the forest on the test set,
  scored on the device over the flattened trees.
"""

from __future__ import annotations

import io
import logging
import math
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...ml import hyperparams as hp
from ...ml.mlupdate import MLUpdate
from ...ops import rdf as rdf_ops
from ...parallel import dist
from ...utils import rng, text
from ..classreg import CategoricalPrediction, NumericPrediction
from ..features import FeatureBlock, FeatureHistory, parse_features
from ..schema import CategoricalValueEncodings, InputSchema
from . import pmml as rdf_pmml
from .pmml import TreeSpecNode

__all__ = ["RDFUpdate", "parse_examples", "distinct_values", "evaluate_forest"]

log = logging.getLogger(__name__)


def distinct_values(rows: Sequence[Sequence[str]], schema: InputSchema) -> Dict[int, List[str]]:
    """Categorical feature index -> distinct values in order of first appearance."""
    cats = [i for i in range(schema.get_num_features()) if schema.is_categorical(i)]
    seen: Dict[int, Dict[str, None]] = {i: {} for i in cats}
    for r in rows:
        for i in cats:
            seen[i].setdefault(r[i], None)
    return {i: list(v.keys()) for i, v in seen.items()}


def parse_csv_block(lines: Sequence[str], schema: InputSchema,
                    encodings: CategoricalValueEncodings):
    """Fast path of ``parse_input_line`` + :func:`parse_examples` for a block of plain CSV
    lines (no JSON arrays, no quoting): one C-level CSV parse (pandas) with numeric columns
    read straight to float64.  Returns ``(X, target, full)`` or None when the block does not
    qualify (the caller then takes the general path)."""
    if not len(lines):
        return None
    from ...textlines import TextLines
    F = schema.get_num_features()
    if isinstance(lines, TextLines):
        # the buffer as drained: parsed in place (no per-line strings)
        buf = lines.joined()
        data = buf.tobytes() if isinstance(buf, np.ndarray) else bytes(buf)
        full = _native_csv_block(data, len(lines), schema, encodings, F)
        if full is not None:
            return _split_full(full, schema)
        lines = list(lines)
    blob = "\n".join(lines)
    # the native parser rejects quotes, backslashes and JSON-array lines itself
    full = _native_csv_block(blob, len(lines), schema, encodings, F)
    if full is not None:
        return _split_full(full, schema)
    if '"' in blob or "\\" in blob or "[" in blob:
        return None
    try:
        import pandas as pd
    except ImportError:                                     # pragma: no cover
        return None
    dtypes = {fi: (np.float64 if schema.is_numeric(fi) else str) for fi in range(F)}
    try:
        df = pd.read_csv(io.StringIO(blob), header=None, dtype=dtypes, names=list(range(F)),
                         keep_default_na=False, na_values={fi: [""] for fi in range(F)
                                                           if schema.is_numeric(fi)},
                         engine="c")
    except (ValueError, pd.errors.ParserError):
        return None
    if len(df) != len(lines) or df.shape[1] != F:
        return None
    n = len(df)
    full = np.zeros((n, F), dtype=np.float64)
    for fi in range(F):
        col = df[fi]
        if schema.is_numeric(fi):
            v = col.to_numpy(dtype=np.float64)
            if np.isnan(v).any() and not schema.is_target(fi):
                return None                                  # empty predictor: general path
            full[:, fi] = v
        elif schema.is_categorical(fi):
            m = encodings.get_value_encoding_map(fi)
            uniq, inv = np.unique(col.to_numpy(dtype=str), return_inverse=True)
            try:
                codes = np.array([m[u] if u != "" else np.nan for u in uniq.tolist()],
                                 dtype=np.float64)
            except KeyError:
                return None                                  # unknown value: general path
            if not schema.is_target(fi) and np.isnan(codes).any():
                return None
            full[:, fi] = codes[inv.reshape(-1)]
    return _split_full(full, schema)


def _split_full(full: np.ndarray, schema: InputSchema):
    idx = list(schema.predictor_feature_indices)
    if idx and idx == list(range(idx[0], idx[0] + len(idx))):
        X = full[:, idx[0]:idx[0] + len(idx)]               # contiguous predictors: a view
    else:
        X = full[:, idx]
    target = full[:, schema.get_target_feature_index()] if schema.has_target() else \
        np.full(len(full), np.nan)
    return X, target, full


def _native_csv_block(blob, n: int, schema: InputSchema,
                      encodings: CategoricalValueEncodings, F: int) -> Optional[np.ndarray]:
    """The block through the native threaded CSV parser (``oryx_csv_numeric_block``: exact
    fast-path doubles, categorical fields as spans mapped here); None when a line does not
    qualify or a value is unknown (the pandas / general path then decides)."""
    from ... import native
    import ctypes
    data = blob if isinstance(blob, bytes) else blob.encode("utf-8")
    is_num = np.array([1 if schema.is_numeric(fi) else 0 for fi in range(F)], dtype=np.uint8)
    full = np.empty((n, F), dtype=np.float64)
    # spans are written for every non-numeric field (numeric entries stay unused)
    span_off = np.empty((n, F), dtype=np.int64)
    span_len = np.empty((n, F), dtype=np.int32)
    vp = ctypes.c_void_p
    got = native.runtime().oryx_csv_numeric_block(
        data, len(data), F, is_num.ctypes.data_as(vp), full.ctypes.data_as(vp),
        span_off.ctypes.data_as(vp), span_len.ctypes.data_as(vp), n)
    if got != n:
        return None
    num_pred = [fi for fi in range(F) if schema.is_numeric(fi) and not schema.is_target(fi)]
    if num_pred and np.isnan(full).any(axis=0)[num_pred].any():
        return None                                          # empty predictor: general path
    buf = np.frombuffer(data, dtype=np.uint8)
    for fi in range(F):
        if schema.is_numeric(fi):
            continue
        if not schema.is_categorical(fi):
            full[:, fi] = 0.0
            continue
        # the column's spans gathered into fixed-width byte strings (vectorised), one
        # dictionary lookup per distinct value
        off, ln = span_off[:, fi], span_len[:, fi]
        L = int(ln.max()) if n else 0
        if L > 0:
            j = np.arange(L)
            g = buf[np.minimum(off[:, None] + j, len(buf) - 1)]
            g[j >= ln[:, None]] = 0
            vals = np.ascontiguousarray(g).view("S%d" % L).ravel()
        else:
            vals = np.zeros(n, dtype="S1")
        uniq, inv = np.unique(vals, return_inverse=True)
        m = encodings.get_value_encoding_map(fi)
        try:
            codes = np.array([m[u.decode("utf-8")] if u else np.nan for u in uniq.tolist()],
                             dtype=np.float64)
        except (KeyError, UnicodeDecodeError):
            return None                                      # unknown value: general path
        if not schema.is_target(fi) and np.isnan(codes).any():
            return None
        full[:, fi] = codes[inv.reshape(-1)]
    return full


def parse_examples(rows: Sequence[Sequence[str]], schema: InputSchema,
                   encodings: CategoricalValueEncodings, require_target: bool = True
                   ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(predictors float64 [n, P], target float64 [n] (NaN if missing), all-features
    float64 [n, F] with categorical encodings (for scoring))."""
    n = len(rows)
    F = schema.get_num_features()
    full = np.zeros((n, F), dtype=np.float64)
    if n == 0:
        pass
    elif all(len(r) == F for r in rows):
        # one C-level conversion per column block instead of per-cell Python work
        arr = np.array(rows, dtype=str).reshape(n, F)
        for fi in range(F):
            col = arr[:, fi]
            if schema.is_numeric(fi):
                if schema.is_target(fi):
                    empty = col == ""
                    vals = np.where(empty, "nan", col).astype(np.float64)
                    full[:, fi] = vals
                else:
                    full[:, fi] = col.astype(np.float64)
            elif schema.is_categorical(fi):
                m = encodings.get_value_encoding_map(fi)
                uniq, inv = np.unique(col, return_inverse=True)
                if schema.is_target(fi):
                    codes = np.array([m[u] if u != "" else np.nan for u in uniq.tolist()],
                                     dtype=np.float64)
                else:
                    codes = np.array([m[u] for u in uniq.tolist()], dtype=np.float64)
                full[:, fi] = codes[inv.reshape(-1)]
    else:
        for fi in range(F):
            if schema.is_numeric(fi):
                col = [r[fi] for r in rows]
                if schema.is_target(fi):
                    full[:, fi] = [float(v) if v != "" else np.nan for v in col]
                else:
                    full[:, fi] = np.asarray(col, dtype=np.float64)
            elif schema.is_categorical(fi):
                m = encodings.get_value_encoding_map(fi)
                if schema.is_target(fi):
                    full[:, fi] = [m[r[fi]] if r[fi] != "" else np.nan for r in rows]
                else:
                    full[:, fi] = [m[r[fi]] for r in rows]
    pred_idx = schema.predictor_feature_indices
    X = full[:, pred_idx]
    target = full[:, schema.get_target_feature_index()] if schema.has_target() else \
        np.full(n, np.nan)
    if require_target and n and np.isnan(target).any():
        raise ValueError("missing target value")
    return X, target, full


def _to_spec(node: rdf_ops.TrainedNode, data: rdf_ops.BinnedData, schema: InputSchema,
             classification: bool) -> TreeSpecNode:
    spec = TreeSpecNode(node.id, node.count)
    if node.feature < 0:
        if classification:
            spec.class_counts = node.stats
        else:
            w = node.stats[0]
            spec.mean = node.stats[1] / w if w > 0 else 0.0
        return spec
    spec.feature = schema.predictor_to_feature_index(node.feature)
    if node.bin < 0:
        spec.left_categories = [int(e) for e in node.cat_left]
    else:
        spec.threshold = float(data.thresholds[node.feature][node.bin])
    spec.left = _to_spec(node.left, data, schema, classification)
    spec.right = _to_spec(node.right, data, schema, classification)
    spec.default_right = node.right.count > node.left.count
    return spec


def evaluate_forest(forest, encodings, schema: InputSchema, full: np.ndarray,
                    target: np.ndarray, device) -> float:
    """Accuracy (classification) or RMSE (regression) of the forest on the given examples."""
    if len(full) == 0:
        return 0.0 if schema.is_classification() else float("nan")
    C = encodings.get_value_count(schema.get_target_feature_index()) \
        if schema.is_classification() else 0
    flat = rdf_ops.flatten_forest(forest, device, C)
    X = torch.from_numpy(full).to(device)
    vote = rdf_ops.forest_vote(flat, X)                               # [n, C|1]
    tgt = torch.from_numpy(target).to(device)
    if schema.is_classification():
        pred = vote.argmax(1)
        return float((pred == tgt.long()).double().mean())
    return float(torch.sqrt(((vote[:, 0] - tgt) ** 2).mean()))


class RDFUpdate(MLUpdate):
    """Sharded like the ALS and k-means updates: each rank parses and trains on its share of
    the records (native parse, resident history of past part files); categorical encodings
    are merged over the ranks (first appearance, rank order), split thresholds come from a
    sample gathered from every rank, the level histograms are all-reduced, and evaluation
    sums per-rank partial counts."""

    # the interval is saved as several part files when large; FeatureHistory adopts each
    # from the interval's parse (models/features.py)
    split_interval_files = True

    sharded_data = True

    def __init__(self, config):
        super().__init__(config)
        self.num_trees = config.get_int("oryx.rdf.num-trees")
        if self.num_trees < 1:
            raise ValueError("num-trees must be >= 1")
        self.hyper_param_values = [
            hp.from_config(config, "oryx.rdf.hyperparams.max-split-candidates"),
            hp.from_config(config, "oryx.rdf.hyperparams.max-depth"),
            hp.from_config(config, "oryx.rdf.hyperparams.impurity"),
        ]
        self.input_schema = InputSchema(config)
        if not self.input_schema.has_target():
            raise ValueError("RDF needs a target feature")
        from ...utils import config as cfg
        rh = cfg.get_optional_bool(config, "oryx.rdf.resident-history")
        self.resident_history = True if rh is None else bool(rh)
        self.history: Optional[FeatureHistory] = None
        self.phase_seconds: Dict[str, float] = {}
        # the "train" phase broken down (train_forest's timings; accumulates like the above)
        self.train_phases: Dict[str, float] = {}

    def get_hyper_parameter_values(self):
        return self.hyper_param_values

    def warm_up(self, context) -> None:
        """Start-up warm-up (``BatchLayer.warm_up``): a forest of the configured size over a
        few thousand random numeric rows of the schema's width, on this rank's device (the
        binning, histogram, split, route and sort kernels load here).  Local."""
        ctx = self._ctx(context)
        dev = ctx.device
        if dev.type != "cuda":
            return
        schema = self.input_schema
        P = schema.get_num_predictors()
        bins = max(2, int(round(float(self.hyper_param_values[0].get_trial_values(1)[0]))))
        depth = max(1, int(round(float(self.hyper_param_values[1].get_trial_values(1)[0]))))
        imp = str(self.hyper_param_values[2].get_trial_values(1)[0])
        rs = np.random.default_rng(1)
        X = rs.normal(0, 1, (8192, P))
        data = rdf_ops.bin_features(X, [False] * P, [0] * P, bins, dev, seed=1,
                                    threshold_source=X)
        local = dist.DistContext(device=dev)
        if schema.is_classification():
            y = torch.from_numpy((X[:, 0] > 0).astype(np.int64))
            rdf_ops.train_forest(data, y, 2, self.num_trees, depth,
                                 imp if imp in ("gini", "entropy") else "gini", seed=1,
                                 ctx=local)
        else:
            rdf_ops.train_forest(data, torch.from_numpy(X[:, 0].copy()), 0, self.num_trees,
                                 depth, "variance", seed=1, ctx=local)
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

    def _tick(self, name: str, t0: float) -> None:
        self.phase_seconds[name] = self.phase_seconds.get(name, 0.0) + time.perf_counter() - t0

    def _parse(self, lines, ctx) -> FeatureBlock:
        tp = time.perf_counter()
        blk = parse_features(lines, self.input_schema, ctx.device, torch.float64,
                             history=self._history_for(ctx.device))
        self._tick("parse", tp)
        return blk

    def _global_encodings(self, blk: FeatureBlock, ctx) -> CategoricalValueEncodings:
        """Encodings over every rank's records (first appearance, rank order); this rank's
        categorical columns are recoded to them in place."""
        schema = self.input_schema
        cats = [f for f in range(schema.get_num_features()) if schema.is_categorical(f)]
        if not cats:
            return CategoricalValueEncodings({})
        mine = {f: blk.values.get(f, []) for f in cats}
        if self._sharded(ctx):
            allv = [None] * ctx.world_size
            torch.distributed.all_gather_object(allv, mine, group=ctx.control)
        else:
            allv = [mine]
        values: Dict[int, List[str]] = {}
        for f in cats:
            index: Dict[str, int] = {}
            for part in allv:
                for v in part.get(f, []):
                    index.setdefault(v, len(index))
            values[f] = list(index.keys())
            local = mine[f]
            remap = np.array([index[v] for v in local], dtype=np.float64)
            if len(local) and not np.array_equal(remap, np.arange(len(local))):
                col = blk.full[:, f]
                ok = ~torch.isnan(col)
                col[ok] = torch.from_numpy(remap).to(col.device, col.dtype)[col[ok].long()]
        return CategoricalValueEncodings(values)

    def _threshold_sample(self, X: torch.Tensor, ns: int, seed: int, ctx) -> torch.Tensor:
        """The rows split thresholds are computed from: this rank's rows on one rank; with
        several, an equal-rate sample of every rank's rows gathered to all (identical bins
        everywhere, as MLlib's sampled split finding)."""
        if not self._sharded(ctx):
            return X
        from ...parallel import shuffle
        n = int(X.shape[0])
        total = sum(shuffle.all_gather_int(n, ctx))
        rate = min(1.0, ns / max(1, total))
        g = np.random.default_rng((seed * 31 + ctx.rank) & ((1 << 62) - 1))
        pick = np.nonzero(g.random(n) < rate)[0] if rate < 1.0 else np.arange(n)
        local = X[torch.from_numpy(pick).to(X.device)].double().cpu().numpy()
        parts = shuffle.all_gather_var(local.reshape(-1), ctx)
        P = int(X.shape[1])
        return torch.from_numpy(np.concatenate(parts).reshape(-1, P))

    def build_model(self, context, train_data, hyper_parameters, candidate_path):
        max_split_candidates = int(hyper_parameters[0])
        max_depth = int(hyper_parameters[1])
        impurity = str(hyper_parameters[2])
        if max_split_candidates < 2:
            raise ValueError("max-split-candidates must be at least 2")
        if max_depth <= 0:
            raise ValueError("max-depth must be at least 1")
        schema = self.input_schema
        ctx = self._ctx(context)
        sharded = self._sharded(ctx)
        blk = self._parse(train_data, ctx)
        if sharded:
            from ...parallel import shuffle
            n_all = sum(shuffle.all_gather_int(len(blk), ctx))
        else:
            n_all = len(blk)
        if n_all == 0:
            return None
        tp = time.perf_counter()
        encodings = self._global_encodings(blk, ctx)
        X = blk.predictors(schema)
        target = blk.target(schema)
        num_pred = [p for p in range(X.shape[1])
                    if not schema.is_categorical(schema.predictor_to_feature_index(p))]
        if len(blk) and (bool(torch.isnan(target).any()) or
                         (num_pred and bool(torch.isnan(X[:, num_pred]).any()))):
            raise ValueError("missing target or numeric feature value")
        P = schema.get_num_predictors()
        categorical = [schema.is_categorical(schema.predictor_to_feature_index(p))
                       for p in range(P)]
        arities = [encodings.get_value_count(schema.predictor_to_feature_index(p))
                   if categorical[p] else 0 for p in range(P)]
        seed = rng.next_seed()
        ns = max(10000, max_split_candidates * max_split_candidates)
        src = self._threshold_sample(X, ns, seed, ctx)
        # one process: every rank parsed everything and bins a disjoint slice
        sl = slice(None) if sharded else slice(ctx.rank, None, ctx.world_size)
        data = rdf_ops.bin_features(X[sl], categorical, arities, max_split_candidates,
                                    ctx.device, seed=seed, threshold_source=src)
        self._tick("bin", tp)
        t0 = time.perf_counter()
        classification = schema.is_classification()
        C = encodings.get_value_count(schema.get_target_feature_index()) if classification \
            else 0
        tgt = target[sl]
        trained = rdf_ops.train_forest(data, tgt, C, self.num_trees, max_depth, impurity,
                                       seed=seed, ctx=ctx, timings=self.train_phases)
        self._tick("train", t0)
        log.info("RDF %d trees depth %d on %d examples x %d predictors: %.3fs", self.num_trees,
                 max_depth, n_all, P, time.perf_counter() - t0)
        if not ctx.is_main and not sharded:
            return None
        tp = time.perf_counter()
        total = trained.predictor_counts.sum()
        if total <= 0:
            importances = np.zeros(P)
        else:
            importances = trained.predictor_counts / total
        roots = [_to_spec(r, data, schema, classification) for r in trained.roots]
        pmml = rdf_pmml.forest_to_pmml(roots, schema, encodings, importances, max_depth,
                                       max_split_candidates, impurity)
        self._tick("pmml", tp)
        return pmml

    def evaluate(self, context, model, model_parent_path, test_data, train_data):
        rdf_pmml.validate_pmml_vs_schema(model, self.input_schema)
        forest, encodings = rdf_pmml.read(model)
        ctx = self._ctx(context)
        schema = self.input_schema
        blk = parse_features(test_data, schema, ctx.device, torch.float64)
        tp = time.perf_counter()
        full = blk.full
        keep = torch.ones(len(blk), dtype=torch.bool, device=full.device)
        # categorical values -> the model's encodings; a value never seen in training drops
        # its example (the reference scores only examples it can encode)
        for f, vals in blk.values.items():
            m = encodings.get_value_encoding_map(f)
            remap = np.array([m.get(v, -1) for v in vals], dtype=np.float64)
            col = full[:, f]
            ok = ~torch.isnan(col)
            mapped = torch.full_like(col, float("nan"))
            if len(remap):
                mapped[ok] = torch.from_numpy(remap).to(col.device, col.dtype)[col[ok].long()]
            keep &= ~(mapped < 0)
            if not schema.is_target(f):
                keep &= ~torch.isnan(mapped)
            full[:, f] = mapped
        full = full[keep]
        target = full[:, schema.get_target_feature_index()]
        keep_t = ~torch.isnan(target)
        full, target = full[keep_t], target[keep_t]
        classification = schema.is_classification()
        C = encodings.get_value_count(schema.get_target_feature_index()) if classification \
            else 0
        if len(full):
            flat = rdf_ops.flatten_forest(forest, ctx.device, C)
            vote = rdf_ops.forest_vote(flat, full.contiguous())
            if classification:
                num = float((vote.argmax(1) == target.long()).double().sum())
            else:
                num = float(((vote[:, 0] - target) ** 2).sum())
        else:
            num = 0.0
        parts = np.array([num, float(len(full))], dtype=np.float64)
        if self._sharded(ctx):
            from ...parallel import shuffle
            parts = shuffle.all_reduce_np(parts, ctx)
        self._tick("eval", tp)
        if classification:
            ev = float(parts[0] / parts[1]) if parts[1] else 0.0
            log.info("Accuracy: %s", ev)
            return ev
        ev = math.sqrt(parts[0] / parts[1]) if parts[1] else float("nan")
        log.info("RMSE: %s", ev)
        return -ev
