"""ALS batch-layer update: parse -> aggregate -> GPU ALS -> PMML + factor files -> publish.

Equivalent of ``ALSUpdate`` (``[mllib]/als/ALSUpdate.java:78-498``) and its helpers
``Evaluation`` / ``EnqueueFeatureVecsFn`` / ``EnqueueFeatureVecsAndKnownItemsFn``:

* input lines ``user,item[,strength[,timestamp]]`` (or JSON arrays) are parsed natively into
  dictionary codes (collision-free, replacing the reference's int-parse-or-hash + reverse map);
* time decay ``r * factor^days`` and the zero-threshold filter, then time-ordered
  aggregation per (user, item): implicit = sum where an empty strength (delete) resets,
  explicit = last value wins -- done with one stable device sort, no shuffles;
* training is :class:`~oryx_amd.models.als.trainer.ALSTrainer` (fused HIP solve kernel);
* outputs ``X/`` and ``Y/`` as gzip ``part-00000.gz`` JSON lines ``[id,[floats]]`` and PMML
  with extensions ``X``, ``Y``, ``features``, ``lambda``, ``implicit``, [``alpha``],
  ``XIDs``, ``YIDs``;
* evaluation: AUC (implicit; per-user positives vs sampled negatives) or -RMSE, on device;
* publishing: ``UP`` ``["Y",id,vec]`` rows first, then ``["X",id,vec,[known items]]``.
"""

from __future__ import annotations

import gzip
import hashlib
import json
import logging
import math
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ... import ingest
from ...ml import hyperparams as hp
from ...ml.mlupdate import MLUpdate
from ...parallel import dist
from ...utils import config as cfg, ioutils, pmml as pmmlu, rng, text
from . import evaluation
from .trainer import ALSTrainer

__all__ = ["ALSUpdate", "aggregate_scores", "decay_rating", "parse_ratings"]

log = logging.getLogger(__name__)


def decay_rating(rating: float, timestamp: int, now: int, factor: float) -> float:
    if timestamp >= now:
        return rating
    days = (now - timestamp) / 86400000.0
    return rating * math.pow(factor, days)


def aggregate_scores(u: np.ndarray, i: np.ndarray, s: np.ndarray, ts: np.ndarray,
                     implicit: bool) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Time-ordered per-(u,i) aggregation (``ALSUpdate.aggregateScores`` + ``SUM_WITH_NAN``).

    Implicit: sum of the values after the last NaN (delete) in time order; a trailing NaN drops
    the pair.  Explicit: the last value; NaN drops the pair.
    """
    if len(u) == 0:
        return u, i, s
    n_i = int(i.max()) + 1
    key = u.astype(np.int64) * n_i + i.astype(np.int64)
    order = np.lexsort((np.arange(len(key)), ts, key))  # by key, then time, then arrival
    key_s, s_s = key[order], s[order]
    starts = np.flatnonzero(np.r_[True, key_s[1:] != key_s[:-1]])
    ends = np.r_[starts[1:], len(key_s)]
    if implicit:
        isnan = np.isnan(s_s)
        # index of the last NaN at or before each position within its group
        idx = np.where(isnan, np.arange(len(s_s)), -1)
        last_nan = np.maximum.accumulate(idx)
        grp_last_nan = last_nan[ends - 1]
        grp_start = np.maximum(starts, grp_last_nan + 1)
        vals = np.where(isnan, 0.0, s_s)
        csum = np.r_[0.0, np.cumsum(vals)]
        out = csum[ends] - csum[grp_start]
        # trailing delete -> NaN (dropped); a group that is all deletes -> NaN
        out = np.where(grp_last_nan == ends - 1, np.nan, out)
    else:
        out = s_s[ends - 1]
    keep = ~np.isnan(out)
    gk = key_s[starts][keep]
    return (gk // n_i).astype(np.int64), (gk % n_i).astype(np.int64), out[keep]


def parse_ratings(lines: Sequence[str], users: ingest.IdDict, items: ingest.IdDict,
                  decay_factor: float = 1.0, zero_threshold: float = 0.0,
                  now_ms: Optional[int] = None):
    now = int(time.time() * 1000) if now_ms is None else now_ms
    u, i, s, ts = ingest.parse_ratings(lines, users, items, default_ts=now)
    if decay_factor < 1.0:
        days = np.maximum(0, now - ts) / 86400000.0
        s = np.where(ts >= now, s, s * np.power(decay_factor, days))
    if zero_threshold > 0.0:
        keep = s > zero_threshold
        u, i, s, ts = u[keep], i[keep], s[keep], ts[keep]
    return u, i, s, ts


def _timestamps(lines: Sequence[str]) -> np.ndarray:
    d1, d2 = ingest.IdDict(), ingest.IdDict()
    _, _, _, ts = ingest.parse_ratings(lines, d1, d2, default_ts=0)
    return ts


def write_features(path: str, ids: List[str], mat: np.ndarray) -> None:
    """``X/`` or ``Y/`` directory with one gzip part of ``[id,[floats]]`` JSON lines."""
    os.makedirs(path, exist_ok=True)
    rows = ingest.format_float_rows(mat)
    with gzip.open(os.path.join(path, "part-00000.gz"), "wt", encoding="utf-8",
                   compresslevel=1) as f:
        for id_, row in zip(ids, rows):
            f.write("[%s,%s]\n" % (json.dumps(id_), row))


def read_features(path: str) -> Tuple[List[str], np.ndarray]:
    ids, vecs = [], []
    for part in sorted(ioutils.list_files(path, "part-*")):
        with ioutils.open_text_maybe_gz(part) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                rec = json.loads(line)
                ids.append(str(rec[0]))
                vecs.append(rec[1])
    mat = np.asarray(vecs, dtype=np.float32) if vecs else np.zeros((0, 0), np.float32)
    return ids, mat


def _fingerprint(u, i, s, *params) -> str:
    """Identity of one training run: the aggregated ratings plus every setting that shapes
    the factors (a checkpoint is only resumed by the same run)."""
    h = hashlib.blake2b(digest_size=20)
    for a in (u, i, s):
        h.update(np.ascontiguousarray(a).tobytes())
    h.update(repr(params).encode())
    return h.hexdigest()


def _latest_model_dir(model_dir: str) -> Optional[str]:
    """The newest ``model-dir/<timestamp>/`` that has both X/ and Y/ factor directories."""
    try:
        names = [n for n in os.listdir(model_dir) if n.isdigit()]
    except OSError:
        return None
    for n in sorted(names, key=int, reverse=True):
        p = os.path.join(model_dir, n)
        if os.path.isdir(os.path.join(p, "X")) and os.path.isdir(os.path.join(p, "Y")):
            return p
    return None


def _warm_start_factors(model_dir: str, features: int, x_ids: List[str], y_ids: List[str]):
    """Previous generation's factor rows for the IDs of this run (NaN rows where absent);
    (None, None) when there is no previous model of the same rank."""
    prev = _latest_model_dir(model_dir)
    if prev is None:
        return None, None
    out = []
    for sub, ids in (("X", x_ids), ("Y", y_ids)):
        old_ids, mat = read_features(os.path.join(prev, sub))
        if mat.ndim != 2 or mat.shape[1] != features:
            log.info("Previous model %s has rank %s, not warm-starting", prev,
                     mat.shape[1] if mat.ndim == 2 else None)
            return None, None
        index = {k: j for j, k in enumerate(old_ids)}
        init = np.full((len(ids), features), np.nan, dtype=np.float32)
        rows = [(a, index[k]) for a, k in enumerate(ids) if k in index]
        if rows:
            dst, src = zip(*rows)
            init[list(dst)] = mat[list(src)]
        out.append(torch.from_numpy(init))
    log.info("Warm-starting ALS from %s", prev)
    return out[0], out[1]


class ALSUpdate(MLUpdate):
    def __init__(self, config):
        super().__init__(config)
        self.iterations = config.get_int("oryx.als.iterations")
        self.implicit = config.get_bool("oryx.als.implicit")
        self.hyper_param_values = [
            hp.from_config(config, "oryx.als.hyperparams.features"),
            hp.from_config(config, "oryx.als.hyperparams.lambda"),
            hp.from_config(config, "oryx.als.hyperparams.alpha"),
        ]
        self.no_known_items = config.get_bool("oryx.als.no-known-items")
        self.decay_factor = config.get_double("oryx.als.decay.factor")
        self.decay_zero_threshold = config.get_double("oryx.als.decay.zero-threshold")
        self.precision = cfg.get_optional_string(config, "oryx.gpu.dtype") or "fp32"
        self.checkpoint_interval = cfg.get_optional_int(config, "oryx.als.checkpoint-interval") \
            or 0
        self.warm_start = bool(cfg.get_optional_bool(config, "oryx.als.warm-start"))
        self.current_model_dir: Optional[str] = None
        if self.iterations <= 0:
            raise ValueError("iterations must be > 0")
        if not (0.0 < self.decay_factor <= 1.0) or self.decay_zero_threshold < 0.0:
            raise ValueError("bad decay settings")
        self._cache: Dict[str, dict] = {}
        self._timings: Dict[str, dict] = {}

    def get_hyper_parameter_values(self):
        return self.hyper_param_values

    # ---------------------------------------------------------------- build
    def _ctx(self, context) -> dist.DistContext:
        if isinstance(context, dist.DistContext):
            return context
        c = getattr(context, "dist", None)
        return c if c is not None else dist.get_context()

    def build_model(self, context, train_data, hyper_parameters, candidate_path):
        features = int(hyper_parameters[0])
        lam = float(hyper_parameters[1])
        alpha = float(hyper_parameters[2])
        if features <= 0 or lam < 0.0 or alpha <= 0.0:
            raise ValueError("bad hyperparameters %s" % (hyper_parameters,))
        users, items = ingest.IdDict(), ingest.IdDict()
        u, i, s, ts = parse_ratings(train_data, users, items, self.decay_factor,
                                    self.decay_zero_threshold)
        u, i, s = aggregate_scores(u, i, s, ts, self.implicit)
        if len(u) == 0:
            log.info("No ratings after aggregation")
            return None
        user_ids, item_ids = users.keys(), items.keys()
        # only IDs that survived aggregation get factors (MLlib only emits rated rows)
        used_u = np.unique(u)
        used_i = np.unique(i)
        remap_u = np.full(len(user_ids), -1, dtype=np.int64)
        remap_u[used_u] = np.arange(len(used_u))
        remap_i = np.full(len(item_ids), -1, dtype=np.int64)
        remap_i[used_i] = np.arange(len(used_i))
        ctx = self._ctx(context)
        seed = rng.next_seed()
        trainer = ALSTrainer(features, lam, alpha, self.implicit, ctx=ctx, seed=seed,
                             precision=self.precision)
        t0 = time.perf_counter()
        # every rank holds the same aggregated triples; each contributes a disjoint slice
        part = slice(ctx.rank, None, ctx.world_size)
        trainer.prepare(torch.from_numpy(remap_u[u][part]), torch.from_numpy(remap_i[i][part]),
                        torch.from_numpy(s[part].astype(np.float32)), len(used_u), len(used_i))
        x_ids = [user_ids[j] for j in used_u]
        y_ids = [item_ids[j] for j in used_i]
        ckpt_dir, fingerprint = None, ""
        if self.checkpoint_interval > 0 and self.current_model_dir:
            fingerprint = _fingerprint(u, i, s, features, lam, alpha, self.implicit,
                                       self.iterations, seed, ctx.world_size)
            ckpt_dir = os.path.join(self.current_model_dir, ".checkpoint",
                                    "als-" + fingerprint[:16])
        x_init = y_init = None
        if self.warm_start and self.current_model_dir:
            x_init, y_init = _warm_start_factors(self.current_model_dir, features, x_ids, y_ids)
        f = trainer.train(self.iterations, checkpoint_dir=ckpt_dir,
                          checkpoint_interval=self.checkpoint_interval, fingerprint=fingerprint,
                          x_init=x_init, y_init=y_init)
        X = f.X.cpu().numpy()
        Y = f.Y.cpu().numpy()
        log.info("ALS %d ratings, %d users, %d items, rank %d: %.3fs", len(u), len(used_u),
                 len(used_i), features, time.perf_counter() - t0)
        if not ctx.is_main:
            return None
        write_features(os.path.join(candidate_path, "X"), x_ids, X)
        write_features(os.path.join(candidate_path, "Y"), y_ids, Y)
        pmml = pmmlu.build_skeleton_pmml()
        pmml.add_extension("X", "X/")
        pmml.add_extension("Y", "Y/")
        pmml.add_extension("features", features)
        pmml.add_extension("lambda", lam)
        pmml.add_extension("implicit", self.implicit)
        if self.implicit:
            pmml.add_extension("alpha", alpha)
        pmml.add_extension_content("XIDs", x_ids)
        pmml.add_extension_content("YIDs", y_ids)
        self._cache[candidate_path] = {"x_ids": x_ids, "y_ids": y_ids, "X": X, "Y": Y}
        its = trainer.timings.get("iteration_ms", [])
        self._timings[candidate_path] = {
            "ratings": int(len(u)), "users": len(used_u), "items": len(used_i),
            "prepare_s": trainer.timings.get("prepare_s"), "iteration_ms": its,
            "resumed_from_iteration": getattr(trainer, "resumed_from", 0),
            "ratings_per_s": (len(u) * 1e3 / (sum(its) / len(its))) if its else None}
        return pmml

    def build_timings(self, candidate_path: str) -> dict:
        return self._timings.pop(candidate_path, {})

    # ---------------------------------------------------------------- evaluate
    def _load(self, model_parent_path: str, pmml) -> dict:
        cached = self._cache.pop(model_parent_path, None)
        if cached is not None:
            return cached
        x_ids, X = read_features(os.path.join(model_parent_path,
                                              pmml.get_extension_value("X")))
        y_ids, Y = read_features(os.path.join(model_parent_path,
                                              pmml.get_extension_value("Y")))
        return {"x_ids": x_ids, "y_ids": y_ids, "X": X, "Y": Y}

    def evaluate(self, context, model, model_parent_path, test_data, train_data):
        f = self._load(model_parent_path, model)
        users, items = ingest.IdDict(), ingest.IdDict()
        u, i, s, ts = parse_ratings(test_data, users, items, self.decay_factor,
                                    self.decay_zero_threshold)
        u, i, s = aggregate_scores(u, i, s, ts, self.implicit)
        xmap = {k: n for n, k in enumerate(f["x_ids"])}
        ymap = {k: n for n, k in enumerate(f["y_ids"])}
        ucodes = np.array([xmap.get(k, -1) for k in users.keys()], dtype=np.int64)
        icodes = np.array([ymap.get(k, -1) for k in items.keys()], dtype=np.int64)
        mu, mi = (ucodes[u] if len(u) else u), (icodes[i] if len(i) else i)
        device = self._ctx(context).device
        X = torch.from_numpy(f["X"]).to(device)
        Y = torch.from_numpy(f["Y"]).to(device)
        if self.implicit:
            # AUC over test positives; items universe = distinct test items (known to the model)
            auc = evaluation.area_under_curve(X, Y, mu, mi, device=device)
            log.info("AUC: %s", auc)
            return auc
        rmse = evaluation.rmse(X, Y, mu, mi, s, device=device)
        log.info("RMSE: %s", rmse)
        return -rmse

    # ---------------------------------------------------------------- publish
    def can_publish_additional_model_data(self) -> bool:
        return True

    def publish_additional_model_data(self, context, pmml, new_data, past_data,
                                      model_parent_path, model_update_topic):
        all_data = list(new_data) + list(past_data or [])
        x_ids, X = read_features(os.path.join(model_parent_path, pmml.get_extension_value("X")))
        y_ids, Y = read_features(os.path.join(model_parent_path, pmml.get_extension_value("Y")))
        log.info("Sending item / Y data as model updates")
        y_rows = ingest.format_float_rows(Y) if len(y_ids) else []
        model_update_topic.send_many(("UP", '["Y",%s,%s]' % (json.dumps(i), r))
                                     for i, r in zip(y_ids, y_rows))
        log.info("Sending user / X data as model updates")
        x_rows = ingest.format_float_rows(X) if len(x_ids) else []
        if self.no_known_items:
            model_update_topic.send_many(("UP", '["X",%s,%s]' % (json.dumps(u), r))
                                         for u, r in zip(x_ids, x_rows))
        else:
            known = known_items(all_data)
            msgs = []
            for uid, r in zip(x_ids, x_rows):
                ks = known.get(uid)
                if ks is None:
                    continue  # join: users without any event are not sent
                msgs.append(("UP", '["X",%s,%s,%s]' % (json.dumps(uid), r,
                                                        json.dumps(sorted(ks)))))
            model_update_topic.send_many(msgs)

    # ---------------------------------------------------------------- split
    def split_new_data_to_train_test(self, new_data):
        ts = _timestamps(new_data)
        if len(ts) == 0:
            return list(new_data), []
        lo, hi = int(ts.min()), int(ts.max())
        log.info("New data timestamp range: %d - %d", lo, hi)
        boundary = int(hi - self.get_test_fraction() * (hi - lo))
        log.info("Splitting at timestamp %d", boundary)
        # lines that fail to parse are dropped by the parser; keep alignment via per-line parse
        train, test = [], []
        if len(ts) == len(new_data):
            for line, t in zip(new_data, ts.tolist()):
                (train if t < boundary else test).append(line)
        else:
            for line in new_data:
                t = _timestamps([line])
                if len(t) == 0:
                    continue
                (train if int(t[0]) < boundary else test).append(line)
        return train, test


def known_items(lines: Sequence[str]) -> Dict[str, set]:
    """User -> known items from all data in time order; an empty strength deletes."""
    users, items = ingest.IdDict(), ingest.IdDict()
    u, i, s, ts = ingest.parse_ratings(lines, users, items, default_ts=0)
    if len(u) == 0:
        return {}
    n_i = int(i.max()) + 1
    key = u * n_i + i
    order = np.lexsort((np.arange(len(key)), ts, key))
    key_s, s_s = key[order], s[order]
    last = np.r_[key_s[1:] != key_s[:-1], True]
    keep = last & ~np.isnan(s_s)
    kk = key_s[keep]
    uu, ii = kk // n_i, kk % n_i
    uk, ik = users.keys(), items.keys()
    # every user with any event is present (possibly with an empty set), as in the
    # reference's groupByKey + join
    out: Dict[str, set] = {uk[a]: set() for a in np.unique(u).tolist()}
    for a, b in zip(uu.tolist(), ii.tolist()):
        out.setdefault(uk[a], set()).add(ik[b])
    return out
