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

Sharded (several ranks, :mod:`oryx_amd.layers.batch` sharded generations): see
:mod:`.sharded` -- each rank parses its share (with its own resident history), IDs get
global codes from native distributed dictionaries, events are routed once to their user's
owner for the time-ordered aggregation (the reference's ``reduceByKey`` shuffle,
``[mllib]/als/ALSUpdate.java:332-352``), dense ids follow the trainer's row ownership so
factors, ID strings and known items stay on their owner, and every rank writes and publishes
its own rows.  The test split boundary uses the global timestamp range.
"""

from __future__ import annotations

import gzip
import hashlib
import json
import logging
import math
import os
import struct
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ... import ingest, native
from ...textlines import TextLines, concat_lines
from ...ml import hyperparams as hp
from ...ml.mlupdate import MLUpdate
from ...parallel import dist, shuffle
from ...ops import textfmt
from ...utils import config as cfg, ioutils, pmml as pmmlu, rng, text
from . import evaluation
from .trainer import ALS_INIT_SEED, ALSTrainer

from .history import RatingsHistory
from . import sharded

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
    # one native sort + group scan (csrc/runtime/oryx_ingest.cpp)
    u = np.ascontiguousarray(u, dtype=np.int64)
    i = np.ascontiguousarray(i, dtype=np.int64)
    s = np.ascontiguousarray(s, dtype=np.float64)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    ou, oi = np.empty(len(u), np.int64), np.empty(len(u), np.int64)
    os_ = np.empty(len(u), np.float64)
    m = native.runtime().oryx_aggregate_scores(
        u.ctypes.data, i.ctypes.data, s.ctypes.data, ts.ctypes.data, len(u),
        int(bool(implicit)), ou.ctypes.data, oi.ctypes.data, os_.ctypes.data)
    return ou[:m], oi[:m], os_[:m]


def aggregate_scores_reference(u: np.ndarray, i: np.ndarray, s: np.ndarray, ts: np.ndarray,
                               implicit: bool) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """numpy model of :func:`aggregate_scores` (tests compare the native and device paths
    with it)."""
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


def aggregate_scores_device(u: np.ndarray, i: np.ndarray, s: np.ndarray, ts: np.ndarray,
                            implicit: bool, device, to_host: bool = True):
    """:func:`aggregate_scores` on the device -- same results.  Events are ordered by
    (user, item) then time then arrival: with ONE stable radix sort of a composite
    ``key << tbits | (ts - min ts)`` key when both fit in 63 bits (an interval's or a few
    months' history), else two stable sorts (time, then key).  Segmented scans do the rest.
    ``to_host=False`` leaves (user, item, value) on the device (int64, int64, fp64)."""
    dev = torch.device(device)
    if len(u) == 0:
        if to_host:
            return tuple(x.cpu().numpy() if isinstance(x, torch.Tensor) else x
                         for x in (u, i, s))
        e = torch.zeros(0, dtype=torch.int64, device=dev)
        return e, e, torch.zeros(0, dtype=torch.float64, device=dev)
    if isinstance(u, torch.Tensor):
        # already on the device (the sharded path's routed events)
        ud, idv = u.to(dev, torch.int32), i.to(dev, torch.int32)
        tt, vv = ts.to(dev, torch.int64), s.to(dev, torch.float64)
    else:
        # dictionary codes travel as int32 (half the bytes of the host's int64)
        ud = torch.from_numpy(np.ascontiguousarray(u, dtype=np.int32)).to(dev)
        idv = torch.from_numpy(np.ascontiguousarray(i, dtype=np.int32)).to(dev)
        tt = torch.from_numpy(np.ascontiguousarray(ts, dtype=np.int64)).to(dev)
        vv = torch.from_numpy(np.ascontiguousarray(s, dtype=np.float64)).to(dev)
    ext = torch.stack([ud.max().long(), idv.max().long(), tt.min(), tt.max()]).cpu().tolist()
    n_u, n_i = int(ext[0]) + 1, int(ext[1]) + 1
    key = ud.long() * n_i + idv.long()
    del ud, idv
    kbits = max(1, (n_u * n_i - 1).bit_length())
    tbits = max(1, int(ext[3] - ext[2]).bit_length())
    if kbits + tbits <= 63:
        comp = (key << tbits) | (tt - ext[2])
        order = torch.sort(comp, stable=True).indices
        del comp
    else:
        # arrival order breaks time ties: stable sort by time, then stable sort by key
        o1 = torch.sort(tt, stable=True).indices
        o2 = torch.sort(key[o1], stable=True).indices
        order = o1[o2]
    del tt
    key_s, s_s = key[order], vv[order]
    del key, vv, order
    n = key_s.numel()
    first = torch.ones(n, dtype=torch.bool, device=dev)
    first[1:] = key_s[1:] != key_s[:-1]
    starts = torch.nonzero(first, as_tuple=False).flatten()
    ends = torch.cat([starts[1:], torch.tensor([n], device=dev)])
    if implicit:
        isnan = torch.isnan(s_s)
        idx = torch.where(isnan, torch.arange(n, device=dev), torch.full((n,), -1, device=dev))
        last_nan = torch.cummax(idx, 0).values
        grp_last_nan = last_nan[ends - 1]
        grp_start = torch.maximum(starts, grp_last_nan + 1)
        vals = torch.where(isnan, torch.zeros_like(s_s), s_s)
        csum = torch.cat([torch.zeros(1, dtype=vals.dtype, device=dev), torch.cumsum(vals, 0)])
        out = csum[ends] - csum[grp_start.clamp_max(n)]
        out = torch.where(grp_last_nan == ends - 1, torch.full_like(out, float("nan")), out)
    else:
        out = s_s[ends - 1]
    keep = ~torch.isnan(out)
    gk = key_s[starts][keep]
    gu = torch.div(gk, n_i, rounding_mode="floor")
    gi = gk - gu * n_i
    if not to_host:
        return gu, gi, out[keep]
    return gu.cpu().numpy(), gi.cpu().numpy(), out[keep].cpu().numpy()


_NO_TS = -(1 << 62)     # parse marker of a line without a timestamp


def parse_ratings(lines: Sequence[str], users: ingest.IdDict, items: ingest.IdDict,
                  decay_factor: float = 1.0, zero_threshold: float = 0.0,
                  now_ms: Optional[int] = None, raw_out: Optional[list] = None,
                  history: Optional[RatingsHistory] = None, device_out: bool = False):
    """Parse + decay + zero-threshold.  ``raw_out`` (a list) receives the undecayed parse
    with lines lacking a timestamp at 0 -- what :func:`known_items_json_parsed` needs -- so
    the publish step can skip a second parse of the same data.  ``history``: reuse the parse
    of past part files seen in earlier generations (:mod:`.history`; same results).
    ``device_out`` (with a GPU history, no time decay): the columns stay device tensors."""
    now = int(time.time() * 1000) if now_ms is None else now_ms
    if device_out and history is not None and history.device.type == "cuda" and \
            decay_factor >= 1.0:
        # (decay keeps the host path: np.power is the reference's arithmetic)
        u, i, s, ts0 = history.parse_ratings(lines, users, items, default_ts=_NO_TS,
                                             device_out=True)
        missing = ts0 == _NO_TS
        if raw_out is not None:
            raw_out.extend([u, i, s, torch.where(missing, torch.zeros_like(ts0), ts0)])
        ts = torch.where(missing, torch.full_like(ts0, now), ts0)
        if zero_threshold > 0.0:
            keep = s > zero_threshold
            u, i, s, ts = u[keep], i[keep], s[keep], ts[keep]
        return u, i, s, ts
    parse = history.parse_ratings if history is not None else ingest.parse_ratings
    if raw_out is not None:
        u, i, s, ts0 = parse(lines, users, items, default_ts=_NO_TS)
        missing = ts0 == _NO_TS
        raw_out.extend([u, i, s, np.where(missing, 0, ts0)])
        ts = np.where(missing, now, ts0)
    else:
        u, i, s, ts = parse(lines, users, items, default_ts=now)
    if decay_factor < 1.0:
        days = np.maximum(0, now - ts) / 86400000.0
        s = np.where(ts >= now, s, s * np.power(decay_factor, days))
    if zero_threshold > 0.0:
        keep = s > zero_threshold
        u, i, s, ts = u[keep], i[keep], s[keep], ts[keep]
    return u, i, s, ts


def _timestamps(lines: Sequence[str]) -> np.ndarray:
    return ingest.parse_timestamps(lines, default_ts=0)


def _blob_keys(blob_ends) -> List[str]:
    """The keys of a (blob, ends) pair as strings."""
    blob, ends = blob_ends
    b = bytes(blob)
    out, at = [], 0
    for e in np.asarray(ends).tolist():
        out.append(b[at:e].decode("utf-8"))
        at = e
    return out


def write_features(path: str, ids, mat, part: int = 0) -> None:
    """``X/`` or ``Y/`` directory with gzip part ``part`` of ``[id,[floats]]`` JSON lines (the
    reference's Spark text output with the gzip codec); ``ids`` a list of strings or a key
    (blob, ends) pair; ``mat`` is a float matrix or its pre-formatted
    :class:`~oryx_amd.ops.textfmt.RowText`.  Lines are assembled and compressed natively
    (multi-member gzip, one member per slice, threads)."""
    os.makedirs(path, exist_ok=True)
    _write_features_to(os.path.join(path, "part-%05d.gz" % part), ids, mat)


def _write_features_to(target: str, ids, mat) -> None:
    rows = mat if isinstance(mat, textfmt.RowText) else textfmt.format_rows(mat)
    block = ingest.assemble_row_messages("", ids if isinstance(ids, tuple) else list(ids), rows)
    ingest.write_gzip(target, block.buf, level=1)


class _Sender:
    """One ``send_block`` on a helper thread (the native append releases the GIL)."""

    def __init__(self, topic, block):
        import threading
        self.error: Optional[BaseException] = None

        def run():
            try:
                topic.send_block("UP", block)
            except BaseException as e:   # noqa: BLE001 -- re-raised by join
                self.error = e
        self._t = threading.Thread(target=run, name="oryx-als-send-y", daemon=True)
        self._t.start()

    def join(self, raise_error: bool = True) -> None:
        self._t.join()
        if raise_error and self.error is not None:
            err, self.error = self.error, None
            raise err


class _FactorFilesWriter:
    """The ``X/`` and ``Y/`` part files written on a background thread while the generation
    goes on (publishing the MODEL and the UP rows, which read nothing from them).  The part
    files are created -- and held open -- before the thread starts and written through their
    descriptors (``/proc/self/fd``), so promoting the candidate directory (a rename) under the
    writer moves them along; :meth:`join` waits and re-raises.  Reference: the model's X/ Y/
    are saved before the updates are published (``ALSUpdate.java:194-230``); here the bytes
    land in the same files, overlapped with the publish."""

    def __init__(self, jobs):
        import threading
        self._fds = []
        targets = []
        for path, ids, rows in jobs:
            os.makedirs(path, exist_ok=True)
            fd = os.open(os.path.join(path, "part-00000.gz"),
                         os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            self._fds.append(fd)
            targets.append(("/proc/self/fd/%d" % fd, ids, rows))
        self.error: Optional[BaseException] = None
        self.seconds = 0.0

        def run():
            t0 = time.perf_counter()
            try:
                for target, ids, rows in targets:
                    _write_features_to(target, ids, rows)
            except BaseException as e:   # noqa: BLE001 -- re-raised by join
                self.error = e
            finally:
                self.seconds = time.perf_counter() - t0
        self._t = threading.Thread(target=run, name="oryx-als-factor-files", daemon=True)
        self._t.start()

    def join(self) -> None:
        self._t.join()
        for fd in self._fds:
            os.close(fd)
        self._fds = []
        if self.error is not None:
            err, self.error = self.error, None
            raise err


_BACKGROUND_FACTOR_FILES = os.environ.get("ORYX_ALS_BACKGROUND_FILES", "1") != "0" and \
    os.path.isdir("/proc/self/fd")


def read_features(path: str) -> Tuple[List[str], np.ndarray]:
    """The ``X/`` / ``Y/`` factor parts back as (ids, fp32 matrix): each part decompressed
    whole and parsed natively (threaded), with a per-line JSON fallback for a part that is not
    in the plain ``[id,[floats]]`` form."""
    ids: List[str] = []
    mats = []
    for part in sorted(ioutils.list_files(path, "part-*")):
        with open(part, "rb") as f:
            raw = f.read()
        if part.endswith(".gz"):
            raw = ingest.read_gzip(raw)
        head = bytes(raw[:1 << 16]).lstrip()
        while b"\n" not in head and len(head) < len(raw):   # a first line past 64 KB
            head = bytes(raw[:len(head) * 4 + (1 << 16)]).lstrip()
        first = head.split(b"\n", 1)[0]
        if not first.strip():
            continue
        got = None
        try:
            k = len(json.loads(first)[1])
            got = ingest.parse_feature_lines(raw, k)
        except (ValueError, IndexError, TypeError):
            got = None
        if got is None:
            p_ids, vecs = [], []
            for line in bytes(raw).decode("utf-8").splitlines():
                line = line.strip()
                if line:
                    rec = json.loads(line)
                    p_ids.append(str(rec[0]))
                    vecs.append(rec[1])
            got = (p_ids, np.asarray(vecs, dtype=np.float32))
        ids.extend(got[0])
        mats.append(got[1])
    if not ids:
        return ids, np.zeros((0, 0), np.float32)
    return ids, mats[0] if len(mats) == 1 else np.concatenate(mats)


def _i64(c: int) -> int:
    return c - (1 << 64) if c >= (1 << 63) else c


_FP_MULS = [_i64(c) for c in (0x9E3779B97F4A7C15, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9,
                              0x27D4EB2F165667C5, 0xFF51AFD7ED558CCD)]


def _fingerprint(u, i, s, *params) -> str:
    """Identity of one training run: the aggregated ratings plus every setting that shapes
    the factors (a checkpoint is only resumed by the same run).  The triples are mixed
    where they live (the device after a GPU aggregation: no 0.5 s host copy and hash of 25M
    triples): every (user, item, score bits, position) goes through a multiply-xorshift
    mix, and two wrapping 64-bit sums of the mixes (one position-weighted) plus the count
    and the settings are hashed."""
    t = [a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
         for a in (u, i, s)]
    dev = t[0].device
    n = t[0].numel()
    c1, c2, c3, c4, c5 = _FP_MULS
    k = torch.arange(n, device=dev, dtype=torch.int64)
    x = t[0].to(torch.int64) * c1 + t[1].to(dev, torch.int64) * c2 + \
        t[2].to(dev, torch.float64).view(torch.int64) * c3 + k * c4
    x = x ^ (x >> 29)
    x = x * c5
    x = x ^ (x >> 32)
    a, b = int(x.sum()), int((x * (k | 1)).sum())
    h = hashlib.blake2b(digest_size=20)
    h.update(struct.pack("<qqq", n, a, b))
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
    sharded_data = True

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
        # the build's undecayed parse of the complete data set, reused by the publish step
        self._raw_parse: Optional[dict] = None
        self._timings: Dict[str, dict] = {}
        self._writers: List[_FactorFilesWriter] = []     # factor files written in background
        # resident parse of past part files across generations (oryx.als.resident-history,
        # default on; models/als/history.py)
        rh = cfg.get_optional_bool(config, "oryx.als.resident-history")
        self.resident_history = True if rh is None else bool(rh)
        self.history: Optional[RatingsHistory] = None
        # cumulative seconds per phase of build / publish (bench_batch.py reads them)
        self.phase_seconds: Dict[str, float] = {}
        # the "train" phase broken down (ALSTrainer.train's laps; accumulates like the above)
        self.train_phases: Dict[str, float] = {}

    def get_hyper_parameter_values(self):
        return self.hyper_param_values

    def warm_up(self, context) -> None:
        """Start-up warm-up (``BatchLayer.warm_up``): a tiny build on this rank's device with
        every configured rank and the configured precision -- the device aggregation, the
        trainer's solve / Gramian kernels, the keyed init and the row formatter load their
        code objects here, not inside the first generation.  Local (no collectives)."""
        ctx = self._ctx(context)
        dev = ctx.device
        if dev.type != "cuda":
            return
        local = dist.DistContext(device=dev)
        feats = sorted({int(round(float(v))) for v in
                        self.hyper_param_values[0].get_trial_values(max(1, self.candidates))})
        rs = np.random.default_rng(1)
        nu, ni, nnz = 512, 256, 8192
        u = rs.integers(0, nu, nnz)
        i = rs.integers(0, ni, nnz)
        ts = rs.integers(0, 1000, nnz)
        ud, idv, sd = aggregate_scores_device(u, i, np.ones(nnz), ts, self.implicit, dev,
                                              to_host=False)
        keys_u = np.arange(nu, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        keys_i = np.arange(ni, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        for k in feats:
            tr = ALSTrainer(k, 0.1, 1.0, self.implicit, ctx=local, seed=1,
                            precision=self.precision, init_seed=ALS_INIT_SEED)
            tr.prepare(ud, idv, sd.to(torch.float32), nu, ni)
            f = tr.train(2, x_keys=keys_u, y_keys=keys_i)
            textfmt.format_rows(f.X)
        torch.cuda.synchronize(dev)

    def _history_for(self, device) -> Optional[RatingsHistory]:
        if not self.resident_history:
            return None
        dev = torch.device(device) if device is not None else torch.device("cpu")
        if self.history is None or self.history.device != dev:
            self.history = RatingsHistory(dev)
        return self.history

    def _raw_parse_slot(self, lines, users, items) -> Optional[list]:
        """A list for parse_ratings' raw output of the training lines, kept for the publish
        step's known items: with test fraction 0 MLUpdate trains on new + past data, exactly
        what that step joins known items from; with a test split the training lines lack only
        the held-out test lines, which the publish step then parses alone and appends
        (``_known_items_parse``)."""
        if not lines:
            self._raw_parse = None
            return None
        out: list = []
        self._raw_parse = {"n": len(lines), "first": lines[0], "last": lines[-1],
                           "users": users, "items": items, "arrays": out}
        return out

    def _known_items_parse(self, all_data):
        """(users, items, u, i, s, ts) of every event of the generation for the known items:
        the build's memoised parse when it covered the whole data set; with a test split, the
        memoised parse of the training lines plus a parse of just the held-out test lines
        into the same dictionaries (instead of re-parsing all of the new data); None when
        neither applies."""
        parsed = self._raw_parse_for(all_data)
        if parsed is not None:
            return parsed
        m = self._raw_parse
        test = getattr(self, "_split_test", None)
        if m is None or len(m["arrays"]) != 4 or test is None or not len(test) or \
                m["n"] + len(test) != len(all_data):
            return None
        users, items = m["users"], m["items"]
        tu, ti, tsv, tts = ingest.parse_ratings(test, users, items, default_ts=_NO_TS)
        tts = np.where(tts == _NO_TS, 0, tts)
        u, i, sv, ts = m["arrays"]
        if isinstance(u, torch.Tensor):
            # the training parse stayed on the device (parse_ratings device_out)
            dv = u.device
            up = lambda a, like: torch.from_numpy(np.ascontiguousarray(a)).to(dv, like.dtype)
            return (users, items, torch.cat([u, up(tu, u)]), torch.cat([i, up(ti, i)]),
                    torch.cat([sv, up(tsv, sv)]), torch.cat([ts, up(tts, ts)]))
        return (users, items, np.concatenate([u, tu]), np.concatenate([i, ti]),
                np.concatenate([sv, tsv]), np.concatenate([ts, tts]))

    def _raw_parse_for(self, lines):
        """(users, items, u, i, s, ts) of the memoised parse when it is of ``lines``."""
        m = self._raw_parse
        if m is None or not lines or len(m["arrays"]) != 4 or m["n"] != len(lines) or \
                m["first"] != lines[0] or m["last"] != lines[-1]:
            return None
        return (m["users"], m["items"]) + tuple(m["arrays"])

    # ---------------------------------------------------------------- build
    def _ctx(self, context) -> dist.DistContext:
        if isinstance(context, dist.DistContext):
            return context
        c = getattr(context, "dist", None)
        return c if c is not None else dist.get_context()

    def _sharded(self, context) -> bool:
        return self._ctx(context).is_distributed and self.dist_ctx is not None and \
            self.dist_ctx.is_distributed

    def build_model(self, context, train_data, hyper_parameters, candidate_path):
        features = int(hyper_parameters[0])
        lam = float(hyper_parameters[1])
        alpha = float(hyper_parameters[2])
        if features <= 0 or lam < 0.0 or alpha <= 0.0:
            raise ValueError("bad hyperparameters %s" % (hyper_parameters,))
        if self._sharded(context):
            return self._build_sharded(context, train_data, features, lam, alpha,
                                       candidate_path)
        ph = self.phase_seconds
        tp = time.perf_counter()
        users, items = ingest.IdDict(), ingest.IdDict()
        u, i, s, ts = parse_ratings(train_data, users, items, self.decay_factor,
                                    self.decay_zero_threshold, raw_out=self._raw_parse_slot(
                                        train_data, users, items),
                                    history=self._history_for(self._ctx(context).device),
                                    device_out=self._ctx(context).device.type == "cuda")
        ph["parse"] = ph.get("parse", 0.0) + time.perf_counter() - tp
        tp = time.perf_counter()
        dev = self._ctx(context).device
        ctx = self._ctx(context)
        user_ids, item_ids = users.keys(), items.keys()
        # every rank holds the same aggregated triples; each contributes a disjoint slice
        part = slice(ctx.rank, None, ctx.world_size)
        if dev.type == "cuda":
            # aggregation, the used-ID masks and the dense remap stay on the device: the
            # aggregated triples go straight into the trainer's CSR build
            ud, idv, sd = aggregate_scores_device(u, i, s, ts, self.implicit, dev,
                                                  to_host=False)
            n_agg = int(ud.numel())
            ph["aggregate"] = ph.get("aggregate", 0.0) + time.perf_counter() - tp
            if n_agg == 0:
                log.info("No ratings after aggregation")
                return None
            tp = time.perf_counter()
            mu = torch.zeros(len(user_ids), dtype=torch.bool, device=dev)
            mi = torch.zeros(len(item_ids), dtype=torch.bool, device=dev)
            mu[ud] = True
            mi[idv] = True
            used_u = torch.nonzero(mu).flatten().cpu().numpy()
            used_i = torch.nonzero(mi).flatten().cpu().numpy()
            tr_u = (torch.cumsum(mu, 0) - 1)[ud][part]
            tr_i = (torch.cumsum(mi, 0) - 1)[idv][part]
            tr_s = sd[part].to(torch.float32)
            triples = lambda: (ud, idv, sd)        # fingerprinted on the device
        else:
            u, i, s = aggregate_scores(u, i, s, ts, self.implicit)
            n_agg = len(u)
            ph["aggregate"] = ph.get("aggregate", 0.0) + time.perf_counter() - tp
            if n_agg == 0:
                log.info("No ratings after aggregation")
                return None
            tp = time.perf_counter()
            # only IDs that survived aggregation get factors (MLlib only emits rated rows)
            used_u = np.unique(u)
            used_i = np.unique(i)
            remap_u = np.full(len(user_ids), -1, dtype=np.int64)
            remap_u[used_u] = np.arange(len(used_u))
            remap_i = np.full(len(item_ids), -1, dtype=np.int64)
            remap_i[used_i] = np.arange(len(used_i))
            tr_u = torch.from_numpy(remap_u[u][part])
            tr_i = torch.from_numpy(remap_i[i][part])
            tr_s = torch.from_numpy(s[part].astype(np.float32))
            triples = lambda: (u, i, s)
        seed = rng.next_seed()
        trainer = ALSTrainer(features, lam, alpha, self.implicit, ctx=ctx, seed=seed,
                             precision=self.precision, init_seed=ALS_INIT_SEED)
        t0 = time.perf_counter()
        trainer.prepare(tr_u, tr_i, tr_s, len(used_u), len(used_i))
        del tr_u, tr_i, tr_s
        x_ids = [user_ids[j] for j in used_u.tolist()]
        y_ids = [item_ids[j] for j in used_i.tolist()]
        ph["ids_remap"] = ph.get("ids_remap", 0.0) + time.perf_counter() - tp - \
            (trainer.timings.get("prepare_s") or 0)
        ckpt_dir, fingerprint = None, ""
        if self.checkpoint_interval > 0 and self.current_model_dir:
            # neither the world size nor the init seed: a checkpoint holds global factors, and
            # a group relaunched on fewer GPUs (parallel/elastic.py) resumes from it
            fingerprint = _fingerprint(*triples(), features, lam, alpha, self.implicit,
                                       self.iterations)
            ckpt_dir = os.path.join(self.current_model_dir, ".checkpoint",
                                    "als-" + fingerprint[:16])
        x_init = y_init = None
        if self.warm_start and self.current_model_dir:
            x_init, y_init = _warm_start_factors(self.current_model_dir, features, x_ids, y_ids)
        ph["csr_prepare"] = ph.get("csr_prepare", 0.0) + (trainer.timings.get("prepare_s") or 0)
        tp = time.perf_counter()
        # random rows keyed by ID hash (this rank's rows: every world_size-th)
        W_, R_ = max(1, ctx.world_size), ctx.rank
        # (key bytes straight from the native dictionaries: no Python strings re-encoded)
        xh = ingest.blob_hash64(*users.keys_blob(np.ascontiguousarray(used_u[R_::W_])))
        yh = ingest.blob_hash64(*items.keys_blob(np.ascontiguousarray(used_i[R_::W_])))
        f = trainer.train(self.iterations, checkpoint_dir=ckpt_dir,
                          checkpoint_interval=self.checkpoint_interval, fingerprint=fingerprint,
                          x_init=x_init, y_init=y_init, x_keys=xh, y_keys=yh)
        X, Y = f.X, f.Y                 # stay on the device for the evaluation
        if self.get_test_fraction() <= 0.0:
            X = Y = None                # no evaluation: only the row text is kept
        elif X._base is not None or Y._base is not None:
            # compact copies: a view would keep the trainer's padded buffers alive
            X, Y = X.clone(), Y.clone()
        if f.X.device.type == "cuda":
            torch.cuda.synchronize(f.X.device)
        ph["train"] = ph.get("train", 0.0) + time.perf_counter() - tp
        for key in ("init_ms", "checkpoint_ms", "factors_ms"):
            if key in trainer.timings:
                self.train_phases[key[:-3]] = self.train_phases.get(key[:-3], 0.0) + \
                    trainer.timings[key] / 1e3
        its_ms = trainer.timings.get("iteration_ms", [])
        self.train_phases["iterations"] = self.train_phases.get("iterations", 0.0) + \
            sum(its_ms) / 1e3
        tp = time.perf_counter()
        # the rows' JSON text, formatted where the factors live (GPU: textfmt.hip); reused by
        # the X/ Y/ files and the UP messages
        x_rows = textfmt.format_rows(f.X) if ctx.is_main else None
        y_rows = textfmt.format_rows(f.Y) if ctx.is_main else None
        ph["format_rows"] = ph.get("format_rows", 0.0) + time.perf_counter() - tp
        log.info("ALS %d ratings, %d users, %d items, rank %d: %.3fs", n_agg, len(used_u),
                 len(used_i), features, time.perf_counter() - t0)
        if not ctx.is_main:
            return None
        tp = time.perf_counter()
        # the IDs' bytes straight from the native dictionaries (the X/ Y/ files and the UP
        # messages take them as (blob, ends): no Python string is encoded again)
        x_blob = users.keys_blob(np.ascontiguousarray(used_u, dtype=np.int64))
        y_blob = items.keys_blob(np.ascontiguousarray(used_i, dtype=np.int64))
        jobs = [(os.path.join(candidate_path, "X"), x_blob, x_rows),
                (os.path.join(candidate_path, "Y"), y_blob, y_rows)]
        if _BACKGROUND_FACTOR_FILES:
            # written beside the rest of the generation (joined at its end: join_files)
            self._writers.append(_FactorFilesWriter(jobs))
        else:
            for path, ids, rows in jobs:
                write_features(path, ids, rows)
        ph["write_factors"] = ph.get("write_factors", 0.0) + time.perf_counter() - tp
        tp = time.perf_counter()
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
        ph["pmml"] = ph.get("pmml", 0.0) + time.perf_counter() - tp
        self._cache[candidate_path] = {"x_ids": x_ids, "y_ids": y_ids, "X": X, "Y": Y,
                                       "x_rows": x_rows, "y_rows": y_rows,
                                       "x_blob": x_blob, "y_blob": y_blob,
                                       "x_codes": np.asarray(used_u), "users": users}
        its = trainer.timings.get("iteration_ms", [])
        self._timings[candidate_path] = {
            "ratings": n_agg, "users": len(used_u), "items": len(used_i),
            "prepare_s": trainer.timings.get("prepare_s"), "iteration_ms": its,
            "resumed_from_iteration": getattr(trainer, "resumed_from", 0),
            "ratings_per_s": (n_agg * 1e3 / (sum(its) / len(its))) if its else None}
        return pmml

    # ---------------------------------------------------------------- sharded path
    def _build_sharded(self, context, lines, features, lam, alpha, candidate_path):
        """Every rank builds from its share (:mod:`.sharded`)."""
        ctx = self._ctx(context)
        want_known = self.get_test_fraction() == 0.0 and not self.no_known_items
        pmml, model = sharded.build(self, ctx, lines, features, lam, alpha, candidate_path,
                                    want_known, history=self._history_for(ctx.device))
        if model is not None:
            self._cache[candidate_path] = {"sharded": model}
        return pmml

    def _evaluate_sharded(self, context, model_parent_path, test_data):
        return sharded.evaluate(self, self._ctx(context),
                                self._cache[model_parent_path]["sharded"], test_data)

    def _publish_sharded(self, context, pmml, new_data, past_data, model_parent_path, topic):
        ctx = self._ctx(context)
        src = getattr(self, "promoted_from", None)
        f = self._cache.get(src) if src else None
        have = int(f is not None and "sharded" in f)
        # every rank must take the same path: the winner of one candidate group (parallelism
        # > 1) was built in memory only by that group's ranks
        if int(shuffle.all_reduce_np(np.array([have], dtype=np.int64), ctx, op="min")[0]):
            sharded.publish(self, ctx, f["sharded"], concat_lines([new_data, past_data]),
                            topic)
        else:
            sharded.publish_from_files(self, ctx, model_parent_path,
                                       concat_lines([new_data, past_data]), topic)

    def publish_needs_model(self) -> bool:
        """The sharded publish works from each rank's build or the factor part files, never
        from the PMML."""
        return not self._sharded(self.dist_ctx) if self.dist_ctx is not None else True

    def build_timings(self, candidate_path: str) -> dict:
        return self._timings.pop(candidate_path, {})

    # ---------------------------------------------------------------- evaluate
    def _load(self, model_parent_path: str, pmml, from_files: bool = False) -> dict:
        cached = None if from_files else self._cache.get(model_parent_path)
        if cached is not None:
            return cached
        x_ids, X = read_features(os.path.join(model_parent_path,
                                              pmml.get_extension_value("X")))
        y_ids, Y = read_features(os.path.join(model_parent_path,
                                              pmml.get_extension_value("Y")))
        return {"x_ids": x_ids, "y_ids": y_ids, "X": X, "Y": Y}

    def evaluate(self, context, model, model_parent_path, test_data, train_data):
        if self._sharded(context):
            return self._evaluate_sharded(context, model_parent_path, test_data)
        tp = time.perf_counter()
        try:
            return self._evaluate_local(context, model, model_parent_path, test_data)
        finally:
            self.phase_seconds["eval"] = self.phase_seconds.get("eval", 0.0) + \
                time.perf_counter() - tp

    def _evaluate_local(self, context, model, model_parent_path, test_data):
        f = self._load(model_parent_path, model)
        users, items = ingest.IdDict(), ingest.IdDict()
        u, i, s, ts = parse_ratings(test_data, users, items, self.decay_factor,
                                    self.decay_zero_threshold)
        device = self._ctx(context).device
        # test IDs -> model rows through native dictionaries of the model's IDs
        for key, ids in (("x_dict", f["x_ids"]), ("y_dict", f["y_ids"])):
            if key not in f:
                d = ingest.IdDict()
                d.encode(list(ids))
                f[key] = d
        ucodes = f["x_dict"].find_blob(*users.keys_blob())
        icodes = f["y_dict"].find_blob(*items.keys_blob())
        if device.type == "cuda":
            au, ai, av = aggregate_scores_device(u, i, s, ts, self.implicit, device,
                                                 to_host=False)
            mu = torch.from_numpy(ucodes).to(device)[au] if au.numel() else au
            mi = torch.from_numpy(icodes).to(device)[ai] if ai.numel() else ai
        else:
            au, ai, av = aggregate_scores(u, i, s, ts, self.implicit)
            mu = ucodes[au] if len(au) else au
            mi = icodes[ai] if len(ai) else ai
        if f.get("X") is None or f.get("Y") is None:       # released or never kept
            f = dict(f)
            f.update({k: v for k, v in self._load(model_parent_path, model,
                                                           from_files=True).items()
                      if k in ("X", "Y")})
        X = f["X"] if isinstance(f["X"], torch.Tensor) else torch.from_numpy(f["X"])
        Y = f["Y"] if isinstance(f["Y"], torch.Tensor) else torch.from_numpy(f["Y"])
        cached = self._cache.get(model_parent_path)
        if cached is not None:
            self._release_factors(cached)
        X, Y = X.to(device), Y.to(device)
        if self.implicit:
            # AUC over test positives; items universe = distinct test items (known to the model)
            auc = evaluation.area_under_curve(X, Y, mu, mi, device=device)
            log.info("AUC: %s", auc)
            return auc
        rmse = evaluation.rmse(X, Y, mu, mi, av, device=device)
        log.info("RMSE: %s", rmse)
        return -rmse

    def _release_factors(self, f: dict) -> None:
        """A candidate's factor matrices are not needed once it is evaluated (publish uses the
        row text): free them instead of pinning device memory while later candidates train."""
        f["X"] = f["Y"] = None

    # ---------------------------------------------------------------- publish
    def can_publish_additional_model_data(self) -> bool:
        return True

    def publish_additional_model_data(self, context, pmml, new_data, past_data,
                                      model_parent_path, model_update_topic):
        tp = time.perf_counter()
        try:
            if self._sharded(context):
                self._publish_sharded(context, pmml, new_data, past_data, model_parent_path,
                                      model_update_topic)
            else:
                self._publish_local(pmml, new_data, past_data, model_parent_path,
                                    model_update_topic)
        finally:
            self.phase_seconds["publish_up"] = self.phase_seconds.get("publish_up", 0.0) + \
                time.perf_counter() - tp
            # the generation is done: drop the candidates' factors and the parse memo
            self._cache.clear()
            self._raw_parse = None
            self._split_test = None
        self.join_files()

    def join_files(self) -> None:
        """Wait for the factor part files written in the background (every candidate's);
        re-raises a writer's error.  The generation ends only once its files are complete."""
        tp = time.perf_counter()
        writers, self._writers = self._writers, []
        err = None
        for w in writers:
            try:
                w.join()
            except BaseException as e:   # noqa: BLE001 -- after every writer has finished
                err = err or e
            self.phase_seconds["write_factors_total"] = \
                self.phase_seconds.get("write_factors_total", 0.0) + w.seconds
        if writers:
            self.phase_seconds["write_factors_wait"] = \
                self.phase_seconds.get("write_factors_wait", 0.0) + time.perf_counter() - tp
        if err is not None:
            raise err

    def _published_rows(self, pmml, model_parent_path):
        """(x_ids, X rows text, y_ids, Y rows text) of the promoted model: from the build's
        cache when the winner was built in this process (IDs as native (blob, ends) pairs),
        else read back from its files."""
        src = getattr(self, "promoted_from", None)
        f = self._cache.get(src) if src else None
        if f is not None and f.get("x_rows") is not None:
            return (f.get("x_blob") or f["x_ids"]), f["x_rows"], \
                (f.get("y_blob") or f["y_ids"]), f["y_rows"]
        x_ids, X = read_features(os.path.join(model_parent_path, pmml.get_extension_value("X")))
        y_ids, Y = read_features(os.path.join(model_parent_path, pmml.get_extension_value("Y")))
        return x_ids, textfmt.format_rows(X), y_ids, textfmt.format_rows(Y)

    def _publish_local(self, pmml, new_data, past_data, model_parent_path, model_update_topic):
        all_data = concat_lines([new_data, past_data])
        x_ids, x_text, y_ids, y_text = self._published_rows(pmml, model_parent_path)

        def count(ids):
            return len(ids[1]) if isinstance(ids, tuple) else len(ids)

        ph = self.phase_seconds

        def lap(name, t0):
            ph["pub_" + name] = ph.get("pub_" + name, 0.0) + time.perf_counter() - t0
            return time.perf_counter()

        tp = time.perf_counter()
        log.info("Sending item / Y data as model updates")
        y_send = None
        if count(y_ids):
            y_block = ingest.assemble_row_messages("Y", y_ids, y_text)
            tp = lap("assemble_y", tp)
            if self.no_known_items or not count(x_ids):
                model_update_topic.send_block("UP", y_block)
                tp = lap("send_y", tp)
            else:
                # the Y block goes to the log on a helper thread while the known items are
                # computed (device sorts, native text); it is appended before the X block
                y_send = _Sender(model_update_topic, y_block)
        log.info("Sending user / X data as model updates")
        if not count(x_ids):
            return
        if self.no_known_items:
            model_update_topic.send_block("UP", ingest.assemble_row_messages("X", x_ids, x_text))
            lap("send_x", tp)
            return
        try:
            self._publish_x_known(all_data, users_x=(x_ids, x_text), topic=model_update_topic,
                                  y_send=y_send, lap=lap)
        finally:
            if y_send is not None:
                y_send.join(raise_error=False)

    def _publish_x_known(self, all_data, users_x, topic, y_send, lap):
        """The X rows with each user's known items (see :meth:`_publish_local`)."""
        x_ids, x_text = users_x
        model_update_topic = topic
        tp = time.perf_counter()
        parsed = self._known_items_parse(all_data)
        dev = self.dist_ctx.device if self.dist_ctx is not None else None
        if parsed is None:
            users, items = ingest.IdDict(), ingest.IdDict()
            hist = self._history_for(dev) if dev is not None else self.history
            parse = hist.parse_ratings if hist is not None else ingest.parse_ratings
            parsed = (users, items) + tuple(parse(all_data, users, items, default_ts=0))
        users = parsed[0]
        known, present = known_items_spans(*parsed, device=dev)
        tp = lap("known_items", tp)
        if known is None:
            if y_send is not None:
                y_send.join()
            return
        # join: users without any event are not sent
        n_u = len(present)
        src = getattr(self, "promoted_from", None)
        f = self._cache.get(src) if src else None
        if f is not None and f.get("users") is users and f.get("x_codes") is not None:
            code = np.asarray(f["x_codes"], dtype=np.int64)    # (x row j = user code used_u[j])
        else:
            code = users.encode(list(x_ids) if not isinstance(x_ids, tuple)
                                else _blob_keys(x_ids))
        ok = code < n_u
        ok[ok] = present[code[ok]]
        kidx = np.where(ok, code, -1)
        x_block = ingest.assemble_row_messages("X", x_ids, x_text, known, kidx)
        tp = lap("assemble_x", tp)
        if y_send is not None:
            y_send.join()                 # Y rows first, as the reference publishes them
            tp = lap("wait_y", tp)
        model_update_topic.send_block("UP", x_block)
        lap("send_x", tp)

    # ---------------------------------------------------------------- split
    def split_new_data_to_train_test(self, new_data):
        sharded = self.dist_ctx is not None and self.dist_ctx.is_distributed
        if isinstance(new_data, TextLines):
            # one native pass for the range, one for the split (no per-line arrays)
            rg = ingest.ts_range(new_data)
            if sharded:
                big = np.iinfo(np.int64).max
                mm = shuffle.all_reduce_np(np.array([-(rg[0]) if rg else -big,
                                                     rg[1] if rg else -big],
                                                    dtype=np.int64), self.dist_ctx, op="max")
                if mm[1] == -big:
                    return new_data, []
                rg = (int(-mm[0]), int(mm[1]))
            if rg is None:
                return new_data, []
            lo, hi = rg
            log.info("New data timestamp range: %d - %d", lo, hi)
            boundary = int(hi - self.get_test_fraction() * (hi - lo))
            log.info("Splitting at timestamp %d", boundary)
            train, test = ingest.split_by_time(new_data, boundary)
            self._split_test = test           # the publish step's known items add these
            return train, test
        ts = _timestamps(new_data)
        if sharded:
            # the boundary comes from the global timestamp range of the new data
            big = np.iinfo(np.int64).max
            mm = shuffle.all_reduce_np(np.array([-(int(ts.min()) if len(ts) else big),
                                                 int(ts.max()) if len(ts) else -big],
                                                dtype=np.int64), self.dist_ctx, op="max")
            if mm[1] == -big:
                return new_data, []
            lo, hi = int(-mm[0]), int(mm[1])
        elif len(ts) == 0:
            return new_data, []
        else:
            lo, hi = int(ts.min()), int(ts.max())
        log.info("New data timestamp range: %d - %d", lo, hi)
        boundary = int(hi - self.get_test_fraction() * (hi - lo))
        log.info("Splitting at timestamp %d", boundary)
        # lines that fail to parse are dropped by the parser; keep alignment via per-line parse
        if len(ts) == len(new_data) and isinstance(new_data, TextLines):
            is_train = ts < boundary
            return new_data.take(is_train), new_data.take(~is_train)
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


def known_items_json(lines: Sequence[str], device=None) -> Dict[str, str]:
    """User -> JSON array text of its known items (sorted by ID), as :func:`known_items`
    but with the time-ordered last-event selection as device sorts and the per-user lists
    joined from one array of JSON-encoded item names."""
    users, items = ingest.IdDict(), ingest.IdDict()
    u, i, s, ts = ingest.parse_ratings(lines, users, items, default_ts=0)
    return known_items_json_parsed(users, items, u, i, s, ts, device)


def known_items_json_parsed(users, items, u, i, s, ts, device=None) -> Dict[str, str]:
    """:func:`known_items_json` from already parsed events (lines without a timestamp at 0)."""
    text, present = known_items_spans(users, items, u, i, s, ts, device)
    if text is None:
        return {}
    rows = text.rows()
    uk = users.keys()
    return {uk[a]: rows[a] for a in np.flatnonzero(present).tolist()}


def known_items_spans(users, items, u, i, s, ts, device=None):
    """Known items of every user code as JSON array text (``RowText`` indexed by user code,
    item names in ID-string order) and the mask of users with any event; ``(None, None)``
    without events.  The last event per (user, item) in time order decides: a NaN strength
    (empty value) removes the item.  Sorting runs on ``device``, the text natively."""
    if len(u) == 0:
        return None, None
    ik = items.keys()
    n_i, n_u = len(ik), len(users)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if isinstance(u, torch.Tensor):
        # (the build's parse, still on the device)
        dev = u.device
        key = u.long() * n_i + i.long()
        tt = ts
        nan_all = torch.isnan(s)
        present = np.zeros(n_u, dtype=bool)
        present[torch.unique(u).cpu().numpy()] = True
    else:
        key = torch.from_numpy(u * n_i + i).to(dev)
        tt = torch.from_numpy(ts).to(dev)
        nan_all = torch.from_numpy(np.isnan(s)).to(dev)
        present = np.zeros(n_u, dtype=bool)
        present[u] = True
    o1 = torch.sort(tt, stable=True).indices
    order = o1[torch.sort(key[o1], stable=True).indices]
    key_s = key[order]
    nan_s = nan_all[order]
    last = torch.ones_like(key_s, dtype=torch.bool)
    last[:-1] = key_s[1:] != key_s[:-1]
    kk = key_s[last & ~nan_s]
    # within a user, items in ID-string order
    name_rank = np.empty(n_i, dtype=np.int64)
    name_rank[np.argsort(np.array(ik, dtype=object), kind="stable")] = np.arange(n_i)
    uu = torch.div(kk, n_i, rounding_mode="floor")
    ii = kk - uu * n_i
    rk = torch.from_numpy(name_rank).to(dev)[ii]
    o2 = torch.sort(uu * n_i + rk, stable=True).indices
    uu = uu[o2].cpu().numpy()
    ii = ii[o2].cpu().numpy()
    return ingest.known_items_text(items, uu, ii, n_u), present


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
