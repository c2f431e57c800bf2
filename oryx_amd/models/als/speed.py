"""ALS speed layer: batched GPU fold-in of new interactions into the current factors.

Equivalent of ``ALSSpeedModel`` / ``ALSSpeedModelManager``
(``[speed-app]/als/ALSSpeedModel.java:35-151``, ``ALSSpeedModelManager.java:65-215``):

* ``consume``: ``MODEL`` creates/keeps a model and prunes to ``XIDs``/``YIDs`` (recent IDs
  survive); ``UP`` sets X/Y rows (from the batch layer and from this layer's own output);
* ``build_updates``: nothing until ``fraction_loaded >= oryx.speed.min-model-load-fraction``;
  then the interval's input is time-ordered and aggregated like the batch layer, the
  Gramians XᵀX / YᵀY are formed on the device and inverted (RRQR with the reference's
  singularity check -- a singular Gramian skips the interval; the inverses are cached until
  the factors change), and ALL events are folded in at once by the fused HIP kernel
  ``oryx_als_foldin`` (``csrc/kernels/foldin.hip``: dot, target, inverse x rhs in double, axpy;
  rows read from the device mirrors by index) on a dedicated stream, instead of B independent
  k x k solves.  Each event yields ``["X",u,vec,[i]]`` and ``["Y",i,vec,[u]]``,
  whose factor rows are formatted to JSON text on the device (``csrc/kernels/textfmt.hip``)
  and assembled natively with the IDs from the parse dictionaries
  (``oryx_assemble_als_updates``).
"""

from __future__ import annotations

import json
import logging
import os
import threading
from typing import Iterable, Iterator, List, Optional, Set

import numpy as np
import torch

from ... import ingest, native
from ...api import Dataset, KeyMessage, SpeedModel, SpeedModelManager
from ...ops import als as als_ops, textfmt
from ...utils import mathx, pmml as pmmlu, text
from .batch import aggregate_scores
from .common import FeatureVectors

# queue the Gramian inverses on the fold-in stream before the micro-batch's host parse, so the
# certified fp64 inverse kernel runs under it (ORYX_SPEED_PREFETCH_INV=0: after the parse)
_PREFETCH_INV = os.environ.get("ORYX_SPEED_PREFETCH_INV", "1") != "0"
# blocks per micro-batch on the GPU path (build_update_blocks' chunks=None): each block's row
# text is copied to the host just before the block is handed to the publisher.  One block:
# 2 and 4 blocks measured 0.3-0.9 ms slower per 10k events -- each append's fixed cost
# outweighs the copy it overlaps (profiles/r6_speed_chunks_ab.txt)
_SPEED_CHUNKS = int(os.environ.get("ORYX_SPEED_CHUNKS", "1"))

__all__ = ["ALSSpeedModel", "ALSSpeedModelManager"]

log = logging.getLogger(__name__)


def _default_device():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class ALSSpeedModel(SpeedModel):
    def __init__(self, features: int, implicit: bool, device=None):
        if features <= 0:
            raise ValueError("features must be > 0")
        self.device = device or _default_device()
        self.features = features
        self.implicit = implicit
        self.X = FeatureVectors(features, self.device)
        self.Y = FeatureVectors(features, self.device)
        self._expected_users: Set[str] = set()
        self._expected_items: Set[str] = set()
        self._lock = threading.Lock()

    def get_features(self) -> int:
        return self.features

    def is_implicit(self) -> bool:
        return self.implicit

    def get_user_vector(self, user):
        return self.X.get_vector(user)

    def get_item_vector(self, item):
        return self.Y.get_vector(item)

    def set_user_vector(self, user, vector) -> None:
        if len(vector) != self.features:
            raise ValueError("wrong vector length")
        self.X.set_vector(user, vector)
        with self._lock:
            self._expected_users.discard(user)

    def set_item_vector(self, item, vector) -> None:
        if len(vector) != self.features:
            raise ValueError("wrong vector length")
        self.Y.set_vector(item, vector)
        with self._lock:
            self._expected_items.discard(item)

    def set_user_vectors(self, ids, mat) -> None:
        self.X.set_vectors(ids, mat)
        with self._lock:
            self._expected_users.difference_update(ids)

    def set_item_vectors(self, ids, mat) -> None:
        self.Y.set_vectors(ids, mat)
        with self._lock:
            self._expected_items.difference_update(ids)

    def retain_recent_and_user_ids(self, users) -> None:
        self.X.retain_recent_and_ids(users)
        with self._lock:
            self._expected_users = set(users)
            self.X.remove_all_ids_from(self._expected_users)

    def retain_recent_and_item_ids(self, items) -> None:
        self.Y.retain_recent_and_ids(items)
        with self._lock:
            self._expected_items = set(items)
            self.Y.remove_all_ids_from(self._expected_items)

    def get_xtx_solver(self):
        return mathx.get_solver(self.X.get_vtv())

    def get_yty_solver(self):
        return mathx.get_solver(self.Y.get_vtv())

    def solver_inverses(self):
        """(inverse of XtX, inverse of YtY) as fp64 device tensors, recomputed only when the
        factors changed since the last call; raises SingularMatrixSolverException like the
        solvers; None when a matrix is empty.

        On a GPU both Gramians come from the fused fp32 MFMA kernel (``ops.als.gramian``) and
        are inverted on the device by an fp64 Cholesky (one host sync for both).  The device
        result is used only when it certifies what the reference's RRQR check
        (``LinearSystemSolver.getSolver``, ``mathx.get_solver``) would accept: for SPD A every
        |R_ii| of a pivoted QR is >= lambda_min(A) >= 1 / ||A^-1||_F, so
        1 / ||A^-1||_F > ||A||_inf * ratio implies the RRQR test passes.  Anything else
        (near-singular, empty) takes the host RRQR path, which keeps its exact semantics
        (the exception and its apparent rank)."""
        key = (self.X.version, self.Y.version)
        if getattr(self, "_inv_key", None) == key:
            return self._inv
        if self.device is not None and self.device.type == "cuda":
            pending = getattr(self, "_inv_pending", None)
            self._inv_pending = None
            if pending is None or pending[0] != key:
                pending = (key,) + self._device_inverses_start()
            inv = self._device_inverses_finish(*pending[1:])
            if inv is not None:
                self._inv_key, self._inv = key, inv
                return inv
        xtx = self.get_xtx_solver()
        yty = self.get_yty_solver()
        if xtx is None or yty is None:
            inv = None
        else:
            inv = (torch.from_numpy(xtx.inverse()).to(self.device),
                   torch.from_numpy(yty.inverse()).to(self.device))
        self._inv_key, self._inv = key, inv
        return inv

    def prefetch_inverses(self, stream=None) -> None:
        """Queue the device Gramians + Cholesky inverses for the current factors (on
        ``stream``) without waiting; :meth:`solver_inverses` then only collects them.  Called
        before each GPU micro-batch's host parse (``_PREFETCH_INV``): since the inverses became
        one fused launch (``spd_inverse_pair``, ~0.11 ms on the device) the launch is cheap; in
        round 3 the ~0.6 ms of separate launches only moved into the parse phase
        (r3_speed_profile_*)."""
        if self.device is None or self.device.type != "cuda":
            return
        key = (self.X.version, self.Y.version)
        if getattr(self, "_inv_key", None) == key:
            return
        ctx = torch.cuda.stream(stream) if stream is not None else _null_ctx()
        with ctx:
            self._inv_pending = (key,) + self._device_inverses_start()

    def _device_inverses_start(self):
        if self.X.size() == 0 or self.Y.size() == 0:
            return None, None
        if self.features <= 128 and native.kernels_available():
            # both Gramians (fp32 MFMA) and both certified inverses in one more launch
            # (csrc/kernels/spdinv.hip)
            # (kept current by rank-one corrections: FeatureVectors.gramian)
            grams = [store.gramian().float().contiguous() for store in (self.X, self.Y)]
            k = self.features
            invs = [torch.empty((k, k), dtype=torch.float64, device=self.device)
                    for _ in range(2)]
            ok = torch.empty(2, dtype=torch.int32, device=self.device)
            rc = native.kernels().oryx_spd_inverse_pair(
                grams[0].data_ptr(), grams[1].data_ptr(), k, invs[0].data_ptr(),
                invs[1].data_ptr(), float(mathx.SINGULARITY_THRESHOLD_RATIO), ok.data_ptr(),
                native.stream_ptr(self.device))
            native.check(rc, "oryx_spd_inverse_pair")
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))   # the launching stream
            return (invs, ok, grams), ev
        invs, oks = [], []
        for store in (self.X, self.Y):
            a = store.gramian()
            chol, info = torch.linalg.cholesky_ex(a)
            inv = torch.cholesky_inverse(chol)
            thr = a.abs().sum(1).max() * mathx.SINGULARITY_THRESHOLD_RATIO
            oks.append((info == 0) & torch.isfinite(inv).all() & (inv.norm() * thr < 1.0))
            invs.append(inv)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return (invs, torch.stack(oks).all()), ev

    def _device_inverses_finish(self, work, ev):
        if work is None:
            return None
        torch.cuda.current_stream(self.device).wait_event(ev)
        invs, ok = work[0], work[1]
        if not bool(ok.cpu().min() if ok.dtype == torch.int32 else ok.item()):
            return None
        return invs[0], invs[1]

    def warm(self) -> float:
        """Build what the first micro-batch would otherwise build under traffic: both stores'
        native id -> row maps (a 20M-ID store takes seconds), their device mirrors, the
        Gramians and their inverses.  Called by the manager's consumer once the model is
        completely loaded (and again after each new MODEL has loaded); later writes are kept
        current incrementally (row-map journal, dirty rows, rank-one Gramian corrections).
        Returns the seconds taken."""
        import time
        t0 = time.perf_counter()
        self.X.synced_rowmap()
        self.Y.synced_rowmap()
        if self.device is not None and self.device.type == "cuda" and \
                self.X.size() and self.Y.size():
            try:
                inv = self.solver_inverses()
            except mathx.SingularMatrixSolverException:
                inv = None     # the interval reports it, as it would have
            if inv is not None and self.features <= 256 and native.kernels_available():
                self._warm_foldin(inv)
        return time.perf_counter() - t0

    def _warm_foldin(self, inv) -> None:
        """One fold-in of a single event (row 0 of each store, output discarded) and the
        formatting of its rows: the kernels' first launches -- code objects loaded, 10 ms
        each -- happen here and not in the first micro-batch, which otherwise held the GPU
        while the serving process beside it answered requests (r6_traffic_*_v5)."""
        from ...ops import textfmt as tf
        k = self.features
        dev = self.device
        xm, ym = self.X.device_view()[0], self.Y.device_view()[0]
        r = torch.zeros(1, dtype=torch.int64, device=dev)
        vals = torch.ones(1, dtype=torch.float32, device=dev)
        new = torch.empty((2, k), dtype=torch.float32, device=dev)
        flags = torch.empty(2, dtype=torch.uint8, device=dev)
        xinv, yinv = inv
        lib = native.require_kernels()
        native.check(lib.oryx_als_foldin(
            xm.contiguous().data_ptr(), ym.contiguous().data_ptr(), k, r.data_ptr(),
            r.data_ptr(), vals.data_ptr(), xinv.contiguous().data_ptr(),
            yinv.contiguous().data_ptr(), int(self.implicit), 1, new[:1].data_ptr(),
            new[1:].data_ptr(), flags[:1].data_ptr(), flags[1:].data_ptr(),
            native.stream_ptr(dev)), "oryx_als_foldin")
        tf.format_rows_and(new, flags)
        torch.cuda.synchronize(dev)

    def get_fraction_loaded(self) -> float:
        with self._lock:
            expected = len(self._expected_users) + len(self._expected_items)
        if expected == 0:
            return 1.0
        loaded = float(self.X.size() + self.Y.size())
        return loaded / (loaded + expected)

    def __repr__(self):
        return "ALSSpeedModel[features:%d, implicit:%s, X:(%d users), Y:(%d items), " \
               "fractionLoaded:%s]" % (self.features, self.implicit, self.X.size(),
                                       self.Y.size(), self.get_fraction_loaded())


class ALSSpeedModelManager(SpeedModelManager):
    def __init__(self, config):
        self.no_known_items = config.get_bool("oryx.als.no-known-items")
        self.min_model_load_fraction = config.get_double("oryx.speed.min-model-load-fraction")
        if not (0.0 <= self.min_model_load_fraction <= 1.0):
            raise ValueError("bad min-model-load-fraction")
        self.model: Optional[ALSSpeedModel] = None
        self._stream = None
        self._dicts = None
        self._batch = None     # ingest.SpeedBatch of the GPU path (reused)
        self._text_ws: dict = {}   # device buffer of the UP rows' text (textfmt)
        self._warmed = None    # the model last warmed (ALSSpeedModel.warm) once loaded
        self.warm_s: Optional[float] = None
        # milliseconds per phase of the last build_updates (parse_aggregate, inverses, lookup
        # of the batch's IDs in the stores, foldin = kernel + validity flags to the host,
        # format_rows = GPU row text + copy, assemble = native UP message assembly)
        self.last_phase_ms = {}

    def consume(self, updates: Iterator[KeyMessage], context=None) -> None:
        countdown = 10000
        for km in updates:
            key, message = km.key, km.message
            if key is None:
                raise ValueError("Bad message: %r" % (km,))
            if key == "UP":
                if self.model is None:
                    continue
                take = getattr(updates, "take_buffered", None)
                if take is not None:
                    from .serving import apply_up_batch, drain_up_blocks
                    batch = [message] + [m.message for m in take(lambda m: m.key == "UP",
                                                                 poll=False)]
                    apply_up_batch(self.model, batch)
                    countdown -= len(batch) + drain_up_blocks(self.model, updates)
                    if countdown <= 0:
                        log.info("%s", self.model)
                        countdown = 10000
                    self._maybe_warm()
                    continue
                update = text.read_json(message)
                id_ = str(update[1])
                vec = np.asarray(update[2], dtype=np.float32)
                if update[0] == "X":
                    self.model.set_user_vector(id_, vec)
                elif update[0] == "Y":
                    self.model.set_item_vector(id_, vec)
                else:
                    raise ValueError("Bad message: %r" % (km,))
                countdown -= 1
                if countdown <= 0:
                    log.info("%s", self.model)
                    countdown = 10000
                self._maybe_warm()
            elif key in ("MODEL", "MODEL-REF"):
                log.info("Loading new model")
                pmml = pmmlu.read_pmml_from_update_key_message(key, message)
                features = int(pmml.get_extension_value("features"))
                implicit = pmml.get_extension_value("implicit").lower() == "true"
                if self.model is None or features != self.model.get_features():
                    log.warning("No previous model, or # features has changed; creating new one")
                    self.model = ALSSpeedModel(features, implicit)
                xids = set(pmml.get_extension_content("XIDs") or [])
                yids = set(pmml.get_extension_content("YIDs") or [])
                self.model.retain_recent_and_user_ids(xids)
                self.model.retain_recent_and_item_ids(yids)
                self._warmed = None        # warm again once this model has loaded
                # the loop frame outlives this message: drop the ID sets (20M strings in
                # a set stay in every gen-2 GC walk until the next model otherwise)
                del xids, yids, pmml
                log.info("Model updated: %s", self.model)
            else:
                raise ValueError("Bad message: %r" % (km,))

    def _maybe_warm(self) -> None:
        """Warm the model on this (consumer) thread once it has completely loaded: the first
        micro-batch after a load otherwise built the 20M-entry row maps and the device
        mirrors itself -- a 5 s interval under traffic at 20M x 250
        (profiles/r5_traffic_20m_250_*_v4.json)."""
        m = self.model
        if m is None or self._warmed is m or m.get_fraction_loaded() < 1.0:
            return
        self._warmed = m
        self.warm_s = m.warm()
        log.info("Speed model warmed in %.2fs", self.warm_s)

    def _device_stream(self, device):
        if device.type != "cuda":
            return None
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=device)
        return self._stream

    def build_updates(self, new_data: Dataset) -> List[str]:
        """All UP messages of the interval (one :class:`~oryx_amd.api.MessageBlock` on the
        GPU path)."""
        blocks = [b.materialize() if hasattr(b, "materialize") else b
                  for b in self.build_update_blocks(new_data, chunks=1)]
        if not blocks:
            return []
        return blocks[0] if len(blocks) == 1 else [m for b in blocks for m in b]

    def build_update_blocks(self, new_data: Dataset, chunks: Optional[int] = None):
        """The interval's UP messages as a generator of blocks over consecutive event ranges
        (the same messages in the same order as :meth:`build_updates`): a publisher appends
        block j on another thread while block j + 1 is assembled
        (:func:`oryx_amd.layers.speed.publish_blocks`).  One block by default: on the GPU
        box, 4 blocks ran slower (8.3 -> 9.4 ms per 10k events) -- the threaded assembler and
        the log append's CRC threads compete for the same cores, and the append itself is
        bound by the kernel's page-cache copy (profiles/r3_speed_profile_*.txt)."""
        model = self.model
        if model is None or model.get_fraction_loaded() < self.min_model_load_fraction:
            return
        import time
        t0 = time.perf_counter()
        dev = model.device
        if dev.type == "cuda" and model.features <= 256:
            # the GPU path: lines parsed on the native threads straight to store rows
            # (ingest.SpeedBatch; no per-batch dictionaries), aggregated natively
            if self._batch is None:
                self._batch = ingest.SpeedBatch()
            sb = self._batch
            if _PREFETCH_INV:
                try:
                    model.prefetch_inverses(self._device_stream(dev))
                except mathx.SingularMatrixSolverException:
                    pass          # solver_inverses reports it after the parse, as before
            xm, ym = model.X.synced_rowmap(), model.Y.synced_rowmap()
            with model.X.read_lock(), model.Y.read_lock():
                sb.parse(new_data.values(), xm, ym, default_ts=0)
            u, i, s = sb.aggregate(model.is_implicit())
            self.last_phase_ms = {"parse_aggregate": (time.perf_counter() - t0) * 1e3}
            if len(u):
                yield from self._build_updates_fused(model, sb, u, i, s, chunks)
            return
        # per-batch dictionaries, reused (cleared) so their tables are not reallocated and
        # re-faulted every micro-batch
        if self._dicts is None:
            self._dicts = (ingest.IdDict(), ingest.IdDict())
        users, items = (d.clear() for d in self._dicts)
        u, i, s, ts = ingest.parse_ratings(new_data.values(), users, items, default_ts=0)
        u, i, s = aggregate_scores(u, i, s, ts, model.is_implicit())
        self.last_phase_ms = {"parse_aggregate": (time.perf_counter() - t0) * 1e3}
        if len(u) == 0:
            return
        out = self._build_updates_host(model, users, items, u, i, s)
        if out:
            yield out

    def _build_updates_host(self, model, users, items, u, i, s) -> List[str]:
        try:
            xtx = model.get_xtx_solver()
            yty = model.get_yty_solver()
        except mathx.SingularMatrixSolverException:
            return []
        if xtx is None or yty is None:
            return []
        uk, ik = users.keys(), items.keys()
        u_ids = [uk[j] for j in u.tolist()]
        i_ids = [ik[j] for j in i.tolist()]
        dev = model.device
        stream = self._device_stream(dev)
        ctx = torch.cuda.stream(stream) if stream is not None else _null_ctx()
        with ctx:
            xmat, _, _ = model.X.device_view()
            ymat, _, _ = model.Y.device_view()
            xrows = np.array([model.X.row_of(a) if model.X.row_of(a) is not None else -1
                              for a in u_ids], dtype=np.int64)
            yrows = np.array([model.Y.row_of(b) if model.Y.row_of(b) is not None else -1
                              for b in i_ids], dtype=np.int64)
            xr = torch.from_numpy(np.maximum(xrows, 0)).to(dev)
            yr = torch.from_numpy(np.maximum(yrows, 0)).to(dev)
            xpres = torch.from_numpy(xrows >= 0).to(dev)
            ypres = torch.from_numpy(yrows >= 0).to(dev)
            xu = torch.where(xpres[:, None], xmat[xr] if len(xmat) else
                             torch.zeros(len(xr), model.features, device=dev),
                             torch.zeros((), device=dev))
            yi = torch.where(ypres[:, None], ymat[yr] if len(ymat) else
                             torch.zeros(len(yr), model.features, device=dev),
                             torch.zeros((), device=dev))
            # the reference folds in strength.floatValue() (ALSSpeedModelManager.java:170)
            vals = torch.from_numpy(np.asarray(s, dtype=np.float32).astype(np.float64)).to(dev)
            yinv = torch.from_numpy(yty.inverse()).to(dev)
            xinv = torch.from_numpy(xtx.inverse()).to(dev)
            new_x, valid_x = als_ops.fold_in(yinv, vals, xu, xpres, yi, model.is_implicit())
            new_y, valid_y = als_ops.fold_in(xinv, vals, yi, ypres, xu, model.is_implicit())
            # Yi absent -> no X update; Xu absent -> no Y update (computeUpdatedXu(null) = null)
            valid_x = valid_x & ypres
            valid_y = valid_y & xpres
            nx, vx = new_x.cpu().numpy(), valid_x.cpu().numpy()
            ny, vy = new_y.cpu().numpy(), valid_y.cpu().numpy()
        x_rows = ingest.format_float_rows(nx)
        y_rows = ingest.format_float_rows(ny)
        out: List[str] = []
        for j in range(len(u_ids)):
            if vx[j]:
                out.append(self._to_update_json("X", u_ids[j], x_rows[j], i_ids[j]))
            if vy[j]:
                out.append(self._to_update_json("Y", i_ids[j], y_rows[j], u_ids[j]))
        return out

    def _build_updates_fused(self, model, sb, u, i, s, chunks: int = 1):
        """Fold-in of the aggregated pairs (``u`` / ``i``: store rows, -1 for IDs the stores
        lack) with the fused HIP kernel, rows formatted on the GPU, UP messages assembled from
        the micro-batch's own key bytes (``sb``: the parsed :class:`~oryx_amd.ingest.
        SpeedBatch`)."""
        import time
        from ... import native
        ph = self.last_phase_ms
        t0 = time.perf_counter()
        try:
            inv = model.solver_inverses()
        except mathx.SingularMatrixSolverException:
            return
        if inv is None:
            return
        ph["inverses"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        xinv, yinv = inv
        dev = model.device
        k = model.features
        t0 = time.perf_counter()
        n = len(u)
        lib = native.require_kernels()
        stream = self._device_stream(dev)
        with torch.cuda.stream(stream):
            xmat, _, _ = model.X.device_view()
            ymat, _, _ = model.Y.device_view()
            xm = xmat if len(xmat) else torch.zeros((1, k), device=dev)
            ym = ymat if len(ymat) else torch.zeros((1, k), device=dev)
            xr = torch.from_numpy(np.ascontiguousarray(u, dtype=np.int64)).to(dev)
            yr = torch.from_numpy(np.ascontiguousarray(i, dtype=np.int64)).to(dev)
            # the reference folds in strength.floatValue() (ALSSpeedModelManager.java:170)
            vals = torch.from_numpy(np.asarray(s, dtype=np.float32)).to(dev)
            # both sides' rows in one matrix (formatted in one pass), flags likewise
            new = torch.empty((2 * n, k), dtype=torch.float32, device=dev)
            flags = torch.empty(2 * n, dtype=torch.uint8, device=dev)
            new_x, new_y, vx, vy = new[:n], new[n:], flags[:n], flags[n:]
            rc = lib.oryx_als_foldin(xm.contiguous().data_ptr(), ym.contiguous().data_ptr(), k,
                                     xr.data_ptr(), yr.data_ptr(), vals.data_ptr(),
                                     xinv.contiguous().data_ptr(), yinv.contiguous().data_ptr(),
                                     int(model.is_implicit()), n, new_x.data_ptr(),
                                     new_y.data_ptr(), vx.data_ptr(), vy.data_ptr(),
                                     native.stream_ptr(dev))
            native.check(rc, "oryx_als_foldin")
            ph["foldin"] = (time.perf_counter() - t0) * 1e3
            t0 = time.perf_counter()
            # the updated rows become JSON text on the device (csrc/kernels/textfmt.hip); the
            # row ends and validity flags come back first, then the text of each block's rows
            # just before the block is handed on, so a block's append (on the publisher's
            # thread) overlaps the next block's copy
            rows, valid = textfmt.format_rows_device(new, flags, self._text_ws)
        ph["format_rows"] = (time.perf_counter() - t0) * 1e3
        ph["assemble"] = 0.0
        vxh, vyh = valid[:n] > 0, valid[n:] > 0
        chunks = max(1, min(int(chunks or _SPEED_CHUNKS), n // 1024 or 1))
        # x rows are rows [0, n) of the formatted matrix, y rows [n, 2n): one view each over
        # the host buffer, filled per block
        xrows, yrows = rows.view(0, n), rows.view(n, 2 * n)
        for c in range(chunks):
            t0 = time.perf_counter()
            lo, hi = n * c // chunks, n * (c + 1) // chunks
            with torch.cuda.stream(stream):
                rows.fetch([(lo, hi), (n + lo, n + hi)])
            ph["format_rows"] += (time.perf_counter() - t0) * 1e3
            t0 = time.perf_counter()
            # formatted by the log's writer threads straight into the update-log segment
            # when published to a native topic (ingest.DeferredUpBlock), so the assembly
            # time shows in the append
            blk = sb.deferred(lo, hi, xrows, yrows, vxh, vyh, not self.no_known_items)
            ph["assemble"] += (time.perf_counter() - t0) * 1e3
            yield blk

    def _to_update_json(self, matrix: str, id_: str, vec_json: str, other: str) -> str:
        if self.no_known_items:
            return '["%s",%s,%s]' % (matrix, json.dumps(id_), vec_json)
        return '["%s",%s,%s,[%s]]' % (matrix, json.dumps(id_), vec_json, json.dumps(other))

    def close(self) -> None:
        pass


class _null_ctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
