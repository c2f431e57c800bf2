"""ALS shared pieces: fold-in math and feature-vector stores.

* :func:`compute_target_qui` / :func:`compute_updated_xu` -- scalar host versions of
  ``ALSUtils`` (``[app-common]/als/ALSUtils.java:37-106``), bit-faithful to the reference's
  float/double mix (used by ``/recommendToAnonymous`` etc.; the speed layer uses the batched
  device form in :func:`oryx_amd.ops.als.fold_in`).
* :class:`FeatureVectors` -- ``id -> vector`` store with "recent IDs" and Gramian
  (``[app-common]/als/FeatureVectors.java:36-161``), backed by a growable matrix: a numpy host
  mirror (O(1) lookups without device syncs) plus, when a device is given, a device-resident
  copy in HBM that is refreshed lazily in one batched H2D copy per query burst.  Removed rows
  are zeroed and recycled.  The device copy is what the GPU top-N scan reads.
"""

from __future__ import annotations

import math
import mmap
import threading
import time
from typing import Callable, Collection, Dict, Iterable, List, Optional, Sequence, Set, Tuple

import numpy as np
import torch

from ...utils import lang, mathx

__all__ = ["compute_target_qui", "compute_updated_xu", "FeatureVectors"]


def compute_target_qui(implicit: bool, value: float, current_value: float) -> float:
    if implicit:
        if value > 0.0 and current_value < 1.0:
            diff = 1.0 - max(0.0, current_value)
            return current_value + (value / (1.0 + value)) * diff
        if value < 0.0 and current_value > 0.0:
            diff = -min(1.0, current_value)
            return current_value + (value / (value - 1.0)) * diff
        return float("nan")
    return value


def compute_updated_xu(solver, value: float, xu: Optional[np.ndarray], yi: Optional[np.ndarray],
                       implicit: bool) -> Optional[np.ndarray]:
    if yi is None:
        return None
    qui = 0.0 if xu is None else mathx.dot(xu, yi)
    target = compute_target_qui(implicit, value, 0.5 if xu is None else qui)
    if math.isnan(target):
        return None
    dqui = target - qui
    # Java: float[] dQuiYi ... dQuiYi[i] *= dQui (double): product in double, one rounding
    dqui_yi = (np.asarray(yi, dtype=np.float32).astype(np.float64) * dqui).astype(np.float32)
    dxu = solver.solve_f_to_f(dqui_yi)
    if xu is None:
        return dxu
    return (np.asarray(xu, dtype=np.float32) + dxu).astype(np.float32)


def _big_zeros(shape) -> np.ndarray:
    """Zeroed fp32 array; above 1 GiB an anonymous mapping advised for transparent huge
    pages (a 20 GB factor matrix filled 24 MB at a time otherwise takes a page fault per
    4 KB -- seconds of a model load)."""
    nbytes = int(np.prod(shape)) * 4
    if nbytes < (1 << 30) or not hasattr(mmap, "MADV_HUGEPAGE"):
        return np.zeros(shape, dtype=np.float32)
    m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    try:
        m.madvise(mmap.MADV_HUGEPAGE)
    except OSError:
        pass
    return np.frombuffer(m, dtype=np.float32, count=int(np.prod(shape))).reshape(shape)


class FeatureVectors:
    """Thread-safe ``id -> float32[k]`` store; optional device mirror for GPU scans."""

    def __init__(self, features: int, device: Optional[torch.device] = None,
                 initial_capacity: int = 1024, partitioner: Optional[Callable] = None,
                 row_pad: int = 1):
        self.k = int(features)
        self.device = device
        # device rows are ``ld`` floats apart (k rounded up to ``row_pad``, pad columns zero):
        # the serving scan kernel reads the mirror in place in whole 16-float steps
        self.ld = -(-self.k // max(1, int(row_pad))) * max(1, int(row_pad))
        self._lock = lang.AutoReadWriteLock()
        self._index: Dict[str, int] = {}
        # row -> ID (None: free row) and row -> "added since the last retain" flags, as
        # numpy arrays rather than a list and a set of strings: neither is a cyclic-GC
        # container, so a 20M-row store adds nothing to a gen-2 collection's walk (the list
        # and set of 20M item IDs cost the serving process ~1 s of stopped handlers per pass)
        self._ids = np.empty(0, dtype=object)
        self._recent_rows = np.zeros(0, dtype=bool)
        self._free: List[int] = []
        cap = max(16, int(initial_capacity))
        self._host = np.zeros((cap, self.k), dtype=np.float32)
        self._host_valid = np.zeros(cap, dtype=bool)
        self._n_rows = 0                      # high-water mark of used rows
        self._dirty: Set[int] = set()
        self._dirty_all = False
        self._dev = None                      # fp32 [cap, k]
        self._dev_valid = None                # bool [cap]
        self._dev_norm = None                 # fp32 [cap]
        self._dev_lock = threading.RLock()
        # VtV kept current by rank-one corrections (gramian()): the Gramian of the state at the
        # last full computation, plus the old (removed / overwritten) and new row values since
        self._gram: Optional[torch.Tensor] = None
        self._gram_sub: List[np.ndarray] = []
        self._gram_add: List[np.ndarray] = []
        self._gram_pending = 0
        self._gram_corrected = 0
        self._gram_lock = threading.Lock()
        self.gram_stats = {"full": 0, "incremental": 0}
        self.partitioner = partitioner        # rows -> partition ids (device LSH)
        self._dev_part = None
        self.version = 0
        # bumped only when the ID <-> row assignment changes (IDs added or removed), not by
        # value updates: caches keyed by ID (id_array, rescorer row masks) survive the latter
        self.id_version = 0
        # rows changed since the last take_index_dirty() (serving ItemIndex); None = all
        # rows changed since each index consumer's last take_index_state (token -> rows; None:
        # everything may have changed).  One set per consumer: two indexes over one store
        # (e.g. a single-GPU and an item-sharded one) must not consume each other's changes
        self._idx_dirty: Dict[int, Optional[Set[int]]] = {}
        # native id -> row mirror (ingest.RowMap) for bulk lookups, built on first use and
        # then kept current from a journal of id insertions / removals
        self._rowmap = None
        self._journal: Optional[list] = None

    # ---------------------------------------------------------------- basic map API
    def size(self) -> int:
        return len(self._index)

    def __len__(self):
        return self.size()

    def __contains__(self, id_: str) -> bool:
        return id_ in self._index

    def get_vector(self, id_: str) -> Optional[np.ndarray]:
        with self._lock.read():
            row = self._index.get(id_)
            if row is None:
                return None
            return self._host[row].copy()

    def row_of(self, id_: str) -> Optional[int]:
        return self._index.get(id_)

    def id_of_row(self, row: int) -> Optional[str]:
        return self._ids[row] if 0 <= row < self._n_rows else None

    def _alloc_row(self) -> int:
        if self._free:
            return self._free.pop()
        row = self._n_rows
        if row >= self._host.shape[0]:
            cap = self._host.shape[0] * 2
            host = np.zeros((cap, self.k), dtype=np.float32)
            host[:self._host.shape[0]] = self._host
            valid = np.zeros(cap, dtype=bool)
            valid[:self._host_valid.shape[0]] = self._host_valid
            self._host, self._host_valid = host, valid
            self._dirty_all = True
            self._idx_mark_all()
        self._n_rows += 1
        self._ids_fit(self._n_rows)
        return row

    def _ids_fit(self, rows: int) -> None:
        """Grow the row -> ID and recent-flag arrays to hold ``rows`` rows."""
        cap = len(self._ids)
        if rows <= cap:
            return
        cap = max(rows, 2 * cap, 1024)
        ids = np.empty(cap, dtype=object)
        ids[:len(self._ids)] = self._ids
        rec = np.zeros(cap, dtype=bool)
        rec[:len(self._recent_rows)] = self._recent_rows
        self._ids, self._recent_rows = ids, rec

    def set_vector(self, id_: str, vector) -> None:
        v = np.asarray(vector, dtype=np.float32)
        if v.shape != (self.k,):
            raise ValueError("vector length %s != features %d" % (v.shape, self.k))
        with self._lock.write():
            row = self._index.get(id_)
            old = None
            if row is None:
                row = self._alloc_row()
                self._index[id_] = row
                self._ids[row] = id_
                self._recent_rows[row] = True
                self.id_version += 1
                if self._journal is not None:
                    self._journal.append((True, id_, row))
            elif self._gram is not None and self._host_valid[row]:
                old = self._host[row][None].copy()
            if self._gram is not None:
                self._gram_note(old, v[None])
            self._host[row] = v
            self._host_valid[row] = True
            self._dirty.add(row)
            self._idx_mark((row,))
            self.version += 1

    def _idx_mark(self, rows) -> None:
        for d in self._idx_dirty.values():
            if d is not None:
                d.update(rows)

    def _idx_mark_all(self) -> None:
        for t in self._idx_dirty:
            self._idx_dirty[t] = None

    def register_index_consumer(self) -> int:
        """A token for :meth:`take_index_state`; its first call reports everything."""
        with self._lock.write():
            token = len(self._idx_dirty) + 1
            while token in self._idx_dirty:
                token += 1
            self._idx_dirty[token] = None
            return token

    def take_index_dirty(self, token: int = 0) -> Optional[np.ndarray]:
        """Rows changed since the previous call (None: everything may have changed)."""
        return self.take_index_state(token)[1]

    def take_index_state(self, token: int = 0) -> Tuple[int, Optional[np.ndarray]]:
        """(version, rows changed since this consumer's previous call), read together under
        the write lock (None rows: everything may have changed).  A consumer that then takes
        :meth:`device_view` sees at least these changes; a write landing in between shows up
        again in the next call's rows, so re-applying it is all that can happen."""
        with self._lock.write():
            ver = self.version
            d = self._idx_dirty.get(token)
            self._idx_dirty[token] = set()
        if d is None:
            return ver, None
        return ver, np.fromiter(d, dtype=np.int64, count=len(d))

    def _ensure_capacity(self, rows: int) -> None:
        cap = self._host.shape[0]
        if rows <= cap:
            return
        while cap < rows:
            cap *= 2
        host = np.zeros((cap, self.k), dtype=np.float32)
        host[:self._host.shape[0]] = self._host
        valid = np.zeros(cap, dtype=bool)
        valid[:self._host_valid.shape[0]] = self._host_valid
        self._host, self._host_valid = host, valid
        self._dirty_all = True
        self._idx_mark_all()

    def reserve_extra(self, extra: int) -> None:
        """Grow the host matrix to hold ``extra`` more new rows in one step (a model load
        knows how many IDs are coming: doubling 20M x 250 fp32 rows up from the initial
        capacity copied ~30 GB along the way)."""
        with self._lock.write():
            rows = self._n_rows + max(0, int(extra))
            cap = self._host.shape[0]
            if rows <= cap:
                return
            host = _big_zeros((rows, self.k))
            host[:cap] = self._host
            valid = np.zeros(rows, dtype=bool)
            valid[:cap] = self._host_valid
            self._host, self._host_valid = host, valid
            self._dirty_all = True
            self._idx_mark_all()

    def set_vectors(self, ids: Sequence[str], matrix: np.ndarray) -> None:
        """Bulk insert/update (model loading): new IDs get one contiguous block of rows; an ID
        repeated within the batch ends with its last row."""
        matrix = np.asarray(matrix, dtype=np.float32)
        if matrix.ndim != 2 or matrix.shape[1] != self.k or len(ids) != matrix.shape[0]:
            raise ValueError("bad matrix shape %s for %d ids" % (matrix.shape, len(ids)))
        with self._lock.write():
            index = self._index
            if index and not index.keys().isdisjoint(ids):
                rows = np.fromiter((index.get(i, -1) for i in ids), dtype=np.int64,
                                   count=len(ids))
            else:
                # no ID of the batch is stored yet (a model load): one C-level disjointness
                # pass instead of a Python-level lookup per ID
                rows = np.full(len(ids), -1, dtype=np.int64)
            new_pos = np.nonzero(rows < 0)[0]
            if len(new_pos):
                new_ids = [ids[j] for j in new_pos.tolist()] if len(new_pos) < len(ids) \
                    else (ids if isinstance(ids, list) else list(ids))
                start = self._n_rows
                before = len(index)
                index.update(zip(new_ids, range(start, start + len(new_ids))))
                dup = len(index) - before != len(new_ids)
                if dup:
                    for i in new_ids:
                        index.pop(i, None)
                if dup:
                    # duplicates within the batch: fall back to the one-by-one path
                    self._gram_drop()
                    for id_, v in zip(ids, matrix):
                        row = index.get(id_)
                        if row is None:
                            row = self._alloc_row()
                            index[id_] = row
                            self._ids[row] = id_
                            self._recent_rows[row] = True
                            self.id_version += 1
                            if self._journal is not None:
                                self._journal.append((True, id_, row))
                        self._host[row] = v
                        self._host_valid[row] = True
                        self._dirty.add(row)
                    self._idx_mark_all()
                    self.version += 1
                    return
                self._ensure_capacity(start + len(new_ids))
                new_rows = np.arange(start, start + len(new_ids), dtype=np.int64)
                if self._journal is not None:
                    self._journal.append((True, new_ids, new_rows))
                end = start + len(new_ids)
                self._ids_fit(end)
                self._ids[start:end] = new_ids
                self._recent_rows[start:end] = True
                self.id_version += 1
                self._n_rows = start + len(new_ids)
                rows[new_pos] = new_rows
                if len(new_pos) == len(ids):
                    # every ID new (the bulk load): one contiguous block, slice copies
                    end = start + len(ids)
                    if self._gram is not None:
                        self._gram_note(None, matrix)
                    self._host[start:end] = matrix
                    self._host_valid[start:end] = True
                    self._mark_written(rows)
                    return
            if self._gram is not None:
                if len(np.unique(rows)) != len(rows):
                    self._gram_drop()          # a repeated row: only its last value stays
                else:
                    was = self._host_valid[rows]
                    self._gram_note(self._host[rows[was]] if was.any() else None, matrix)
            self._host[rows] = matrix
            self._host_valid[rows] = True
            self._mark_written(rows)

    def _mark_written(self, rows: np.ndarray) -> None:
        """Dirty tracking for a bulk write (write lock held): per-row sets while they stay
        small, else everything (a model load would otherwise put every one of its millions
        of rows into Python sets, and the device refresh then re-uploads in full anyway)."""
        if self._dirty_all or len(rows) + len(self._dirty) > max(1024, self._n_rows // 8):
            self._dirty_all = True
            self._dirty.clear()
            self._idx_mark_all()
        else:
            self._dirty.update(rows.tolist())
            self._idx_mark(rows.tolist())
        self.version += 1

    def remove_vector(self, id_: str) -> None:
        with self._lock.write():
            self._remove_locked(id_)

    def _remove_locked(self, id_: str) -> None:
        row = self._index.pop(id_, None)
        if row is not None and self._journal is not None:
            self._journal.append((False, id_, row))
        if row is not None:
            if self._gram is not None and self._host_valid[row]:
                self._gram_note(self._host[row][None].copy(), None)
            self._host[row] = 0.0
            self._host_valid[row] = False
            self._ids[row] = None
            self._recent_rows[row] = False
            self.id_version += 1
            self._free.append(row)
            self._dirty.add(row)
            self._idx_mark((row,))
            self.version += 1

    def native_rows(self, d) -> np.ndarray:
        """Rows of every key of the native dictionary ``d`` (``ingest.IdDict``) in code
        order, -1 for IDs not in the store: one native translation instead of a Python dict
        lookup per ID (the speed layer resolves a micro-batch's users / items this way)."""
        with self._lock.write():
            self._sync_rowmap()
            return self._rowmap.translate(d)

    def synced_rowmap(self):
        """The native id -> row map (``ingest.RowMap``), brought up to date with every write
        so far.  Readers hold :meth:`read_lock` while they use it (only the sync mutates
        it, under the write lock)."""
        with self._lock.write():
            self._sync_rowmap()
            return self._rowmap

    def read_lock(self):
        return self._lock.read()

    def _sync_rowmap(self) -> None:
        from ... import ingest
        if self._rowmap is None:
            self._rowmap = ingest.RowMap()
            ids = list(self._index.keys())
            self._rowmap.set(ids, np.fromiter(self._index.values(), dtype=np.int64,
                                              count=len(ids)))
            self._journal = []
        elif self._journal:
            # replay in order, batching runs of the same kind
            run_kind, run_ids, run_rows = None, [], []

            def flush():
                if run_kind:
                    self._rowmap.set(run_ids, np.asarray(run_rows, dtype=np.int64))
                elif run_kind is not None:
                    self._rowmap.remove(run_ids)
            for kind, ids, rows in self._journal:
                if kind != run_kind:
                    flush()
                    run_kind, run_ids, run_rows = kind, [], []
                if isinstance(ids, list):
                    run_ids.extend(ids)
                    run_rows.extend(np.asarray(rows).tolist())
                else:
                    run_ids.append(ids)
                    run_rows.append(int(rows))
            flush()
            self._journal = []

    def add_all_ids_to(self, out: Set[str]) -> None:
        with self._lock.read():
            out.update(self._index.keys())

    def remove_all_ids_from(self, out: Set[str]) -> None:
        with self._lock.read():
            out.difference_update(self._index.keys())

    def add_all_recent_to(self, out: Set[str]) -> None:
        with self._lock.read():
            n = self._n_rows
            out.update(self._ids[:n][self._recent_rows[:n]].tolist())

    def all_ids(self) -> List[str]:
        with self._lock.read():
            return list(self._index.keys())

    def retain_recent_and_ids(self, new_model_ids: Collection[str]) -> None:
        keep = new_model_ids if isinstance(new_model_ids, (set, frozenset)) else set(new_model_ids)
        with self._lock.write():
            rec = self._recent_rows
            for id_ in [i for i, r in self._index.items() if i not in keep and not rec[r]]:
                self._remove_locked(id_)
            self._recent_rows[:] = False

    def for_each(self, fn: Callable[[str, np.ndarray], None]) -> None:
        with self._lock.read():
            for id_, row in self._index.items():
                fn(id_, self._host[row])

    def get_vtv(self) -> Optional[np.ndarray]:
        """Gramian VᵀV (float64) on the device when present, else on the host."""
        if self.size() == 0:
            return None
        if self.device is not None and self.device.type == "cuda":
            return self.gramian().cpu().numpy()
        with self._lock.read():
            m = self._host[:self._n_rows][self._host_valid[:self._n_rows]]
            return mathx.transpose_times_self(m)

    # ---------------------------------------------------------------- incremental Gramian
    # corrections kept per row change; past this many pending rows (or once the corrections
    # since the last full computation add up to the store's size) the next call recomputes
    GRAM_MAX_PENDING = 1 << 16

    def _gram_note(self, old: Optional[np.ndarray], new: Optional[np.ndarray]) -> None:
        """Record a change for gramian() (write lock held; called only while _gram is set)."""
        n = 0
        if old is not None and len(old):
            self._gram_sub.append(np.array(old, dtype=np.float32))
            n = len(old)
        if new is not None and len(new):
            self._gram_add.append(np.array(new, dtype=np.float32))
            n = max(n, len(new))
        self._gram_pending += n
        if self._gram_pending > max(self.GRAM_MAX_PENDING, self._n_rows // 8):
            self._gram_drop()

    def _gram_drop(self) -> None:
        self._gram = None
        self._gram_sub, self._gram_add = [], []
        self._gram_pending = 0

    def gramian(self) -> Optional[torch.Tensor]:
        """VtV (float64 [k, k], on the device mirror's device) of the current vectors.

        The first call (and one after a bulk load) multiplies the whole device mirror; after
        that each call only applies the rank-one corrections of the rows written or removed
        since (new rows' v v^T added, old values' subtracted, in float64): a speed layer whose
        model takes a few hundred UP rows per micro-batch no longer re-reads a 20M x 250
        matrix per interval.  The full product comes back once the corrections since it add up
        to the store's size (drift stays at float64 rounding of that many updates)."""
        if self.device is None or self.size() == 0:
            return None
        from ...ops import als as als_ops
        with self._gram_lock:
            with self._dev_lock, self._lock.write():
                g = self._gram
                full = g is None or self._gram_corrected > max(self._n_rows, 1)
                if full:
                    self._gram_drop()
                    # writers wait for the mirror refresh and the product's launch; rows they
                    # write after it are corrections
                    mat = self.device_view()[0]
                    g = als_ops.gramian(mat).double() if mat.is_cuda else \
                        mat.t().double().matmul(mat.double())
                    if g.is_cuda:
                        # the mirror's rows are read before a later refresh rewrites them
                        torch.cuda.current_stream(g.device).synchronize()
                    self._gram = g
                    self._gram_corrected = 0
                    self.gram_stats["full"] += 1
                    return g.clone()
                sub, add = self._gram_sub, self._gram_add
                self._gram_sub, self._gram_add = [], []
                self._gram_corrected += self._gram_pending
                self._gram_pending = 0
            # (the lock-free part: only this method touches _gram's values)
            dev = g.device
            for mats, sign in ((add, 1.0), (sub, -1.0)):
                if mats:
                    m = torch.from_numpy(np.concatenate(mats)).to(dev, torch.float64)
                    g.addmm_(m.t(), m, alpha=sign)
            self.gram_stats["incremental"] += 1
            return g.clone()

    # ---------------------------------------------------------------- device mirror
    def device_view(self):
        """(matrix fp32 [n, k], valid bool [n], norms fp32 [n]) on the device, refreshed (the
        matrix is a view of rows ``ld`` floats apart)."""
        mat, valid, norm = self._device_refresh()
        return mat[:, :self.k], valid, norm

    def device_rows(self):
        """(padded device matrix fp32 [n, ld], ld), refreshed: what the serving scan reads."""
        mat, _, _ = self._device_refresh()
        return mat, self.ld

    def _upload_full(self, cap: int) -> torch.Tensor:
        if self.ld == self.k:
            return torch.from_numpy(self._host[:cap]).to(self.device, copy=True)
        dev = torch.zeros((cap, self.ld), dtype=torch.float32, device=self.device)
        step = 1 << 20       # bounded staging for the strided copy
        for lo in range(0, cap, step):
            hi = min(cap, lo + step)
            dev[lo:hi, :self.k] = torch.from_numpy(self._host[lo:hi]).to(self.device)
        return dev

    def _device_refresh(self):
        if self.device is None:
            raise RuntimeError("no device mirror")
        with self._dev_lock:
            with self._lock.read():
                n = self._n_rows
                need_full = (self._dev is None or self._dirty_all or
                             self._dev.shape[0] < max(n, 1))
                if need_full:
                    # the device copy tracks the used rows plus 1/8 headroom, not the host's
                    # power-of-two capacity (a 20M-row store would otherwise hold 33.5M rows
                    # of HBM); the read lock keeps writers out during the synchronous copies
                    cap = min(self._host.shape[0], max(1024, n + n // 8))
                    self._dev = None            # free the old mirror before the new one
                    self._dev = self._upload_full(cap)
                    self._dev_valid = torch.from_numpy(self._host_valid[:cap]).to(self.device,
                                                                                  copy=True)
                    self._dev_norm = self._dev.norm(dim=1)
                    self._dirty.clear()
                    self._dirty_all = False
                    dirty_rows = None
                elif self._dirty:
                    t_rf = time.perf_counter()
                    rows = np.fromiter(self._dirty, dtype=np.int64, count=len(self._dirty))
                    vals = torch.from_numpy(self._host[rows]).to(self.device, non_blocking=False)
                    if self.ld != self.k:
                        vals = torch.nn.functional.pad(vals, (0, self.ld - self.k))
                    valid = torch.from_numpy(self._host_valid[rows]).to(self.device)
                    self._dirty.clear()
                    dirty_rows = torch.from_numpy(rows).to(self.device)
                    self._dev.index_copy_(0, dirty_rows, vals)
                    self._dev_valid.index_copy_(0, dirty_rows, valid)
                    self._dev_norm.index_copy_(0, dirty_rows, vals.norm(dim=1))
                else:
                    dirty_rows = torch.empty(0, dtype=torch.int64, device=self.device)
                if self.partitioner is not None:
                    if need_full or self._dev_part is None:
                        self._dev_part = self.partitioner(self._dev[:, :self.k])
                    elif dirty_rows is not None and dirty_rows.numel():
                        self._dev_part[dirty_rows] = self.partitioner(
                            self._dev[dirty_rows][:, :self.k])
                if dirty_rows is not None and dirty_rows.numel():
                    # (the last dirty-row refresh's host time: latency attribution)
                    self.last_refresh_ms = (time.perf_counter() - t_rf) * 1e3
            return self._dev[:n], self._dev_valid[:n], self._dev_norm[:n]

    def device_partitions(self) -> Optional[torch.Tensor]:
        if self._dev_part is None:
            return None
        return self._dev_part[:self._n_rows]

    def id_array(self) -> np.ndarray:
        """Every row's ID (None for free rows) as a numpy object array -- a view of the
        store's own row -> ID array, no copy: candidate IDs are then one fancy index
        (``id_array()[rows]``), not a Python list built per request.  Use it at once (a row
        freed and reused later shows its new ID)."""
        with self._lock.read():
            return self._ids[:self._n_rows]

    def key_suffixes(self) -> np.ndarray:
        """int64 per row: the numeric suffix of the row's ID (-1: free row or no digits),
        from the native id -> row mirror (``ingest.RowMap.key_suffixes``)."""
        rm = self.synced_rowmap()
        with self._lock.read():
            return rm.key_suffixes(self._n_rows)

    def row_mask(self, ids, device=None):
        """Bool tensor over the store's rows: True at the rows of ``ids`` (on ``device``)."""
        import torch
        rows = self.host_rows(ids)
        m = torch.zeros(max(self._n_rows, 1), dtype=torch.bool)
        if rows:
            m[torch.as_tensor(rows, dtype=torch.int64)] = True
        return m.to(device) if device is not None else m

    def ids_of_rows(self, rows) -> List[Optional[str]]:
        ids = self._ids
        n = self._n_rows
        return [ids[r] if 0 <= r < n else None for r in rows]

    def host_rows(self, ids: Iterable[str]) -> List[int]:
        idx = self._index
        return [r for r in (idx.get(i) for i in ids) if r is not None]

    def __repr__(self):
        return "FeatureVectors[size:%d]" % self.size()
