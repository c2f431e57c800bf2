"""Batched top-N over a GPU-resident item matrix (the ALS serving hot path).

:class:`ItemIndex` orders the serving model's items by LSH bucket, so a query's candidate
buckets are contiguous position ranges; :meth:`ItemIndex.scan` scores up to 16 queries per
launch of the fused HIP kernel ``oryx_topn_scan2`` (``csrc/kernels/topn.hip``: fp32 MFMA
scoring, cosine scale, candidate-bucket mask, excluded items and a per-wave LDS top-KL in the
epilogue) and merges the per-wave candidates with one small ``topk``.  Only the union of the
batch's candidate ranges is read, so an LSH sample rate of 0.3 reads ~30% of the matrix for a
single query (the reference scans candidate partitions on a thread pool:
``[serving-app]/als/model/ALSServingModel.java:289-335``, ``LocalitySensitiveHash.java:156-177``,
bounded heaps ``TopNConsumer.java:55-74``).

One device copy of the items: on the store's own GPU the index holds only a bucket-sorted
permutation (position -> store row) and the kernel reads the store's padded device mirror in
place, so value updates cost the index nothing and new items / bucket moves re-sort a
permutation, not the matrix.  Shards of an item-sharded index on other GPUs
(:class:`ShardedItemIndex`) keep their own share of the rows.

Request depth: ``how_many`` up to 64 per (wave, query) list in the batched launch, 256 / 1024
in deeper single-pass launches, and beyond that repeated passes that exclude what earlier
passes returned -- every depth is exact.
"""

from __future__ import annotations

import collections
import ctypes
import itertools
import os
import threading
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import native

__all__ = ["ItemIndex", "ShardedItemIndex", "TopNQuery", "MAX_BATCH", "MAX_HOW_MANY",
           "kernel_ok"]

MAX_BATCH = 16          # queries per kernel launch
MAX_HOW_MANY = 64       # candidates each wave keeps per query in the batched launch
_EMPTY_I64 = np.zeros(0, dtype=np.int64)
BF16_POOL = 64          # candidates the bf16 scan re-ranks exactly per query
BF16_MAX_HOW_MANY = 32  # deeper requests scan in fp32


def _upload(arrays, device) -> List[torch.Tensor]:
    """Host arrays to the device in ONE copy: packed back to back (16-byte aligned) into a
    pinned staging buffer, then viewed per array on the device."""
    offs, total = [], 0
    for a in arrays:
        offs.append(total)
        total += -(-a.nbytes // 16) * 16
    host = torch.empty(max(total, 16), dtype=torch.uint8, pin_memory=True)
    hb = host.numpy()
    for a, o in zip(arrays, offs):
        hb[o:o + a.nbytes] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
    dev = host.to(device, non_blocking=True)
    out = []
    for a, o in zip(arrays, offs):
        t = dev[o:o + a.nbytes].view(_TORCH_DTYPE[a.dtype.str])
        out.append(t.view(a.shape))
    return out


_TORCH_DTYPE = {np.dtype(np.float32).str: torch.float32, np.dtype(np.int64).str: torch.int64,
                np.dtype(np.int32).str: torch.int32, np.dtype(np.uint32).str: torch.int32}


# fp32 scan bytes (rows x padded rank x 4) from which the bf16 scan is used
BF16_MIN_BYTES = int(os.environ.get("ORYX_TOPN_BF16_MIN_BYTES", str(1 << 30)))


def _bf16_default() -> bool:
    """The bf16 scan is on unless ORYX_TOPN_BF16=0 (it is exact: certified or rescanned)."""
    return os.environ.get("ORYX_TOPN_BF16", "1") != "0"
_KLS = (64, 256, 1024)  # per-(wave, query) list lengths the kernel is built for
_KPS = (16, 32, 48, 64, 80, 96, 112, 128, 160, 192, 256)


def _kp(k: int) -> Optional[int]:
    for v in _KPS:
        if v >= k:
            return v
    return None


def row_pad_for(k: int) -> int:
    """Row stride padding for a feature store the scan reads in place (stride = kp)."""
    return _kp(k) or 1


def kernel_ok(device, k: int) -> bool:
    return (device is not None and device.type == "cuda" and _kp(k) is not None
            and native.kernels_available())


@dataclass
class TopNQuery:
    target: np.ndarray                  # [k] fp32
    how_many: int
    cosine: bool = False
    candidates: Optional[np.ndarray] = None   # LSH bucket ids to scan (None: all)
    exclude_rows: Optional[Sequence[int]] = None   # store rows never returned


class ItemIndex:
    """Bucket-sorted view of an item store (see module docstring).  ``shard`` = (d, N) keeps
    only the store rows r with r % N == d, on ``device`` (item sharding over several GPUs:
    :class:`ShardedItemIndex`)."""

    def __init__(self, store, num_buckets: int, device=None, shard: Tuple[int, int] = (0, 1),
                 managed: bool = False, bf16: Optional[bool] = None):
        self.store = store
        # managed: a ShardedItemIndex takes the store's changes once and hands every shard
        # its share; the shard never consumes the store's dirty set itself
        self._managed = bool(managed)
        self._token = None if managed else store.register_index_consumer()
        self.k = store.k
        self.kp = _kp(self.k)
        self.device = torch.device(device) if device is not None else store.device
        self.shard = (int(shard[0]), int(shard[1]))
        self.num_buckets = max(1, int(num_buckets))
        # bucket id num_buckets marks a dead position (a row that moved or left since the
        # last sort): no query's bucket mask ever holds it
        self.dead_bucket = self.num_buckets
        self.words = (self.num_buckets + 1 + 31) // 32
        # borrowed: the kernel reads the store's device mirror in place (same GPU, rows kp
        # floats apart); otherwise this index keeps its own rows
        self.borrowed = (self.shard[1] == 1 and store.device is not None and
                         self.device == torch.device(store.device) and
                         getattr(store, "ld", self.k) == self.kp)
        self._lock = threading.Lock()
        self.version = -1
        self.Ys = None          # owned mode: fp32 [n][kp] sorted by bucket
        self.perm = None        # borrowed mode: int32 [n] position -> store row
        self.bucket_of = None   # int32 [n]
        self.pos_of_row = None  # int64 [store capacity] -> position or -1 (device)
        self.row_of_pos = None  # int64 [n] (device) and host copy
        self.row_of_pos_h = None
        self.bucket_start = None   # host int64 [num_buckets + 1]
        # positions [0, n_main) are sorted by bucket; [n_main, n) is the delta segment: rows
        # added or re-bucketed since that sort, appended as they come and scanned by every
        # query (the kernel's bucket mask filters them); n_dead positions are dead
        self.n = 0
        self.n_main = 0
        self.n_dead = 0
        self.cap = 0
        self.rebuilds = 0
        self.incremental = 0       # refreshes absorbed without a re-sort
        # (wall-clock start, ms, what, rows) of each refresh / bf16 conversion that did work:
        # what a latency record lines its slow requests up with (bench_traffic.py)
        self.event_log = collections.deque(maxlen=512)
        self.delta_added = 0       # rows appended to the delta segment, ever
        self._built = False
        # bf16 scan with exact fp32 re-rank of a certified candidate pool (_launch_bf16):
        # dot-product queries of <= BF16_MAX_HOW_MANY on the store's own GPU
        self.bf16 = (bf16 if bf16 is not None else _bf16_default()) and self.borrowed and \
            self.kp is not None
        self.kpb = -(-self.kp // 32) * 32 if self.kp else None
        self._yb = None            # bf16 [rows, kpb] mirror of the store's rows (store order)
        self._yb_key = None        # (store version, rows) the mirror was converted at
        self._yb_token = store.register_index_consumer() if self.bf16 else None
        self._max_norm = 0.0       # >= every mirrored row's L2 norm
        self.bf16_certified = 0
        self.bf16_fallbacks = 0

    # ------------------------------------------------------------------ maintenance
    def refresh(self, state: Optional[Tuple[int, Optional[np.ndarray]]] = None) -> None:
        """Bring the index up to the store.  ``state`` = (version, changed rows) taken by the
        owning :class:`ShardedItemIndex`; otherwise this index takes them itself -- version and
        rows together, before the device view, so no write can fall between them."""
        st = self.store
        if state is None:
            if self._managed or (self.version == st.version and self._built):
                return
        with self._lock:
            if state is None:
                if self.version == st.version and self._built:
                    return
                state = st.take_index_state(self._token)
            t_wall, t0 = time.time(), time.perf_counter()
            ver, dirty = state
            mat, valid, _ = st.device_view()
            parts = st.device_partitions()
            t1 = time.perf_counter()
            what = "incremental"
            if not self._built or dirty is None or not self._update_in_place(mat, valid, parts,
                                                                             dirty):
                self._rebuild(mat, valid, parts)
                what = "rebuild"
            self.version = ver
            t2 = time.perf_counter()
            self.event_log.append((t_wall, (t2 - t0) * 1e3, what,
                                   -1 if dirty is None else len(dirty),
                                   {"device_view_ms": round((t1 - t0) * 1e3, 2),
                                    "update_ms": round((t2 - t1) * 1e3, 2)}))

    def _buckets(self, parts, rows):
        if parts is None:
            return torch.zeros(rows.numel(), dtype=torch.int64, device=rows.device)
        return parts[rows].to(torch.int64)

    def _rebuild(self, mat, valid, parts) -> None:
        """Re-sort every live row by bucket; room for a delta segment of max(64K, n / 16)
        positions behind the sorted ones."""
        dev = self.device
        rows = torch.nonzero(valid, as_tuple=False).flatten()
        d, nsh = self.shard
        if nsh > 1:
            rows = rows[rows % nsh == d]
        b = self._buckets(parts, rows)
        order = torch.argsort(b, stable=True)
        rows = rows[order]
        b = b[order]
        n = int(rows.numel())
        cap = n + max(1 << 16, n // 16)
        if self.borrowed:
            perm = torch.zeros(cap, dtype=torch.int32, device=dev)
            perm[:n] = rows.to(torch.int32)
            self.perm = perm
            self.Ys = None
        else:
            ys = torch.zeros((cap, self.kp), dtype=torch.float32, device=dev)
            # gathered in slices of 1M rows: a whole-matrix mat[rows] temporary would add
            # another full copy of the item factors to the peak HBM of a rebuild
            step = 1 << 20
            for lo in range(0, n, step):
                hi = min(n, lo + step)
                ys[lo:hi, :self.k] = mat[rows[lo:hi]].to(dev)
            self.Ys = ys
            self.perm = None
        rows = rows.to(dev)
        b = b.to(dev)
        bucket_of = torch.full((cap,), self.dead_bucket, dtype=torch.int32, device=dev)
        bucket_of[:n] = b.to(torch.int32)
        self.bucket_of = bucket_of
        pos = torch.full((mat.shape[0],), -1, dtype=torch.int64, device=dev)
        if n:
            pos[rows] = torch.arange(n, device=dev)
        self.pos_of_row = pos
        self.pos_of_row_h = pos.cpu().numpy()
        rop = torch.full((cap,), -1, dtype=torch.int64, device=dev)
        rop[:n] = rows
        self.row_of_pos = rop
        self.row_of_pos_h = rop.cpu().numpy()
        counts = torch.bincount(b, minlength=self.num_buckets).cpu().numpy()
        self.bucket_start = np.zeros(self.num_buckets + 1, dtype=np.int64)
        np.cumsum(counts[:self.num_buckets], out=self.bucket_start[1:])
        self.n = self.n_main = n
        self.n_dead = 0
        self.cap = cap
        self.rebuilds += 1
        self._built = True

    def _grow_row_maps(self, rows: int) -> None:
        """The store grew: extend the row -> position maps (device and host) to ``rows``."""
        old = self.pos_of_row.numel()
        if rows <= old:
            return
        rows = max(rows, old + old // 2)
        pos = torch.full((rows,), -1, dtype=torch.int64, device=self.device)
        pos[:old] = self.pos_of_row
        self.pos_of_row = pos
        ph = np.full(rows, -1, dtype=np.int64)
        ph[:old] = self.pos_of_row_h
        self.pos_of_row_h = ph

    def _update_in_place(self, mat, valid, parts, dirty: np.ndarray) -> bool:
        """Absorb the changed rows without a re-sort (ALSServingModel.setItemVector moves one
        item between LSH partitions, ALSServingModel.java:161-183): a row that stays in its
        bucket needs nothing when the kernel reads the store's mirror (a row copy otherwise);
        a row that left its bucket, or left the store, kills its position (bucket -> dead);
        a new or moved row is appended to the delta segment.  Returns False when a re-sort is
        due instead: many changes at once, the delta segment full, or many dead positions."""
        if len(dirty) == 0:
            return True
        if len(dirty) > max(4096, self.n_main // 16):
            return False
        dev = self.device
        d, nsh = self.shard
        dirty = np.asarray(dirty, dtype=np.int64)
        if nsh > 1:
            dirty = dirty[dirty % nsh == d]
            if len(dirty) == 0:
                return True
        self._grow_row_maps(int(mat.shape[0]))
        src = torch.from_numpy(dirty).to(mat.device)
        rows = src.to(dev)
        pos = self.pos_of_row[rows]
        ok = valid[src].to(dev)
        nb = self._buckets(parts, src).to(dev)
        cur = torch.where(pos >= 0, self.bucket_of[pos.clamp(min=0)].to(torch.int64),
                          torch.full_like(pos, -1))
        stay = (pos >= 0) & ok & (nb == cur)
        kill = (pos >= 0) & ~stay
        add = ok & ~stay
        n_kill, n_add = (int(v) for v in torch.stack([kill.sum(), add.sum()]).tolist())
        if self.n + n_add > self.cap or \
                self.n_dead + n_kill > max(1 << 14, self.n_main // 8):
            return False
        if not self.borrowed and bool(stay.any()):
            self.Ys[pos[stay], :self.k] = mat[src[stay.to(src.device)]].to(dev)
        if n_kill:
            kp_ = pos[kill]
            self.bucket_of[kp_] = self.dead_bucket
            self.row_of_pos[kp_] = -1
            self.pos_of_row[rows[kill]] = -1
            kh = kp_.cpu().numpy()
            self.row_of_pos_h[kh] = -1
            self.pos_of_row_h[rows[kill].cpu().numpy()] = -1
            self.n_dead += n_kill
        if n_add:
            q = torch.arange(self.n, self.n + n_add, dtype=torch.int64, device=dev)
            ra = rows[add]
            if self.borrowed:
                self.perm[q] = ra.to(torch.int32)
            else:
                self.Ys[q, :self.k] = mat[src[add.to(src.device)]].to(dev)
            self.bucket_of[q] = nb[add].to(torch.int32)
            self.row_of_pos[q] = ra
            self.pos_of_row[ra] = q
            rh = ra.cpu().numpy()
            self.row_of_pos_h[self.n:self.n + n_add] = rh
            self.pos_of_row_h[rh] = np.arange(self.n, self.n + n_add, dtype=np.int64)
            self.n += n_add
            self.delta_added += n_add
        self.incremental += 1
        return True

    # ------------------------------------------------------------------ queries
    def scan(self, queries: Sequence[TopNQuery]) -> List[Tuple[np.ndarray, np.ndarray]]:
        """Per query: (store rows, scores) of the best ``how_many``, descending (exact for
        any depth)."""
        self.refresh()
        out: List[Optional[Tuple[np.ndarray, np.ndarray]]] = [None] * len(queries)
        deep = [j for j, q in enumerate(queries) if q.how_many > _KLS[-1]]
        for j in deep:
            out[j] = self._scan_deep(queries[j])
        rest = [j for j in range(len(queries)) if out[j] is None]
        # one launch per (cosine, list length) group, as many queries as its LDS holds
        groups = {}
        for j in rest:
            q = queries[j]
            kl = next(v for v in _KLS if v >= q.how_many)
            groups.setdefault((bool(q.cosine), kl), []).append(j)
        for (cos, kl), idx in sorted(groups.items()):
            per = min(MAX_BATCH, int(native.require_kernels().oryx_topn_max_queries(kl)))
            for lo in range(0, len(idx), per):
                part = idx[lo:lo + per]
                for j, r in zip(part, self._launch([queries[j] for j in part], cos, kl)):
                    out[j] = r
        return out

    def scan_async(self, queries: Sequence[TopNQuery]):
        """Launch :meth:`scan` and return ``finish()`` -> its results.  A batch that is one
        fp32 launch (the common micro-batch) only queues its work here: the kernel, the
        merge and the copy back into pinned memory run while the caller prepares the next
        batch, and ``finish()`` waits for them; anything else completes inside this call."""
        self.refresh()
        if queries and self.n > 0 and len(queries) <= MAX_BATCH:
            cos = bool(queries[0].cosine)
            kl = next((v for v in _KLS if v >= max(q.how_many for q in queries)), None)
            if kl is not None and all(bool(q.cosine) == cos for q in queries) and \
                    len(queries) <= int(native.require_kernels().oryx_topn_max_queries(kl)) \
                    and not self._bf16_queries(queries, cos, kl):
                # the scan groups by list length: one group only when every query maps to kl
                if all(next(v for v in _KLS if v >= q.how_many) == kl for q in queries):
                    return self._launch_fp32(queries, cos, kl, asynchronous=True)
        out = self.scan(queries)
        return lambda: out

    def _scan_deep(self, q: TopNQuery) -> Tuple[np.ndarray, np.ndarray]:
        """``how_many`` beyond one list: passes of the deepest list, each excluding the rows
        the previous passes returned (scores arrive in descending order across passes)."""
        kl = _KLS[-1]
        rows_all, sc_all = [], []
        excl = list(q.exclude_rows) if q.exclude_rows is not None else []
        left = q.how_many
        while left > 0:
            take = min(left, kl)
            sub = TopNQuery(q.target, take, q.cosine, q.candidates,
                            excl + [int(r) for part in rows_all for r in part])
            r, v = self._launch([sub], bool(q.cosine), kl)[0]
            rows_all.append(r)
            sc_all.append(v)
            left -= take
            if len(r) < take:
                break           # the candidates ran out
        return (np.concatenate(rows_all) if rows_all else np.zeros(0, dtype=np.int64),
                np.concatenate(sc_all) if sc_all else np.zeros(0, dtype=np.float32))

    def _matrix(self):
        """(device matrix pointer owner, row stride) the kernel reads, and the permutation."""
        if self.borrowed:
            # device_rows() applies every store write so far; writes that landed after this
            # index's last refresh may have removed, reused or re-bucketed rows the
            # permutation still names: bring the permutation up to the same version first
            # (anything later still is filtered from the results in _launch)
            if self.version != self.store.version:
                self.refresh()
            mat, ld = self.store.device_rows()
            return mat, ld, self.perm
        return self.Ys, self.kp, None

    def _bf16_queries(self, qs: Sequence[TopNQuery], cosine: bool, kl: int) -> List[int]:
        """Positions of the queries the bf16 scan takes.  It halves the bytes a scan reads;
        below BF16_MIN_BYTES of fp32 rows the scan is launch-bound anyway and the exact
        re-rank's extra ops cost more than it saves."""
        big = self.n * (self.kp or 0) * 4 >= BF16_MIN_BYTES
        if not (self.bf16 and big and not cosine and kl == MAX_HOW_MANY and self.n > 0):
            return []
        return [j for j, q in enumerate(qs) if q.how_many <= BF16_MAX_HOW_MANY]

    def _launch(self, qs: Sequence[TopNQuery], cosine: bool, kl: int = MAX_HOW_MANY):
        shallow = self._bf16_queries(qs, cosine, kl)
        if not shallow:
            return self._launch_fp32(qs, cosine, kl)
        out: List[Optional[Tuple[np.ndarray, np.ndarray]]] = [None] * len(qs)
        res, failed = self._launch_bf16([qs[j] for j in shallow])
        for j, r in zip(shallow, res):
            out[j] = r
        rest = [shallow[f] for f in failed] + [j for j in range(len(qs)) if j not in shallow]
        if rest:
            for j, r in zip(rest, self._launch_fp32([qs[j] for j in rest], cosine, kl)):
                out[j] = r
        return out

    # ------------------------------------------------------------------ bf16 scan
    def _bf16_rows(self) -> torch.Tensor:
        """The bf16 mirror of the store's device rows, brought up to date: the rows written
        since the last call are converted (all of them after a reallocation), and the norm
        bound follows them.  The changed rows are taken before the device rows are read, so
        a write landing in between is converted again next time, never missed."""
        st = self.store
        if self._yb is not None and self._yb_key is not None and \
                self._yb_key[0] == st.version and self._yb_key[1] == self._yb.shape[0]:
            return self._yb            # nothing written since the last conversion
        t_wall, t0 = time.time(), time.perf_counter()
        ver, dirty = st.take_index_state(self._yb_token)
        mat, _ = st.device_rows()
        rows = mat.shape[0]
        yb = self._yb
        k = self.k
        _, _, norms = st.device_view()
        if yb is None or yb.shape[0] != rows or dirty is None or len(dirty) > rows // 8:
            if yb is None or yb.shape[0] != rows:
                yb = torch.zeros((rows, self.kpb), dtype=torch.bfloat16, device=mat.device)
            step = 1 << 20
            for lo in range(0, rows, step):
                hi = min(rows, lo + step)
                yb[lo:hi, :k] = mat[lo:hi, :k].to(torch.bfloat16)
            self._max_norm = float(norms[:rows].max()) if rows else 0.0
        elif len(dirty):
            d = torch.from_numpy(np.asarray(dirty, dtype=np.int64)).to(mat.device)
            d = d[d < rows]
            if d.numel():
                yb[d, :k] = mat[d, :k].to(torch.bfloat16)
                self._max_norm = max(self._max_norm, float(norms[d].max()))
        self._yb = yb
        self._yb_key = (ver, rows)
        self.event_log.append((t_wall, (time.perf_counter() - t0) * 1e3, "bf16",
                               -1 if dirty is None else len(dirty)))
        return yb

    def _launch_bf16(self, qs: Sequence[TopNQuery]):
        """Dot-product queries through the bf16 scan: the kernel keeps each query's best
        BF16_POOL candidates by bf16 score (items and query rounded to bf16, fp32
        accumulation); those are re-scored exactly in fp32 and the query's top how_many
        taken from them.  The pool is certified to hold the exact answer when every item
        outside it scores below the pool's how_many-th exact score: an item's bf16 score is
        within E = (2u + u^2 + 2k 2^-24) |x| max|y| of its fp32 score (u = 2^-8, the bf16
        rounding of both operands; Cauchy-Schwarz), so outside items score at most
        (pool's last bf16 score) + E.  Uncertified queries are returned in ``failed`` (the
        caller rescans them in fp32).  Returns (results, failed indices)."""
        dev = self.device
        lib = native.require_kernels()
        nq = len(qs)
        kl = MAX_HOW_MANY
        prep = self._prep(qs, self.kpb)
        if prep is None:
            empty = (np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.float32))
            return [empty for _ in qs], []
        Qd, rs_d, t0_d, bits_d, ptr_d, ex_d, n_ranges, n_tiles = prep
        mat, ld, perm = self._matrix()
        yb = self._bf16_rows()          # covers every row the permutation names
        waves = int(lib.oryx_topn_waves_kl(n_tiles, kl))
        o_sc = torch.empty((waves, nq, kl), dtype=torch.float32, device=dev)
        o_rw = torch.empty((waves, nq, kl), dtype=torch.int32, device=dev)
        rc = lib.oryx_topn_scan3(
            mat.data_ptr(), yb.data_ptr(), self.kpb,
            perm.data_ptr() if perm is not None else None, int(ld), Qd.data_ptr(), self.kpb,
            nq, 0, kl, self.bucket_of.data_ptr() if bits_d is not None else None,
            bits_d.data_ptr() if bits_d is not None else None, self.words, rs_d.data_ptr(),
            t0_d.data_ptr(), n_ranges, n_tiles,
            ptr_d.data_ptr() if ptr_d is not None else None,
            ex_d.data_ptr() if ex_d is not None else None,
            o_sc.data_ptr(), o_rw.data_ptr(), native.stream_ptr(dev))
        native.check(rc, "oryx_topn_scan3")
        pool = min(BF16_POOL, waves * kl)
        sc = o_sc.permute(1, 0, 2).reshape(nq, -1)
        rw = o_rw.permute(1, 0, 2).reshape(nq, -1)
        v, i = torch.topk(sc, pool, dim=1)                 # bf16 scores, descending
        pos = torch.gather(rw, 1, i)
        # exact fp32 scores of the pool: gather its rows, one batched dot with the queries
        # (invalid slots -- position -1 -- score row 0 and are dropped on the host)
        rows = torch.index_select(self.perm, 0, pos.clamp(min=0).flatten())
        fp = torch.index_select(mat, 0, rows).view(nq, pool, ld)
        # (ld <= kpb; both operands' columns past k are zero)
        exact = torch.bmm(fp, Qd[:nq, :ld].unsqueeze(2)).squeeze(2)
        h = torch.cat([v.view(torch.int32), pos, exact.view(torch.int32)], 1).cpu().numpy()
        v_h = h[:, :pool].view(np.float32)
        pos_h = h[:, pool:2 * pool]
        ex_h = h[:, 2 * pool:].view(np.float32).copy()
        okm = np.isfinite(v_h) & (pos_h >= 0)
        ex_h[~okm] = -np.inf
        u = 2.0 ** -8
        c = 2 * u + u * u + 2 * self.k * 2.0 ** -24
        out: List[Optional[Tuple[np.ndarray, np.ndarray]]] = [None] * nq
        failed = []
        for j, q in enumerate(qs):
            hm = q.how_many
            order = np.argsort(-ex_h[j], kind="stable")[:hm]
            tau = ex_h[j, order[-1]] if len(order) == hm else -np.inf
            x = np.asarray(q.target, dtype=np.float64)[:self.k]
            bound = c * float(np.sqrt(x @ x)) * self._max_norm
            if int(okm[j].sum()) < pool or (np.isfinite(tau) and v_h[j, -1] + bound < tau):
                self.bf16_certified += 1
                out[j] = self._finish_one(ex_h[j, order], pos_h[j, order])
            else:
                self.bf16_fallbacks += 1
                failed.append(j)
        return out, failed

    def _finish_one(self, vj: np.ndarray, pj: np.ndarray,
                    row_of_pos: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        keep = np.isfinite(vj) & (pj >= 0)
        rows = (self.row_of_pos_h if row_of_pos is None else row_of_pos)[pj[keep]]
        vj = np.asarray(vj[keep], dtype=np.float32)
        if len(rows) and bool((rows < 0).any()):       # killed after the launch
            live = rows >= 0
            rows, vj = rows[live], vj[live]
        valid_h = self.store._host_valid if self.borrowed else None
        if valid_h is not None and len(rows):
            live = valid_h[np.minimum(rows, len(valid_h) - 1)] & (rows < len(valid_h))
            if not live.all():
                rows, vj = rows[live], vj[live]
        return rows, vj

    def _prep(self, qs: Sequence[TopNQuery], kp: int):
        """Launch inputs shared by the scans, packed by one native call
        (``oryx_topn_prep``) straight into a pinned staging buffer and sent in ONE
        host-to-device copy: queries [MAX_BATCH, kp], candidate ranges and their tile prefix,
        per-query bucket bitmaps, excluded positions.  Returns (Q, ranges, tile0, bits or
        None, ptr or None, excluded or None, n_ranges, n_tiles) device tensors / counts, or
        None when nothing is scanned."""
        nq, k = len(qs), self.k
        targets = np.empty((nq, k), dtype=np.float32)
        for j, q in enumerate(qs):
            targets[j] = np.asarray(q.target, dtype=np.float32)[:k]
        vp = ctypes.c_void_p
        cand_ptr = cand = cand_all = None
        if any(q.candidates is not None for q in qs):
            cl = [np.asarray(q.candidates, dtype=np.int64) if q.candidates is not None else
                  _EMPTY_I64 for q in qs]
            cand_ptr = np.zeros(nq + 1, dtype=np.int64)
            np.cumsum([len(c) for c in cl], out=cand_ptr[1:])
            cand = np.concatenate(cl) if cand_ptr[-1] else np.zeros(1, dtype=np.int64)
            cand_all = np.fromiter((q.candidates is None for q in qs), dtype=np.uint8, count=nq)
        ex_ptr = ex_rows = None
        if any(q.exclude_rows is not None and len(q.exclude_rows) for q in qs):
            el = [q.exclude_rows if q.exclude_rows is not None else () for q in qs]
            ex_ptr = np.zeros(nq + 1, dtype=np.int64)
            np.cumsum([len(e) for e in el], out=ex_ptr[1:])
            ex_rows = np.fromiter(itertools.chain.from_iterable(el), dtype=np.int64,
                                  count=int(ex_ptr[-1]))
        if cand_ptr is None and self.n_dead:
            # dead positions are masked by bucket: every query scans every (live) bucket
            cand_ptr = np.zeros(nq + 1, dtype=np.int64)
            cand = np.zeros(1, dtype=np.int64)
            cand_all = np.ones(nq, dtype=np.uint8)
        nb = self.num_buckets if cand_ptr is not None else 1
        cap = MAX_BATCH * kp * 4 + (nb + 1) * 16 + (nb + 2) * 8 + nq * self.words * 4 + \
            (nq + 1) * 4 + (len(ex_rows) + 1 if ex_rows is not None else 0) * 4 + 6 * 16
        host = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
        info = np.empty(9, dtype=np.int64)
        pos = self.pos_of_row_h
        rc = native.runtime().oryx_topn_prep(
            nq, k, kp, MAX_BATCH, targets.ctypes.data_as(vp),
            cand_ptr.ctypes.data_as(vp) if cand_ptr is not None else None,
            cand.ctypes.data_as(vp) if cand is not None else None,
            cand_all.ctypes.data_as(vp) if cand_all is not None else None,
            self.num_buckets, self.words, self.bucket_start.ctypes.data_as(vp),
            int(self.n_main),
            ex_ptr.ctypes.data_as(vp) if ex_ptr is not None else None,
            ex_rows.ctypes.data_as(vp) if ex_rows is not None else None,
            pos.ctypes.data_as(vp), len(pos), int(self.n_main), int(self.n),
            ctypes.c_void_p(host.data_ptr()), cap, info.ctypes.data_as(vp))
        if rc == 1:
            return None
        if rc != 0:
            raise RuntimeError("oryx_topn_prep: staging buffer too small")
        nr, n_tiles, o_rs, o_t0, o_bits, o_ptr, o_ex, used, n_ex = (int(v) for v in info)
        dev = host[:used].to(self.device, non_blocking=True)
        Qd = dev[:MAX_BATCH * kp * 4].view(torch.float32).view(MAX_BATCH, kp)
        rs_d = dev[o_rs:o_rs + nr * 16].view(torch.int64).view(nr, 2)
        t0_d = dev[o_t0:o_t0 + (nr + 1) * 8].view(torch.int64)
        bits_d = dev[o_bits:o_bits + nq * self.words * 4].view(torch.int32).view(
            nq, self.words) if o_bits >= 0 else None
        ptr_d = dev[o_ptr:o_ptr + (nq + 1) * 4].view(torch.int32) if o_ptr >= 0 else None
        ex_d = dev[o_ex:o_ex + n_ex * 4].view(torch.int32) if o_ex >= 0 else None
        return Qd, rs_d, t0_d, bits_d, ptr_d, ex_d, nr, n_tiles

    def _launch_fp32(self, qs: Sequence[TopNQuery], cosine: bool, kl: int = MAX_HOW_MANY,
                     asynchronous: bool = False):
        empty = (np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.float32))
        if self.n == 0 or not qs:
            out = [empty for _ in qs]
            return (lambda: out) if asynchronous else out
        dev = self.device
        lib = native.require_kernels()
        nq = len(qs)
        prep = self._prep(qs, self.kp)
        if prep is None:
            out = [empty for _ in qs]
            return (lambda: out) if asynchronous else out
        Qd, rs_d, t0_d, bits_d, ptr_d, ex_d, n_ranges, n_tiles = prep
        waves = int(lib.oryx_topn_waves_kl(n_tiles, kl))
        o_sc = torch.empty((waves, nq, kl), dtype=torch.float32, device=dev)
        o_rw = torch.empty((waves, nq, kl), dtype=torch.int32, device=dev)
        mat, ld, perm = self._matrix()
        rc = lib.oryx_topn_scan2(
            mat.data_ptr(), perm.data_ptr() if perm is not None else None, int(ld),
            Qd.data_ptr(), self.kp, nq, int(bool(cosine)), int(kl),
            self.bucket_of.data_ptr() if bits_d is not None else None,
            bits_d.data_ptr() if bits_d is not None else None, self.words, rs_d.data_ptr(),
            t0_d.data_ptr(), n_ranges, n_tiles,
            ptr_d.data_ptr() if ptr_d is not None else None,
            ex_d.data_ptr() if ex_d is not None else None,
            o_sc.data_ptr(), o_rw.data_ptr(), native.stream_ptr(dev))
        native.check(rc, "oryx_topn_scan2")
        m = max(q.how_many for q in qs)
        m = min(m, waves * kl)
        sc = o_sc.permute(1, 0, 2).reshape(nq, -1)
        rw = o_rw.permute(1, 0, 2).reshape(nq, -1)
        v, i = torch.topk(sc, m, dim=1)
        pos = torch.gather(rw, 1, i)
        hd = torch.cat([v.view(torch.int32), pos], 1)
        rop = self.row_of_pos_h          # the permutation these positions refer to

        def finish(h):
            v_h, pos_h = h[:, :m].view(np.float32), h[:, m:]
            # (a row removed between the permutation and the launch is never returned)
            return [self._finish_one(v_h[j, :q.how_many], pos_h[j, :q.how_many], rop)
                    for j, q in enumerate(qs)]
        if not asynchronous:
            return finish(hd.cpu().numpy())                               # one copy back
        host = torch.empty(hd.shape, dtype=torch.int32, pin_memory=True)
        host.copy_(hd, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))   # the launching stream, not the current device's

        def wait_and_finish():
            ev.synchronize()
            return finish(host.numpy())
        return wait_and_finish

    # ------------------------------------------------------------------ all scores
    def all_scores_device(self, target: np.ndarray, cosine: bool, candidates=None,
                          exclude_rows=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """(store rows int64, scores fp32) of EVERY candidate item (LSH buckets
        ``candidates``, minus ``exclude_rows``) as device tensors: what an arbitrary rescorer
        must see (``TopNConsumer`` applies the rescorer to each candidate).  One GEMV over the
        rows the index reads."""
        self.refresh()
        dev = self.device
        if self.n == 0:
            e = torch.zeros(0, dtype=torch.int64, device=dev)
            return e, torch.zeros(0, dtype=torch.float32, device=dev)
        mat, ld, perm = self._matrix()
        q = torch.zeros(self.kp, dtype=torch.float32, device=dev)
        q[:self.k] = torch.as_tensor(np.asarray(target, dtype=np.float32)[:self.k], device=dev)
        if self.borrowed:
            # one GEMV over the store's rows in store order (no permutation): rows are the
            # positions of the mask directly
            _, valid, norms = self.store.device_view()
            scores = mat.matmul(q)
            keep = valid.clone()
            if cosine:
                scores = torch.where(norms > 0, scores / norms, torch.zeros_like(scores))
            if candidates is not None:
                parts = self.store.device_partitions()
                if parts is not None:
                    cand = torch.zeros(self.num_buckets, dtype=torch.bool, device=dev)
                    cand[torch.as_tensor(np.asarray(candidates, dtype=np.int64),
                                         device=dev)] = True
                    keep &= cand[parts.long()]
            if exclude_rows is not None and len(exclude_rows):
                er = torch.as_tensor(np.asarray(exclude_rows, dtype=np.int64), device=dev)
                keep[er[er < keep.numel()]] = False
            keep &= torch.isfinite(scores)
            rows = torch.nonzero(keep).flatten()
            return rows, scores[rows]
        scores = mat[:self.n].matmul(q)
        if cosine:
            nrm = mat[:self.n].norm(dim=1)
            scores = torch.where(nrm > 0, scores / nrm, torch.zeros_like(scores))
        keep = torch.isfinite(scores) & (self.bucket_of[:self.n] != self.dead_bucket)
        if candidates is not None:
            cand = torch.zeros(self.num_buckets + 1, dtype=torch.bool, device=dev)
            cand[torch.as_tensor(np.asarray(candidates, dtype=np.int64), device=dev)] = True
            keep &= cand[self.bucket_of[:self.n].long()]
        if exclude_rows is not None and len(exclude_rows):
            er = torch.as_tensor(np.asarray(exclude_rows, dtype=np.int64), device=dev)
            er = er[er < self.pos_of_row.numel()]
            p = self.pos_of_row[er]
            keep[p[p >= 0]] = False
        pos = torch.nonzero(keep).flatten()
        return self.row_of_pos[pos], scores[pos]

    def all_scores(self, target: np.ndarray, cosine: bool, candidates=None,
                   exclude_rows=None) -> Tuple[np.ndarray, np.ndarray]:
        """:meth:`all_scores_device` on the host: (store rows, scores) numpy arrays."""
        rows, sc = self.all_scores_device(target, cosine, candidates, exclude_rows)
        if rows.device.type == "cuda" and rows.numel():
            # pinned staging: one DMA each
            rh = torch.empty(rows.numel(), dtype=torch.int64, pin_memory=True)
            sh = torch.empty(sc.numel(), dtype=torch.float32, pin_memory=True)
            rh.copy_(rows)
            sh.copy_(sc)
            return rh.numpy(), sh.numpy()
        return rows.cpu().numpy(), sc.cpu().numpy()


class ShardedItemIndex:
    """Item-sharded top-N over several GPUs: store row r lives in shard
    r % N on ``devices[r % N]``; a batch of queries is scanned by every shard at once (one
    host thread per device, each launching its own fused scan) and the per-shard candidates
    are merged on the host.  Same interface as :class:`ItemIndex` (``refresh`` / ``scan``)."""

    def __init__(self, store, num_buckets: int, devices: Sequence):
        import concurrent.futures
        self.store = store
        self.shards = [ItemIndex(store, num_buckets, device=dv, shard=(j, len(devices)),
                                 managed=True)
                       for j, dv in enumerate(devices)]
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=len(devices),
                                                           thread_name_prefix="oryx-topn")
        self._lock = threading.Lock()
        self.version = -1
        self._token = store.register_index_consumer()

    @property
    def n(self) -> int:
        return sum(sh.n for sh in self.shards)

    def refresh(self) -> None:
        """Take the store's changes ONCE and give every shard the same (version, rows): each
        keeps the rows r % N == d of them (a shard consuming the shared dirty set itself would
        leave the others with nothing and stale rows)."""
        st = self.store
        if self.version == st.version and all(sh.Ys is not None for sh in self.shards):
            return
        with self._lock:
            if self.version == st.version and all(sh.Ys is not None for sh in self.shards):
                return
            state = st.take_index_state(self._token)
            for f in [self._pool.submit(sh.refresh, state) for sh in self.shards]:
                f.result()
            self.version = state[0]

    def scan_async(self, queries: Sequence[TopNQuery]):
        out = self.scan(queries)
        return lambda: out

    def scan(self, queries: Sequence[TopNQuery]) -> List[Tuple[np.ndarray, np.ndarray]]:
        self.refresh()
        parts = [f.result() for f in [self._pool.submit(sh.scan, queries)
                                       for sh in self.shards]]
        out = []
        for j, q in enumerate(queries):
            rows = np.concatenate([p[j][0] for p in parts])
            sc = np.concatenate([p[j][1] for p in parts])
            # descending by score, ties by row (the single-index order)
            o = np.lexsort((rows, -sc))[:q.how_many]
            out.append((rows[o], sc[o]))
        return out

    def all_scores_device(self, target, cosine: bool, candidates=None, exclude_rows=None):
        r, s = self.all_scores(target, cosine, candidates, exclude_rows)
        dev = self.shards[0].device
        return torch.from_numpy(r).to(dev), torch.from_numpy(s).to(dev)

    def all_scores(self, target, cosine: bool, candidates=None, exclude_rows=None):
        self.refresh()
        parts = [f.result() for f in [self._pool.submit(sh.all_scores, target, cosine,
                                                        candidates, exclude_rows)
                                       for sh in self.shards]]
        return (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))

    def close(self) -> None:
        self._pool.shutdown(wait=False)

