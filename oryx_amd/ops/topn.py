"""Batched top-N over a GPU-resident item matrix (the ALS serving hot path).

:class:`ItemIndex` keeps the serving model's item vectors on the device as fp32 rows sorted by
LSH bucket, so a query's candidate buckets are contiguous row ranges; :meth:`ItemIndex.scan`
scores up to 16 queries per launch of the fused HIP kernel ``oryx_topn_scan``
(``csrc/kernels/topn.hip``: fp32 MFMA scoring, cosine scale, candidate-bucket mask, excluded
items and a per-wave LDS top-64 in the epilogue) and merges the per-wave candidates with one
small ``topk``.  Only the union of the batch's candidate ranges is read, so an LSH sample rate
of 0.3 reads ~30% of the matrix for a single query (the reference scans candidate partitions
on a thread pool: ``[serving-app]/als/model/ALSServingModel.java:289-335``,
``LocalitySensitiveHash.java:156-177``, bounded heaps ``TopNConsumer.java:55-74``).

The index follows the item store (``FeatureVectors``) incrementally: changed rows whose LSH
bucket is unchanged are rewritten in place; new rows, removals and bucket moves trigger a
re-sort (one gather of the matrix on the device).
"""

from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import native

__all__ = ["ItemIndex", "ShardedItemIndex", "TopNQuery", "MAX_BATCH", "MAX_HOW_MANY",
           "kernel_ok"]

MAX_BATCH = 16          # queries per kernel launch
MAX_HOW_MANY = 64       # candidates each wave keeps per query
_KPS = (16, 32, 48, 64, 80, 96, 112, 128, 160, 192, 256)


def _kp(k: int) -> Optional[int]:
    for v in _KPS:
        if v >= k:
            return v
    return None


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
    """Bucket-sorted device copy of an item store (see module docstring).  ``shard`` =
    (d, N) keeps only the store rows r with r % N == d, on ``device`` (item sharding over
    several GPUs: :class:`ShardedItemIndex`)."""

    def __init__(self, store, num_buckets: int, device=None, shard: Tuple[int, int] = (0, 1),
                 managed: bool = False):
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
        self.words = (self.num_buckets + 31) // 32
        self._lock = threading.Lock()
        self.version = -1
        self.Ys = None          # fp32 [n][kp] sorted by bucket
        self.inv_norm = None    # fp32 [n]
        self.bucket_of = None   # int32 [n]
        self.pos_of_row = None  # int64 [store capacity] -> position or -1 (device)
        self.row_of_pos = None  # int64 [n] (device) and host copy
        self.row_of_pos_h = None
        self.bucket_start = None   # host int64 [num_buckets + 1]
        self.n = 0
        self.rebuilds = 0

    # ------------------------------------------------------------------ maintenance
    def refresh(self, state: Optional[Tuple[int, Optional[np.ndarray]]] = None) -> None:
        """Bring the index up to the store.  ``state`` = (version, changed rows) taken by the
        owning :class:`ShardedItemIndex`; otherwise this index takes them itself -- version and
        rows together, before the device view, so no write can fall between them."""
        st = self.store
        if state is None:
            if self._managed or (self.version == st.version and self.Ys is not None):
                return
        with self._lock:
            if state is None:
                if self.version == st.version and self.Ys is not None:
                    return
                state = st.take_index_state(self._token)
            ver, dirty = state
            mat, valid, _ = st.device_view()
            parts = st.device_partitions()
            if self.Ys is None or dirty is None or not self._update_in_place(mat, valid, parts,
                                                                             dirty):
                self._rebuild(mat, valid, parts)
            self.version = ver

    def _buckets(self, parts, rows):
        if parts is None:
            return torch.zeros(rows.numel(), dtype=torch.int64, device=rows.device)
        return parts[rows].to(torch.int64)

    def _rebuild(self, mat, valid, parts) -> None:
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
        ys = torch.zeros((max(n, 1), self.kp), dtype=torch.float32, device=dev)
        # gathered in slices of 1M rows: a whole-matrix mat[rows] temporary would add another
        # full copy of the item factors to the peak HBM of a rebuild (20 GB at 20M x 250)
        step = 1 << 20
        for lo in range(0, n, step):
            hi = min(n, lo + step)
            ys[lo:hi, :self.k] = mat[rows[lo:hi]].to(dev)
        rows = rows.to(dev)
        b = b.to(dev)
        self.Ys = ys
        nrm = ys[:n].norm(dim=1) if n else torch.zeros(0, device=dev)
        self.inv_norm = torch.where(nrm > 0, 1.0 / nrm, torch.zeros_like(nrm))
        self.bucket_of = b.to(torch.int32).contiguous()
        pos = torch.full((mat.shape[0],), -1, dtype=torch.int64, device=dev)
        if n:
            pos[rows] = torch.arange(n, device=dev)
        self.pos_of_row = pos
        self.row_of_pos = rows
        self.row_of_pos_h = rows.cpu().numpy()
        counts = torch.bincount(b, minlength=self.num_buckets).cpu().numpy()
        self.bucket_start = np.zeros(self.num_buckets + 1, dtype=np.int64)
        np.cumsum(counts, out=self.bucket_start[1:])
        self.n = n
        self.rebuilds += 1

    def _update_in_place(self, mat, valid, parts, dirty: np.ndarray) -> bool:
        if len(dirty) == 0:
            return True
        if len(dirty) > max(4096, self.n // 16):
            return False
        dev = self.device
        d, nsh = self.shard
        dirty = np.asarray(dirty, dtype=np.int64)
        if nsh > 1:
            dirty = dirty[dirty % nsh == d]
            if len(dirty) == 0:
                return True
        src = torch.from_numpy(dirty).to(mat.device)
        rows = src.to(dev)
        if int(rows.max()) >= self.pos_of_row.numel():
            return False
        pos = self.pos_of_row[rows]
        ok = valid[src].to(dev)
        # new / removed rows or a changed bucket need a re-sort
        if bool(((pos < 0) | ~ok).any()):
            return False
        nb = self._buckets(parts, src).to(dev)
        if bool((nb != self.bucket_of[pos].to(torch.int64)).any()):
            return False
        self.Ys[pos, :self.k] = mat[src].to(dev)
        nrm = self.Ys[pos].norm(dim=1)
        self.inv_norm[pos] = torch.where(nrm > 0, 1.0 / nrm, torch.zeros_like(nrm))
        return True

    # ------------------------------------------------------------------ queries
    def scan(self, queries: Sequence[TopNQuery]) -> List[Tuple[np.ndarray, np.ndarray]]:
        """Per query: (store rows, scores) of the best ``how_many``, descending."""
        self.refresh()
        out: List[Tuple[np.ndarray, np.ndarray]] = []
        for lo in range(0, len(queries), MAX_BATCH):
            out.extend(self._scan_batch(queries[lo:lo + MAX_BATCH]))
        return out

    def _scan_batch(self, qs: Sequence[TopNQuery]):
        empty = (np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.float32))
        if self.n == 0:
            return [empty for _ in qs]
        # cosine and dot queries differ in the epilogue: one launch per kind
        res: List[Optional[Tuple[np.ndarray, np.ndarray]]] = [None] * len(qs)
        for cos in (False, True):
            idx = [j for j, q in enumerate(qs) if bool(q.cosine) == cos]
            if idx:
                for j, r in zip(idx, self._launch([qs[j] for j in idx], cos)):
                    res[j] = r
        return res

    def _launch(self, qs: Sequence[TopNQuery], cosine: bool):
        dev = self.device
        lib = native.require_kernels()
        nq = len(qs)
        Q = np.zeros((MAX_BATCH, self.kp), dtype=np.float32)
        for j, q in enumerate(qs):
            Q[j, :self.k] = np.asarray(q.target, dtype=np.float32)[:self.k]
        # candidate ranges: union over the batch; per-query bucket bitmaps when pruning
        use_lsh = any(q.candidates is not None for q in qs)
        bits = None
        if use_lsh:
            allb = np.zeros(self.num_buckets, dtype=bool)
            bits = np.zeros((nq, self.words), dtype=np.uint32)
            for j, q in enumerate(qs):
                c = np.arange(self.num_buckets) if q.candidates is None else \
                    np.asarray(q.candidates, dtype=np.int64)
                allb[c] = True
                np.bitwise_or.at(bits[j], c >> 5, (np.uint32(1) << (c & 31).astype(np.uint32)))
            sel = np.nonzero(allb)[0]
            starts = self.bucket_start[sel]
            ends = self.bucket_start[sel + 1]
            keep = ends > starts
            starts, ends = starts[keep], ends[keep]
            if len(starts) == 0:
                return [(np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.float32))
                        for _ in qs]
            # merge adjacent ranges
            brk = np.nonzero(starts[1:] != ends[:-1])[0] + 1
            rs = np.stack([starts[np.r_[0, brk]], ends[np.r_[brk - 1, len(ends) - 1]]], 1)
        else:
            rs = np.array([[0, self.n]], dtype=np.int64)
        tiles = (rs[:, 1] - rs[:, 0] + 15) // 16
        tile0 = np.zeros(len(rs) + 1, dtype=np.int64)
        np.cumsum(tiles, out=tile0[1:])
        n_tiles = int(tile0[-1])
        # excluded store rows -> sorted positions per query
        ptr = np.zeros(nq + 1, dtype=np.int32)
        ex_parts = []
        any_ex = False
        for j, q in enumerate(qs):
            er = q.exclude_rows
            if er is not None and len(er):
                any_ex = True
                ex_parts.append(np.asarray(er, dtype=np.int64))
            else:
                ex_parts.append(np.zeros(0, dtype=np.int64))
        ex_dev = None
        if any_ex:
            flat = torch.from_numpy(np.concatenate(ex_parts)).to(dev)
            p = self.pos_of_row[flat.clamp(0, self.pos_of_row.numel() - 1)]
            p = torch.where(flat < self.pos_of_row.numel(), p, torch.full_like(p, -1))
            p_h = p.cpu().numpy()
            lo = 0
            chunks = []
            for j, e in enumerate(ex_parts):
                pj = np.sort(p_h[lo:lo + len(e)])
                pj = pj[pj >= 0].astype(np.int32)
                lo += len(e)
                chunks.append(pj)
                ptr[j + 1] = ptr[j] + len(pj)
            ex_dev = torch.from_numpy(np.concatenate(chunks) if ptr[-1] else
                                      np.zeros(1, dtype=np.int32)).to(dev)
        waves = int(lib.oryx_topn_waves(n_tiles))
        o_sc = torch.empty((waves, MAX_BATCH, MAX_HOW_MANY), dtype=torch.float32, device=dev)
        o_rw = torch.empty((waves, MAX_BATCH, MAX_HOW_MANY), dtype=torch.int32, device=dev)
        Qd = torch.from_numpy(Q).to(dev)
        rs_d = torch.from_numpy(np.ascontiguousarray(rs, dtype=np.int64)).to(dev)
        t0_d = torch.from_numpy(tile0).to(dev)
        bits_d = torch.from_numpy(bits).to(dev) if bits is not None else None
        ptr_d = torch.from_numpy(ptr).to(dev) if ex_dev is not None else None
        rc = lib.oryx_topn_scan(
            self.Ys.data_ptr(), self.inv_norm.data_ptr() if cosine else None, Qd.data_ptr(),
            self.kp, nq, self.bucket_of.data_ptr() if bits_d is not None else None,
            bits_d.data_ptr() if bits_d is not None else None, self.words, rs_d.data_ptr(),
            t0_d.data_ptr(), len(rs), n_tiles,
            ptr_d.data_ptr() if ptr_d is not None else None,
            ex_dev.data_ptr() if ex_dev is not None else None,
            o_sc.data_ptr(), o_rw.data_ptr(), native.stream_ptr(dev))
        native.check(rc, "oryx_topn_scan")
        m = max(q.how_many for q in qs)
        m = min(m, waves * MAX_HOW_MANY)
        sc = o_sc[:, :nq].permute(1, 0, 2).reshape(nq, -1)
        rw = o_rw[:, :nq].permute(1, 0, 2).reshape(nq, -1)
        v, i = torch.topk(sc, m, dim=1)
        pos = torch.gather(rw, 1, i)
        v_h, pos_h = v.cpu().numpy(), pos.cpu().numpy()
        out = []
        for j, q in enumerate(qs):
            vj, pj = v_h[j, :q.how_many], pos_h[j, :q.how_many]
            keep = np.isfinite(vj) & (pj >= 0)
            out.append((self.row_of_pos_h[pj[keep]], vj[keep]))
        return out


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

    def close(self) -> None:
        self._pool.shutdown(wait=False)

