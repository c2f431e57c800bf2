"""ALS serving model: GPU-resident item factors, host user factors, known items, top-N.

Equivalent of ``ALSServingModel`` / ``ALSServingModelManager`` / ``LocalitySensitiveHash`` /
``TopNConsumer`` (``[serving-app]/als/model/ALSServingModel.java:58-496``,
``ALSServingModelManager.java:63-154``, ``LocalitySensitiveHash.java:26-188``,
``TopNConsumer.java:55-74``) re-designed for MI355X:

* Y (items) lives in HBM as one fp32 matrix (``FeatureVectors`` device mirror); ``UP`` rows
  are applied to a host mirror and flushed to the device in one batched copy before the next
  query, so a model load of millions of rows costs a few copies;
* top-N runs on the fused HIP scan (:mod:`oryx_amd.ops.topn`, ``csrc/kernels/topn.hip``) over
  a bucket-sorted copy of Y: a query reads only its LSH candidate buckets (``oryx.als.
  sample-rate``), known / excluded items and the candidate-bucket mask are applied in the
  kernel's epilogue, and each wave keeps a top-64 per query in LDS.  Concurrent requests are
  micro-batched (``oryx.serving.max-batch``, ``batch-wait-sec``): one launch scores up to 16
  queries in one pass over the item rows.  Requests with a rescorer (host callbacks) or more
  than 64 results take the unfused torch path (scores, masks, ``topk``);
* YᵀY for anonymous fold-in is a device GEMM, cached until Y changes.
"""

from __future__ import annotations

import collections
import logging
import math
import threading
import time
from typing import Collection, Dict, Iterable, Iterator, List, Optional, Sequence, Set, Tuple

import numpy as np
import torch

from ...api import AbstractServingModelManager, KeyMessage, ServingModel
from ...ops import topn as topn_ops
from ...utils import mathx, pmml as pmmlu, rng, text
from ...utils.lang import AutoReadWriteLock
from .common import FeatureVectors
from .rescorer import Rescorer, RescorerProvider, load_rescorer_providers

__all__ = ["ALSServingModel", "ALSServingModelManager", "LocalitySensitiveHash"]

log = logging.getLogger(__name__)


def rescored_top(ids, scores: np.ndarray, rescorer: Rescorer, how_many: int
                 ) -> List[Tuple[str, float]]:
    """``TopNConsumer`` semantics over EVERY candidate: drop filtered IDs, rescore the rest,
    keep rescored values above -inf (NaN drops an item), best ``how_many`` descending."""
    if isinstance(ids, np.ndarray):
        keep = ids != None                                  # noqa: E711 (element-wise)
        if not keep.all():
            ids, scores = ids[keep], scores[keep]
    else:
        keep = np.array([i is not None for i in ids], dtype=bool)
        if not keep.all():
            ids = [i for i in ids if i is not None]
            scores = scores[keep]
    if not len(ids):
        return []
    allowed = ~np.asarray(rescorer.is_filtered_many(ids), dtype=bool)
    idx = np.flatnonzero(allowed)
    if len(idx) == 0:
        return []
    sel = ids[idx] if isinstance(ids, np.ndarray) else [ids[j] for j in idx.tolist()]
    new = np.asarray(rescorer.rescore_many(sel, np.asarray(scores, dtype=np.float64)[idx]),
                     dtype=np.float64)
    ok = np.flatnonzero(new > -np.inf)
    if len(ok) == 0:
        return []
    if len(ok) > how_many:
        part = np.argpartition(-new[ok], how_many - 1)[:how_many]
        ok = ok[part]
    ok = ok[np.argsort(-new[ok], kind="stable")]
    return [(sel[j], float(new[j])) for j in ok.tolist()]


def _done(result):
    """A finisher that returns ``result`` (bound here, per batch, not late in a loop)."""
    return lambda: result


class TopNBatcher:
    """Micro-batches concurrent top-N requests into shared kernel launches.

    Requests queue up while a launch runs; the worker takes everything queued (up to
    ``max_batch``), optionally waiting ``wait_s`` for more, and answers each request's event.
    A request that finds no launch running, nothing queued and the last launch uncontended (and
    no ``wait_s``) runs inline on its own thread -- a lone client pays no hand-off to the
    worker (20M x 250 at 1 worker: 6.97 -> 6.27 ms mean, p99 12.9 -> 6.5 ms).  With
    ``max_batch <= 1`` requests always run inline.
    """

    def __init__(self, index: "topn_ops.ItemIndex", max_batch: int, wait_s: float):
        self.index = index
        self.max_batch = max(1, int(max_batch))
        self.wait_s = max(0.0, float(wait_s))
        self._cv = threading.Condition()
        self._queue: List[list] = []
        self._thread = None
        self._closed = False
        self._contended = False
        self._busy = False        # a launch (inline or by the worker) is running
        self._last_scan_s = 0.0
        self.batches = 0
        self.requests = 0
        self.inline = 0
        self.slow_log = collections.deque(maxlen=256)

    def submit(self, q: "topn_ops.TopNQuery"):
        if self.max_batch <= 1:
            return self.index.scan([q])[0]
        slot = [q, None, None, threading.Event()]
        with self._cv:
            # (not after a contended launch: concurrent clients keep being batched)
            inline = not self._busy and not self._queue and not self._contended and \
                self.wait_s == 0 and not self._closed
            if inline:
                self._busy = True
            else:
                if self._thread is None:
                    self._thread = threading.Thread(target=self._run, name="OryxTopNBatcher",
                                                    daemon=True)
                    self._thread.start()
                self._queue.append(slot)
                self._cv.notify()
        if inline:
            t0 = time.monotonic()
            try:
                return self.index.scan([q])[0]
            finally:
                self._last_scan_s = time.monotonic() - t0
                with self._cv:
                    self._busy = False
                    self.batches += 1
                    self.requests += 1
                    self.inline += 1
                    # requests that queued up meanwhile go to the worker (batched)
                    self._contended = bool(self._queue)
                    self._cv.notify_all()
        slot[3].wait()
        if slot[2] is not None:
            raise slot[2]
        return slot[1]

    def _run(self) -> None:
        """The worker: takes the queued requests as one batch and launches it; while that
        batch's kernel and copy back run, the next batch is taken and launched, and only then
        is the first one finished (ItemIndex.scan_async) -- the host work of one batch
        overlaps the device work of the other."""
        pending = None            # (batch, finish, t_launch, error) of the batch in flight
        while True:
            batch = None
            with self._cv:
                if pending is None:
                    while (not self._queue or self._busy) and not self._closed:
                        self._cv.wait()
                    if self._closed and not self._queue:
                        return
                    while self._busy:          # closing: let an inline launch finish first
                        self._cv.wait()
                    # wait for stragglers when asked to, or when requests queued up while the
                    # previous launch ran (concurrent clients): a tenth of that launch's time
                    wait = self.wait_s
                    if self._contended and self._last_scan_s > 0:
                        wait = max(wait, min(0.1 * self._last_scan_s, 0.005))
                    if wait > 0 and len(self._queue) < self.max_batch:
                        deadline = time.monotonic() + wait
                        while len(self._queue) < self.max_batch:
                            left = deadline - time.monotonic()
                            if left <= 0:
                                break
                            self._cv.wait(left)
                if self._queue:
                    batch = self._queue[:self.max_batch]
                    del self._queue[:len(batch)]
                    self._busy = True
            launched = None
            if batch is not None:
                t_scan = time.monotonic()
                try:
                    qs = [b[0] for b in batch]
                    start = getattr(self.index, "scan_async", None)
                    if start is not None:
                        fin = start(qs)
                    else:                      # an index without asynchronous launches
                        # bind this batch's result now: the next loop iteration rebinds
                        # the local before this batch is finished
                        fin = _done(self.index.scan(qs))
                    launched = (batch, fin, t_scan, None)
                except Exception as e:   # answered to every waiting request
                    launched = (batch, None, t_scan, e)
            if pending is not None:
                self._finish(pending, more=launched is not None)
            pending = launched

    def _finish(self, pending, more: bool) -> None:
        batch, fin, t_scan, err = pending
        if err is None:
            try:
                res = fin()
                took = time.monotonic() - t_scan
                if took > 0.01:
                    # (wall-clock launch, ms from launch to results, queries) of slow batches
                    self.slow_log.append((time.time() - took, took * 1e3, len(batch)))
                for b, r in zip(batch, res):
                    b[1] = r
            except Exception as e:
                err = e
        if err is not None:
            for b in batch:
                b[2] = err
        with self._cv:
            self._last_scan_s = time.monotonic() - t_scan
            self.batches += 1
            self.requests += len(batch)
            self._contended = bool(self._queue) or len(batch) > 1 or more
            if not more:
                self._busy = False
            self._cv.notify_all()
        for b in batch:
            b[3].set()

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()


def _binom(n: int, k: int) -> int:
    return math.comb(n, k)


class LocalitySensitiveHash:
    MAX_HASHES = 16

    def __init__(self, sample_rate: float, num_features: int, num_cores: Optional[int] = None):
        import os
        if num_cores is None:
            num_cores = os.cpu_count() or 1
        num_hashes = 0
        bits_differing = 0
        while num_hashes < self.MAX_HASHES:
            bits_differing = 0
            num_partitions_to_try = 1
            while bits_differing < num_hashes and num_partitions_to_try < num_cores:
                bits_differing += 1
                num_partitions_to_try += _binom(num_hashes, bits_differing)
            if bits_differing == num_hashes and num_partitions_to_try < num_cores:
                num_hashes += 1
                continue
            if num_partitions_to_try <= sample_rate * (1 << num_hashes):
                break
            num_hashes += 1
        log.info("LSH with %d hashes, querying partitions with up to %d bits differing",
                 num_hashes, bits_differing)
        self.max_bits_differing = bits_differing
        gen = rng.get_random()
        vectors: List[np.ndarray] = []
        for i in range(num_hashes):
            best_total, next_best, since_best = math.inf, None, 0
            while since_best < 1000:
                cand = mathx.random_vector_f(num_features, gen)
                score = self._total_abs_cos(vectors, cand)
                if score < best_total:
                    next_best = cand
                    if score == 0.0:
                        break
                    best_total = score
                    since_best = 0
                else:
                    since_best += 1
            vectors.append(next_best)
        self.hash_vectors = np.array(vectors, dtype=np.float32).reshape(num_hashes, num_features)
        # candidate prototype: all 2^n ints ordered by popcount
        n = num_hashes
        proto = sorted(range(1 << n), key=lambda i: (bin(i).count("1"), i))
        # the reference fills each popcount class in increasing order
        self._prototype = np.array(proto, dtype=np.int64)
        self._all = np.arange(1 << n, dtype=np.int64)
        self._dev_vectors: Dict[str, torch.Tensor] = {}

    @staticmethod
    def _total_abs_cos(existing, new) -> float:
        new_norm = mathx.norm(new)
        s = 0.0
        for e in existing:
            s += abs(mathx.dot(e, new)) / mathx.norm(e) / new_norm
        return s

    def get_num_hashes(self) -> int:
        return self.hash_vectors.shape[0]

    def get_num_partitions(self) -> int:
        return 1 << self.get_num_hashes()

    def get_max_bits_differing(self) -> int:
        return self.max_bits_differing

    def get_index_for(self, vector) -> int:
        index = 0
        for i, h in enumerate(self.hash_vectors):
            if mathx.dot(h, vector) > 0.0:
                index |= 1 << i
        return index

    def get_candidate_indices(self, vector) -> np.ndarray:
        main = self.get_index_for(vector)
        n = self.get_num_hashes()
        if n == self.max_bits_differing:
            return self._all
        if self.max_bits_differing == 0:
            return np.array([main], dtype=np.int64)
        how_many = sum(_binom(n, i) for i in range(self.max_bits_differing + 1))
        return self._prototype[:how_many] ^ main

    def device_partitioner(self, device):
        """rows [m, k] fp32 (device) -> bucket index per row, computed as sign bits of H v."""
        n = self.get_num_hashes()
        if n == 0:
            return None
        key = str(device)
        if key not in self._dev_vectors:
            self._dev_vectors[key] = torch.from_numpy(self.hash_vectors).to(device)
        H = self._dev_vectors[key]
        weights = (1 << torch.arange(n, device=device, dtype=torch.int64))

        def part(rows: torch.Tensor) -> torch.Tensor:
            bits = (rows.matmul(H.t()) > 0).to(torch.int64)
            return (bits * weights).sum(1)
        return part


class ALSServingModel(ServingModel):
    def __init__(self, features: int, implicit: bool, sample_rate: float = 1.0,
                 rescorer_provider: Optional[RescorerProvider] = None,
                 device: Optional[torch.device] = None, max_batch: int = 16,
                 batch_wait_s: float = 0.0, scan_devices: Optional[Sequence] = None):
        if features <= 0 or not (0.0 < sample_rate <= 1.0):
            raise ValueError("bad features / sample rate")
        if device is None:
            device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        self.device = device
        self.sample_rate = sample_rate
        # one GPU scans every candidate bucket at once: size the LSH for the sample rate alone
        self.lsh = LocalitySensitiveHash(sample_rate, features, num_cores=1)
        self.features = features
        self.implicit = implicit
        self.rescorer_provider = rescorer_provider
        self.X = FeatureVectors(features, None)
        # device rows padded to the scan kernel's stride: the top-N index reads them in place
        # (one device copy of Y)
        self.Y = FeatureVectors(features, device,
                                partitioner=self.lsh.device_partitioner(device),
                                row_pad=topn_ops.row_pad_for(features))
        from ... import ingest
        self._kdict = ingest.IdDict()
        self._known: Dict[str, np.ndarray] = {}
        self._known_lock = AutoReadWriteLock()
        self._expected_users: Set[str] = set()
        self._expected_items: Set[str] = set()
        self._expected_lock = threading.Lock()
        self._yty_solver = None
        self._yty_version = -1
        self.index = None
        self.batcher = None
        if topn_ops.kernel_ok(device, features):
            if scan_devices is not None and len(scan_devices) > 1:
                # item-sharded scan over several GPUs (oryx.serving.scan-gpus)
                self.index = topn_ops.ShardedItemIndex(self.Y, self.lsh.get_num_partitions(),
                                                       scan_devices)
            else:
                self.index = topn_ops.ItemIndex(self.Y, self.lsh.get_num_partitions())
            self.batcher = TopNBatcher(self.index, max_batch, batch_wait_s)

    # ---------------------------------------------------------------- accessors
    def get_features(self) -> int:
        return self.features

    def is_implicit(self) -> bool:
        return self.implicit

    def get_rescorer_provider(self) -> Optional[RescorerProvider]:
        return self.rescorer_provider

    def get_user_vector(self, user: str) -> Optional[np.ndarray]:
        return self.X.get_vector(user)

    def get_item_vector(self, item: str) -> Optional[np.ndarray]:
        return self.Y.get_vector(item)

    def set_user_vector(self, user: str, vector) -> None:
        if len(vector) != self.features:
            raise ValueError("wrong vector length")
        self.X.set_vector(user, vector)
        with self._expected_lock:
            self._expected_users.discard(user)

    def set_item_vector(self, item: str, vector) -> None:
        if len(vector) != self.features:
            raise ValueError("wrong vector length")
        self.Y.set_vector(item, vector)
        with self._expected_lock:
            self._expected_items.discard(item)

    def set_user_vectors(self, ids: Sequence[str], mat: np.ndarray) -> None:
        """Bulk :meth:`set_user_vector` (model loads)."""
        self.X.set_vectors(ids, mat)
        with self._expected_lock:
            self._expected_users.difference_update(ids)
            if not self._expected_users:
                # a drained set keeps its 20M-slot table (walked by every gen-2 GC pass)
                self._expected_users = set()

    def set_item_vectors(self, ids: Sequence[str], mat: np.ndarray) -> None:
        self.Y.set_vectors(ids, mat)
        with self._expected_lock:
            self._expected_items.difference_update(ids)
            if not self._expected_items:
                # a drained set keeps its 20M-slot table (walked by every gen-2 GC pass)
                self._expected_items = set()

    # known items are held as int32 codes of one native item dictionary per model (a loaded
    # model has ~20 per user: 10M Python strings in sets would dominate the load time and the
    # host memory); arrays may repeat an item when a message's list did -- readers dedupe
    @property
    def known_items_dict(self):
        return self._kdict

    def get_known_items(self, user: str) -> Set[str]:
        with self._known_lock.read():
            a = self._known.get(user)
        if a is None or len(a) == 0:
            return set()
        keys = self._kdict.key_list()
        return {keys[c] for c in a.tolist()}

    def add_known_items(self, user: str, items: Iterable[str]) -> None:
        items = list(items)
        codes = self._kdict.encode(items).astype(np.int32) if items else \
            np.zeros(0, dtype=np.int32)
        with self._known_lock.write():
            self._merge_known(user, codes)

    def _merge_known(self, user: str, codes: np.ndarray) -> None:
        a = self._known.get(user)
        if a is None or len(a) == 0:
            self._known[user] = codes
        elif len(codes):
            self._known[user] = np.union1d(a, codes).astype(np.int32)

    def add_known_items_many(self, pairs) -> None:
        """Bulk :meth:`add_known_items` over (user, items) pairs under one lock (loads)."""
        pairs = [(u, list(items)) for u, items in pairs]
        flat = [i for _, items in pairs for i in items]
        codes = self._kdict.encode(flat).astype(np.int32) if flat else \
            np.zeros(0, dtype=np.int32)
        with self._known_lock.write():
            pos = 0
            for user, items in pairs:
                self._merge_known(user, codes[pos:pos + len(items)])
                pos += len(items)

    def add_known_item_codes(self, users: Sequence[str], known, rows) -> None:
        """Known items of parsed ``UP`` rows (``ingest.KnownCodes`` of :attr:`known_items_dict`)
        for the rows ``rows`` (log order): one lock, no per-item Python objects."""
        codes, offs, has = known.codes, known.offs, known.has
        with self._known_lock.write():
            km = self._known
            for j in rows:
                if not has[j]:
                    continue
                c = codes[offs[j]:offs[j + 1]]
                u = users[j]
                a = km.get(u)
                if a is None or len(a) == 0:
                    km[u] = c
                elif len(c):
                    km[u] = np.union1d(a, c).astype(np.int32)

    def _known_pairs(self):
        """(user index per known entry, item code per entry, users) with duplicates removed."""
        with self._known_lock.read():
            users = list(self._known.keys())
            arrs = list(self._known.values())
        if not arrs:
            return np.zeros(0, np.int64), np.zeros(0, np.int64), users
        lens = np.fromiter((len(a) for a in arrs), dtype=np.int64, count=len(arrs))
        uidx = np.repeat(np.arange(len(arrs), dtype=np.int64), lens)
        items = np.concatenate(arrs).astype(np.int64) if lens.sum() else np.zeros(0, np.int64)
        if len(items):
            key = np.unique(uidx * (int(items.max()) + 1) + items)
            n_i = int(items.max()) + 1
            uidx, items = key // n_i, key % n_i
        return uidx, items, users

    def get_user_counts(self) -> Dict[str, int]:
        uidx, _, users = self._known_pairs()
        cnt = np.bincount(uidx, minlength=len(users))
        return dict(zip(users, cnt.tolist()))

    def get_item_counts(self) -> Dict[str, int]:
        _, items, _ = self._known_pairs()
        if len(items) == 0:
            return {}
        cnt = np.bincount(items)
        keys = self._kdict.key_list()
        nz = np.flatnonzero(cnt)
        return {keys[c]: int(cnt[c]) for c in nz.tolist()}

    def get_known_item_vectors_for_user(self, user: str):
        if self.get_user_vector(user) is None:
            return None
        known = self.get_known_items(user)
        if not known:
            return None
        out = []
        for item in known:
            v = self.get_item_vector(item)
            if v is not None:
                out.append((item, v))
        return out or None

    def get_all_user_ids(self) -> List[str]:
        return self.X.all_ids()

    def get_all_item_ids(self) -> List[str]:
        return self.Y.all_ids()

    def get_num_users(self) -> int:
        return self.X.size()

    def get_num_items(self) -> int:
        return self.Y.size()

    # ---------------------------------------------------------------- top-N on the GPU
    def _rescored_top_n(self, tgt, cosine, cands, ex, rescorer, how_many):
        """Every candidate through the rescorer: on the device when it has a device form
        (``Rescorer.rescore_device``: scores stay on the GPU, top-N by a device top-k), else
        the host array forms over the candidates' IDs (one fancy index of the store's cached
        ID array, no per-request Python list)."""
        rows, scores = self.index.all_scores_device(tgt, cosine, cands, ex)
        if rows.numel() == 0:
            return []
        new = rescorer.rescore_device(rows, scores, self.Y)
        if new is not None:
            ok = torch.nonzero(new > float("-inf")).flatten()      # NaN compares false
            if ok.numel() == 0:
                return []
            v, j = torch.topk(new[ok].double(), min(how_many, ok.numel()))
            r = rows[ok[j]].cpu().numpy()
            ids = self.Y.id_array()[r]
            return [(i, float(x)) for i, x in zip(ids.tolist(), v.cpu().tolist())
                    if i is not None]
        rh, sh = rows.cpu().numpy(), scores.cpu().numpy()
        return rescored_top(self.Y.id_array()[rh], sh, rescorer, how_many)

    def top_n(self, target: np.ndarray, how_many: int, cosine: bool = False,
              exclude: Optional[Collection[str]] = None,
              rescorer: Optional[Rescorer] = None) -> List[Tuple[str, float]]:
        """Best ``how_many`` items by ``dot(y, target)`` (or ``/|y|`` when ``cosine``).

        ``exclude``: item IDs never returned.  ``rescorer``: filter + rescore applied to every
        candidate item (exact ``TopNConsumer`` semantics).  Any depth is exact: the fused
        kernel handles deep requests in one or more passes.
        """
        if how_many <= 0 or self.Y.size() == 0:
            return []
        lsh_on = self.lsh.get_max_bits_differing() < self.lsh.get_num_hashes()
        cands = self.lsh.get_candidate_indices(target) if lsh_on else None
        if self.index is not None:
            ex = self.Y.host_rows(exclude) if exclude else None
            tgt = np.asarray(target, dtype=np.float32)
            if rescorer is not None:
                return self._rescored_top_n(tgt, cosine, cands, ex, rescorer, how_many)
            q = topn_ops.TopNQuery(tgt, how_many, cosine, cands, ex)
            if self.batcher is not None and how_many <= topn_ops.MAX_HOW_MANY:
                rows, scores = self.batcher.submit(q)
            else:
                rows, scores = self.index.scan([q])[0]
            out = []
            for id_, v in zip(self.Y.ids_of_rows(rows.tolist()), scores.tolist()):
                if id_ is not None:
                    out.append((id_, float(v)))
            return out
        # no kernel (CPU device): torch over the store's device mirror
        mat, valid, norms = self.Y.device_view()
        n = mat.shape[0]
        if n == 0:
            return []
        q = torch.as_tensor(np.asarray(target, dtype=np.float32), device=mat.device)
        scores = mat.matmul(q)
        if cosine:
            scores = scores / norms
        neg_inf = torch.tensor(float("-inf"), device=mat.device)
        scores = torch.where(valid, scores, neg_inf)
        parts = self.Y.device_partitions()
        if parts is not None and cands is not None:
            cand = torch.zeros(self.lsh.get_num_partitions(), dtype=torch.bool,
                               device=mat.device)
            cand[torch.from_numpy(np.asarray(cands)).to(mat.device)] = True
            scores = torch.where(cand[parts], scores, neg_inf)
        if exclude:
            rows = self.Y.host_rows(exclude)
            if rows:
                scores[torch.as_tensor(rows, device=mat.device)] = float("-inf")
        if rescorer is not None:
            live = torch.nonzero(scores > float("-inf")).flatten()
            rows = live.cpu().numpy()
            return rescored_top(self.Y.ids_of_rows(rows.tolist()),
                                scores[live].cpu().numpy(), rescorer, how_many)
        m = min(how_many, n)
        vals, idx = torch.topk(scores, m)
        vals, idx = vals.cpu().numpy(), idx.cpu().numpy()
        out = []
        for v, i in zip(vals, idx):
            if v == float("-inf"):
                break
            id_ = self.Y.id_of_row(int(i))
            if id_ is not None:
                out.append((id_, float(v)))
        return out

    def get_yty_solver(self):
        ver = self.Y.version
        if self._yty_solver is not None and self._yty_version == ver:
            return self._yty_solver
        vtv = self.Y.get_vtv()
        solver = mathx.get_solver(vtv)
        self._yty_solver, self._yty_version = solver, ver
        return solver

    # ---------------------------------------------------------------- model-update pruning
    def retain_recent_and_user_ids(self, users: Collection[str]) -> None:
        self.X.retain_recent_and_ids(users)
        with self._expected_lock:
            self._expected_users = set(users)
            self.X.remove_all_ids_from(self._expected_users)
            # the expected rows arrive as UP messages next: room for all of them at once
            self.X.reserve_extra(len(self._expected_users))

    def retain_recent_and_item_ids(self, items: Collection[str]) -> None:
        self.Y.retain_recent_and_ids(items)
        with self._expected_lock:
            self._expected_items = set(items)
            self.Y.remove_all_ids_from(self._expected_items)
            self.Y.reserve_extra(len(self._expected_items))

    def retain_recent_and_known_items(self, users: Collection[str], items: Collection[str]
                                      ) -> None:
        recent_users: Set[str] = set()
        self.X.add_all_recent_to(recent_users)
        with self._known_lock.write():
            for u in [u for u in self._known if u not in users and u not in recent_users]:
                del self._known[u]
        recent_items: Set[str] = set()
        self.Y.add_all_recent_to(recent_items)
        keys = self._kdict.key_list()
        keep = np.fromiter((k in items or k in recent_items for k in keys), dtype=bool,
                           count=len(keys))
        if keep.all():
            return
        with self._known_lock.write():
            for u, a in list(self._known.items()):
                if len(a):
                    self._known[u] = a[keep[a]]

    def warm(self) -> float:
        """Take, once the model has loaded, every first-time path that the first ``UP`` rows
        after a load would otherwise take under traffic: the known-items key cache (sized with
        headroom), one row of each store re-written with its own value (dirty-row upload, the
        index's incremental update, the bf16 mirror's row conversion) and a scan.  Values and
        answers are unchanged.  Returns the seconds taken."""
        t0 = time.perf_counter()
        self._kdict.key_list()
        def some_id(store):
            for r in range(min(64, store.size())):
                id_ = store.id_of_row(r)
                if id_ is not None:
                    return id_
            return None
        for store in (self.X, self.Y):
            id_ = some_id(store)
            vec = store.get_vector(id_) if id_ is not None else None
            if vec is not None:
                store.set_vectors([id_], vec[None])
        if self.index is not None and self.device.type == "cuda":
            # a throwaway model of the same shape on the same device, whose items move between
            # LSH buckets: the index's incremental kill / append paths launch their kernels
            # for the first time here -- code objects are loaded on demand, ~100 ms on the
            # first UP rows after a 20M-item load otherwise (r6_traffic_20m_250_lsh03_v6) --
            # without a single write to this model
            tmp = ALSServingModel(self.features, self.implicit, self.sample_rate,
                                  device=self.device, max_batch=1)
            g = np.random.default_rng(0)
            ids = ["w%d" % j for j in range(512)]
            tmp.set_item_vectors(ids, g.standard_normal((512, self.features)).astype(np.float32))
            q = g.standard_normal(self.features).astype(np.float32)
            tmp.top_n(q, 1)
            tmp.set_item_vectors(ids[:64], -g.standard_normal((64, self.features))
                                 .astype(np.float32))
            tmp.top_n(q, 1)
            tmp.top_n(q, 1, cosine=True, exclude=ids[:1])
            del tmp
        if self.Y.size():
            self.top_n(np.zeros(self.features, dtype=np.float32), 1)
            iid = some_id(self.Y)
            y = self.get_item_vector(iid) if iid is not None else None
            if y is not None:
                self.top_n(y, 1, cosine=True, exclude=[iid])      # /similarity's scan
            uid = some_id(self.X)
            u = self.get_user_vector(uid) if uid is not None else None
            if u is not None:
                self.top_n(u, 1, exclude=self.get_known_items(uid) or None)
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return time.perf_counter() - t0

    def get_fraction_loaded(self) -> float:
        with self._expected_lock:
            expected = len(self._expected_users) + len(self._expected_items)
        if expected == 0:
            return 1.0
        loaded = float(self.get_num_users() + self.get_num_items())
        return loaded / (loaded + expected)

    def __repr__(self):
        return ("ALSServingModel[features:%d, implicit:%s, X:(%d users), Y:(%d items), "
                "fractionLoaded:%s, device:%s]" % (self.features, self.implicit,
                                                   self.get_num_users(), self.get_num_items(),
                                                   self.get_fraction_loaded(), self.device))


def apply_up_batch(model, messages: List[str]) -> None:
    """Apply ``UP`` rows in bulk: ``ingest.parse_up_batch`` then one ``set_vectors`` per
    matrix (the later row wins for a repeated ID), known items added per user; messages the
    native parser rejects go through the per-message path (and raise as it does)."""
    from ... import ingest
    kinds, ids, vecs, known = ingest.parse_up_batch(
        messages, model.get_features(), known_dict=ingest._known_mode(model))
    apply_up_parsed(model, kinds, ids, vecs, known, messages)


def drain_up_blocks(model, updates) -> int:
    """Apply the ``UP`` runs the update iterator can parse straight from the log
    (:meth:`~oryx_amd.serving.layer.UpdateIterator.take_up_block`) until a different message
    or the end of what is available; returns rows applied.  The next block is read and
    parsed (native, without the GIL) on a helper thread while this one is applied to the
    model; only that thread touches the iterator until the run ends."""
    take = getattr(updates, "take_up_block", None)
    if take is None:
        return 0
    from concurrent.futures import ThreadPoolExecutor
    from ... import ingest
    k = model.get_features()
    kd = ingest._known_mode(model)
    done = 0
    with ThreadPoolExecutor(max_workers=1, thread_name_prefix="oryx-up-parse") as ex:
        fut = ex.submit(take, k, known_dict=kd)
        while True:
            t0 = time.perf_counter()
            blk = fut.result()
            t1 = time.perf_counter()
            if blk is None:
                DRAIN_STATS["wait_s"] += t1 - t0
                break
            fut = ex.submit(take, k, known_dict=kd)
            apply_up_parsed(model, *blk)
            done += len(blk[0])
            DRAIN_STATS["wait_s"] += t1 - t0
            DRAIN_STATS["apply_s"] += time.perf_counter() - t1
            DRAIN_STATS["rows"] += len(blk[0])
            DRAIN_STATS["blocks"] += 1
    return done


# where a bulk model load spends its time (the bench's time-to-ready record reads these):
# waiting for the parse thread's next block vs applying blocks on this thread
DRAIN_STATS = {"wait_s": 0.0, "apply_s": 0.0, "rows": 0, "blocks": 0}


def apply_up_parsed(model, kinds, ids, vecs, known, messages=None) -> None:
    """Apply parsed ``UP`` rows (see :func:`apply_up_batch`) in message order; kind-2 rows
    (the native parser's rejects) are re-parsed from ``messages`` on the per-message path.

    The batch is cut at every kind-2 row, so an ID updated both by a rejected row and a parsed
    row ends with whichever came last in the log, as on the per-message path."""
    kinds = np.asarray(kinds)
    bad = np.nonzero(kinds == 2)[0].tolist()
    if bad and messages is None:
        raise ValueError("unparseable UP rows without their messages")
    lo = 0
    for cut in bad + [len(kinds)]:
        if cut > lo:
            _apply_parsed_run(model, kinds, ids, vecs, known, lo, cut)
        if cut < len(kinds):
            _apply_up_message(model, messages[cut])
        lo = cut + 1


def _apply_parsed_run(model, kinds, ids, vecs, known, lo: int, hi: int) -> None:
    from ... import ingest
    for kind, setter in ((0, "set_user_vectors"), (1, "set_item_vectors")):
        sel = lo + np.nonzero(kinds[lo:hi] == kind)[0]
        if not len(sel):
            continue
        # the bulk setters keep the last row of an ID repeated within the batch
        t0 = time.perf_counter()
        if len(sel) == hi - lo:
            getattr(model, setter)(ids[lo:hi], vecs[lo:hi])
        else:
            getattr(model, setter)([ids[j] for j in sel.tolist()], vecs[sel])
        DRAIN_STATS["set_" + setter[4:8] + "_s"] = \
            DRAIN_STATS.get("set_" + setter[4:8] + "_s", 0.0) + time.perf_counter() - t0
        if known is None:
            continue
        if kind == 0 and isinstance(known, ingest.KnownCodes):
            if hasattr(model, "add_known_item_codes"):
                model.add_known_item_codes(ids, known, sel.tolist())
        elif kind == 0 and hasattr(model, "add_known_items_many"):
            model.add_known_items_many((ids[j], known[j]) for j in sel.tolist() if known[j])
        elif kind == 0 and hasattr(model, "add_known_items"):
            for j in sel.tolist():
                if known[j]:
                    model.add_known_items(ids[j], known[j])


def _apply_up_message(model, message) -> None:
    update = text.read_json(message)
    vector = np.asarray(update[2], dtype=np.float32)
    if update[0] == "X":
        model.set_user_vector(str(update[1]), vector)
        if len(update) > 3 and hasattr(model, "add_known_items"):
            model.add_known_items(str(update[1]), [str(x) for x in update[3]])
    elif update[0] == "Y":
        model.set_item_vector(str(update[1]), vector)
    else:
        raise ValueError("Bad message: %r" % (message,))


class ALSServingModelManager(AbstractServingModelManager):
    def __init__(self, config):
        super().__init__(config)
        self.sample_rate = config.get_double("oryx.als.sample-rate")
        from ...utils import config as cfg
        self.max_batch = cfg.get_optional_int(config, "oryx.serving.max-batch") or 16
        wait = config.get_double("oryx.serving.batch-wait-sec") \
            if config.has_path("oryx.serving.batch-wait-sec") else 0.0
        self.batch_wait_s = float(wait)
        self.rescorer_provider = load_rescorer_providers(
            config.get_string("oryx.als.rescorer-provider-class")
            if config.has_path("oryx.als.rescorer-provider-class") else None)
        if not (0.0 < self.sample_rate <= 1.0):
            raise ValueError("sample-rate must be in (0,1]")
        # oryx.serving.scan-gpus > 1: the item matrix is sharded over that many GPUs for the
        # top-N scan (ShardedItemIndex); 1 = one GPU (horizontal replicas scale out instead)
        ng = cfg.get_optional_int(config, "oryx.serving.scan-gpus") or 1
        self.scan_devices = None
        if ng > 1 and torch.cuda.is_available():
            avail = torch.cuda.device_count()
            self.scan_devices = [torch.device("cuda", j % avail) for j in range(ng)]
        self.model: Optional[ALSServingModel] = None
        # the last UP applications: (wall-clock start, ms, rows) -- what a latency record
        # correlates its slow requests with (bench_traffic.py)
        self.apply_log = collections.deque(maxlen=1024)
        self._warmed = None          # the model last warmed (ALSServingModel.warm)
        self.warm_s: Optional[float] = None

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
                    # a run of UP rows already fetched: one native parse, bulk row updates
                    # the decoded UP rows already fetched, then the rest of the run parsed
                    # natively from the log buffer
                    t_wall, t0 = time.time(), time.perf_counter()
                    batch = [message] + [m.message for m in take(lambda m: m.key == "UP",
                                                                 poll=False)]
                    apply_up_batch(self.model, batch)
                    n_up = len(batch) + drain_up_blocks(self.model, updates)
                    self.apply_log.append((t_wall, (time.perf_counter() - t0) * 1e3, n_up))
                    countdown -= n_up
                    self._maybe_warm()
                    if countdown <= 0:
                        log.info("%s", self.model)
                        countdown = 10000
                    continue
                update = text.read_json(message)
                id_ = str(update[1])
                vector = np.asarray(update[2], dtype=np.float32)
                which = update[0]
                if which == "X":
                    self.model.set_user_vector(id_, vector)
                    if len(update) > 3:
                        self.model.add_known_items(id_, [str(x) for x in update[3]])
                elif which == "Y":
                    self.model.set_item_vector(id_, vector)
                else:
                    raise ValueError("Bad message: %r" % (km,))
                countdown -= 1
                if countdown <= 0:
                    log.info("%s", self.model)
                    countdown = 10000
                self._maybe_warm()
            elif key in ("MODEL", "MODEL-REF"):
                log.info("Loading new model")
                self._warmed = None
                pmml = pmmlu.read_pmml_from_update_key_message(key, message)
                features = int(pmml.get_extension_value("features"))
                implicit = pmml.get_extension_value("implicit").lower() == "true"
                if self.model is None or features != self.model.get_features():
                    log.warning("No previous model, or # features has changed; creating new one")
                    self.model = ALSServingModel(features, implicit, self.sample_rate,
                                                 self.rescorer_provider,
                                                 max_batch=self.max_batch,
                                                 batch_wait_s=self.batch_wait_s,
                                                 scan_devices=self.scan_devices)
                log.info("Updating model")
                xids = set(pmml.get_extension_content("XIDs") or [])
                yids = set(pmml.get_extension_content("YIDs") or [])
                self.model.retain_recent_and_known_items(xids, yids)
                self.model.retain_recent_and_user_ids(xids)
                self.model.retain_recent_and_item_ids(yids)
                # the loop frame outlives this message: drop the ID sets (20M strings in
                # a set stay in every gen-2 GC walk until the next model otherwise)
                del xids, yids, pmml
                log.info("Model updated: %s", self.model)
            else:
                raise ValueError("Bad message: %r" % (km,))

    def _maybe_warm(self) -> None:
        """Warm the model (:meth:`ALSServingModel.warm`) on this consumer thread once it has
        completely loaded: the first ``UP`` rows after a load otherwise stalled every serving
        thread for 30-40 ms growing the 20M-key known-items cache with the GIL held
        (profiles/r6_traffic_20m_250_lsh03_v4.json, stacks from bench_traffic's stall watch)."""
        m = self.model
        if m is None or self._warmed is m or m.get_fraction_loaded() < 1.0:
            return
        self._warmed = m
        try:
            self.warm_s = m.warm()
            log.info("Serving model warmed in %.2fs", self.warm_s)
        except Exception:   # noqa: BLE001 -- a failed warm-up only costs the first request
            log.exception("Serving model warm-up failed")

    def get_model(self) -> Optional[ALSServingModel]:
        return self.model
