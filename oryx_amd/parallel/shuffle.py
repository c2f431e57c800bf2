"""Key-partitioned exchanges for the sharded batch-layer data path.

The reference's Spark jobs shuffle parsed records by key (``reduceByKey`` / ``groupByKey`` in
``[mllib]/als/ALSUpdate.java:260-352``) and map string IDs to ints by parse-or-hash with a
reverse map collected to the driver.  Here every rank holds only its share of the records;
these helpers do the equivalent exchanges with ``torch.distributed`` all-to-alls:

* :func:`unify_ids` -- a collision-free global dictionary: each distinct string is owned by the
  rank ``crc32(s) % W``; owners number their strings (sorted, so the result is deterministic)
  and global codes are the owners' numbers offset by an exclusive prefix sum, so codes are
  dense in ``[0, total)`` and grouped by owner;
* :func:`route` -- send aligned rows (int64 / float64 columns) to their owner ranks;
* :func:`gather_strings` -- the owners' string tables in global code order, on every rank.

With world size 1 every helper is a local no-op.  Payloads travel as device tensors on the
RCCL backend (gloo on CPU).
"""

from __future__ import annotations

import zlib
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as tdist

from . import dist

__all__ = ["owner_of_strings", "route", "unify_ids", "gather_strings", "all_reduce_np",
           "IdTable", "lookup", "all_gather_var", "all_gather_int"]


def _dev(ctx: dist.DistContext) -> torch.device:
    return ctx.device if ctx.backend == "nccl" else torch.device("cpu")


def owner_of_strings(keys: Sequence[str], world: int) -> np.ndarray:
    return np.fromiter((zlib.crc32(k.encode("utf-8")) % world for k in keys), dtype=np.int64,
                       count=len(keys))


def _exchange(send: torch.Tensor, counts: Sequence[int], ctx) -> torch.Tensor:
    return dist.all_to_all_rows(send, counts, ctx)


def route(owner: np.ndarray, ctx: dist.DistContext, *cols: np.ndarray) -> List[np.ndarray]:
    """Send row j of every column to rank ``owner[j]``; returns the received columns (in
    source-rank order, each source's rows in their original order)."""
    if not ctx.is_distributed:
        return [np.asarray(c) for c in cols]
    W = ctx.world_size
    order = np.argsort(owner, kind="stable")
    counts = np.bincount(owner, minlength=W).tolist()
    dev = _dev(ctx)
    out = []
    for c in cols:
        c = np.asarray(c)
        kind = c.dtype
        if kind.kind == "f":
            t = torch.from_numpy(np.ascontiguousarray(c[order], dtype=np.float64))
        else:
            t = torch.from_numpy(np.ascontiguousarray(c[order], dtype=np.int64))
        got = _exchange(t.to(dev), counts, ctx).cpu().numpy()
        out.append(got.astype(kind, copy=False))
    return out


def _strings_to_blob(keys: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    enc = [k.encode("utf-8") for k in keys]
    lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
    blob = np.frombuffer(b"".join(enc), dtype=np.uint8) if enc else np.zeros(0, np.uint8)
    return blob, lens


def _blob_to_strings(blob: np.ndarray, lens: np.ndarray) -> List[str]:
    raw = blob.tobytes()
    out, p = [], 0
    for n in lens.tolist():
        out.append(raw[p:p + n].decode("utf-8"))
        p += n
    return out


def _route_strings(keys: Sequence[str], owner: np.ndarray, ctx) -> List[str]:
    W = ctx.world_size
    order = np.argsort(owner, kind="stable")
    keys_o = [keys[j] for j in order.tolist()]
    blob, lens = _strings_to_blob(keys_o)
    cnt = np.bincount(owner, minlength=W)
    ends = np.cumsum(cnt)
    starts = ends - cnt
    csum = np.r_[0, np.cumsum(lens)]
    byte_counts = [int(csum[e] - csum[s]) for s, e in zip(starts, ends)]
    dev = _dev(ctx)
    got_lens = _exchange(torch.from_numpy(lens).to(dev), cnt.tolist(), ctx).cpu().numpy()
    got_blob = _exchange(torch.from_numpy(blob.copy()).to(dev), byte_counts, ctx).cpu().numpy()
    return _blob_to_strings(got_blob.astype(np.uint8), got_lens)


def replicate_to_groups(lines: Sequence[str], ctx: dist.DistContext,
                        group_size: int) -> List[str]:
    """Re-shard strings for candidate groups (:func:`dist.split_groups` blocks of
    ``group_size`` contiguous ranks): this rank's lines go to member ``rank % group_size`` of
    EVERY group, so each group together holds the whole data set once.  Returns the lines
    this rank receives (source-rank order)."""
    W = ctx.world_size
    if not ctx.is_distributed or group_size >= W:
        return list(lines)
    G = W // group_size
    m = ctx.rank % group_size
    dests = np.array([g * group_size + m for g in range(G)], dtype=np.int64)
    n = len(lines)
    keys = list(lines) * G
    owner = np.repeat(dests, n)
    return _route_strings(keys, owner, ctx)


class IdTable:
    """The owner side of a global dictionary: this rank's strings and their global codes."""

    def __init__(self, owned: List[str], offset: int, total: int):
        self.owned = owned                    # sorted; global code = offset + position
        self.offset = offset
        self.total = total
        self._index: Optional[Dict[str, int]] = None

    def code_of(self, key: str) -> int:
        if self._index is None:
            self._index = {k: self.offset + j for j, k in enumerate(self.owned)}
        return self._index.get(key, -1)


def unify_ids(keys: Sequence[str], ctx: dist.DistContext) -> Tuple[np.ndarray, IdTable]:
    """Global dense codes for this rank's distinct ``keys`` (see module docstring); returns
    (codes aligned with ``keys``, this rank's :class:`IdTable`)."""
    keys = list(keys)
    if not ctx.is_distributed:
        owned = sorted(set(keys))
        index = {k: j for j, k in enumerate(owned)}
        return (np.fromiter((index[k] for k in keys), dtype=np.int64, count=len(keys)),
                IdTable(owned, 0, len(owned)))
    W = ctx.world_size
    owner = owner_of_strings(keys, W)
    received = _route_strings(keys, owner, ctx)
    owned = sorted(set(received))
    sizes = all_gather_int(len(owned), ctx)
    offset = int(sum(sizes[:ctx.rank]))
    total = int(sum(sizes))
    table = IdTable(owned, offset, total)
    # answer every request in the order received, then route the codes back
    codes_for_received = np.fromiter((table.code_of(k) for k in received), dtype=np.int64,
                                     count=len(received))
    back = _reply(codes_for_received, owner, ctx)
    return back, table


def _reply(values_in_received_order: np.ndarray, owner: np.ndarray, ctx) -> np.ndarray:
    """Inverse of a :func:`route` by ``owner``: values computed by the owners for the rows
    they received come back aligned with the original rows."""
    W = ctx.world_size
    # how many rows each source sent to me == the counts I route back to each source
    sent_counts = np.bincount(owner, minlength=W)
    recv_counts = all_to_all_counts(sent_counts, ctx)
    dev = _dev(ctx)
    got = _exchange(torch.from_numpy(values_in_received_order).to(dev), recv_counts.tolist(),
                    ctx).cpu().numpy()
    # got is ordered by owner rank (then original order within each owner): undo the sort
    order = np.argsort(owner, kind="stable")
    out = np.empty(len(owner), dtype=got.dtype)
    out[order] = got
    return out


def all_to_all_counts(counts: np.ndarray, ctx) -> np.ndarray:
    """counts[j] = rows this rank sends to j -> rows this rank receives from each j."""
    W = ctx.world_size
    allc = all_gather_np(np.asarray(counts, dtype=np.int64), ctx)   # [W, W]
    return allc[:, ctx.rank]


def all_gather_np(a: np.ndarray, ctx) -> np.ndarray:
    """Equal-shape arrays of every rank stacked on a new leading axis."""
    if not ctx.is_distributed:
        return np.asarray(a)[None]
    dev = _dev(ctx)
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    parts = [torch.empty_like(t) for _ in range(ctx.world_size)]
    dist.all_gather_list(parts, t, ctx)
    return torch.stack(parts).cpu().numpy()


def all_gather_int(v: int, ctx) -> List[int]:
    return [int(x) for x in all_gather_np(np.array([v], dtype=np.int64), ctx)[:, 0]]


def all_gather_var(a: np.ndarray, ctx) -> List[np.ndarray]:
    """Variable-length 1-D arrays of every rank (rank order)."""
    a = np.ascontiguousarray(a)
    if not ctx.is_distributed:
        return [a]
    sizes = all_gather_int(len(a), ctx)
    m = max(sizes) if sizes else 0
    pad = np.zeros(max(m, 1), dtype=a.dtype)
    pad[:len(a)] = a
    got = all_gather_np(pad, ctx)
    return [got[r, :sizes[r]] for r in range(ctx.world_size)]


def gather_strings(table: IdTable, ctx, keep: Optional[np.ndarray] = None) -> List[str]:
    """Every owner's strings in global code order (optionally only codes with ``keep``)."""
    own = table.owned
    if keep is not None:
        sel = keep[table.offset:table.offset + len(own)]
        own = [k for k, f in zip(own, sel.tolist()) if f]
    if not ctx.is_distributed:
        return list(own)
    blob, lens = _strings_to_blob(own)
    blobs = all_gather_var(blob, ctx)
    lenss = all_gather_var(lens, ctx)
    out: List[str] = []
    for b, l in zip(blobs, lenss):
        out.extend(_blob_to_strings(b.astype(np.uint8), l))
    return out


def all_reduce_np(a: np.ndarray, ctx, op: str = "sum") -> np.ndarray:
    if not ctx.is_distributed:
        return np.asarray(a)
    dev = _dev(ctx)
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    red = {"sum": tdist.ReduceOp.SUM, "max": tdist.ReduceOp.MAX, "min": tdist.ReduceOp.MIN}[op]
    tdist.all_reduce(t, op=red, group=ctx.group)
    return t.cpu().numpy()


def lookup(keys: Sequence[str], table: IdTable, ctx,
           mapping: Optional[np.ndarray] = None) -> np.ndarray:
    """Global code of each key (asked of its owner rank; -1 when the dictionary lacks it),
    optionally translated through ``mapping`` (a full array indexed by global code)."""
    keys = list(keys)
    if not ctx.is_distributed:
        codes = np.fromiter((table.code_of(k) for k in keys), dtype=np.int64, count=len(keys))
    else:
        owner = owner_of_strings(keys, ctx.world_size)
        received = _route_strings(keys, owner, ctx)
        answer = np.fromiter((table.code_of(k) for k in received), dtype=np.int64,
                             count=len(received))
        codes = _reply(answer, owner, ctx)
    if mapping is not None and len(codes):
        codes = np.where(codes >= 0, mapping[np.maximum(codes, 0)], -1)
    return codes


# ---------------------------------------------------------------------- blob dictionaries
# The sharded ALS batch layer's global dictionaries keep every key in native dictionaries
# (ingest.IdDict) and move keys between ranks as byte blobs: no Python string per key on the
# hot path (the string helpers above cost ~1 us per key per step).

def _blob_reorder(blob: np.ndarray, ends: np.ndarray, order: np.ndarray
                  ) -> Tuple[np.ndarray, np.ndarray]:
    """Keys ``order`` of a (blob, ends) key list, as a new (blob, ends)."""
    ends = np.asarray(ends, dtype=np.int64)
    if len(order) == 0:
        return np.zeros(0, dtype=np.uint8), np.zeros(0, dtype=np.int64)
    starts = np.r_[0, ends[:-1]]
    lens = ends - starts
    lo = lens[order]
    new_ends = np.cumsum(lo)
    total = int(new_ends[-1])
    # byte j of the output comes from starts[order[k]] + (j - new_start[k])
    src = np.repeat(starts[order] - (new_ends - lo), lo) + np.arange(total, dtype=np.int64)
    return np.ascontiguousarray(blob)[src], new_ends


def route_blob(blob: np.ndarray, ends: np.ndarray, owner: np.ndarray, ctx: dist.DistContext
               ) -> Tuple[np.ndarray, np.ndarray]:
    """Send key j of a (blob, ends) list to rank ``owner[j]``; returns the received keys as
    (blob, ends) in source-rank order, each source's keys in their original order."""
    W = ctx.world_size
    owner = np.asarray(owner, dtype=np.int64)
    order = np.argsort(owner, kind="stable")
    b, e = _blob_reorder(blob, ends, order)
    lens = np.diff(np.r_[0, e])
    cnt = np.bincount(owner, minlength=W)
    kend = np.cumsum(cnt)
    bend = np.r_[0, e][kend]
    byte_counts = np.diff(np.r_[0, bend]).tolist()
    dev = _dev(ctx)
    got_lens = _exchange(torch.from_numpy(np.ascontiguousarray(lens)).to(dev), cnt.tolist(),
                         ctx).cpu().numpy()
    got_blob = _exchange(torch.from_numpy(np.ascontiguousarray(b)).to(dev), byte_counts,
                         ctx).cpu().numpy()
    return got_blob.astype(np.uint8, copy=False), np.cumsum(got_lens)


class ShardedDict:
    """A global string dictionary over the ranks of ``ctx``: key s is owned by rank
    ``crc32(s) % W``; the owner numbers its keys in arrival order (source rank, then each
    source's first-appearance order -- deterministic for deterministic inputs) in a native
    :class:`~oryx_amd.ingest.IdDict` ``own``, and global code = ``offsets[owner]`` + the owner's
    code, so global codes are dense in ``[0, total)`` and grouped by owner."""

    def __init__(self, own, offsets: np.ndarray, ctx: dist.DistContext):
        self.own = own
        self.offsets = np.asarray(offsets, dtype=np.int64)
        self.ctx = ctx

    @property
    def total(self) -> int:
        return int(self.offsets[-1])

    @property
    def size(self) -> int:
        """Keys this rank owns."""
        return len(self.own)

    @property
    def lo(self) -> int:
        return int(self.offsets[self.ctx.rank])

    def owner_of(self, codes: np.ndarray) -> np.ndarray:
        return np.searchsorted(self.offsets, np.asarray(codes), side="right") - 1

    def owner_of_t(self, codes: torch.Tensor) -> torch.Tensor:
        off = torch.as_tensor(self.offsets, device=codes.device)
        return torch.searchsorted(off, codes, right=True) - 1

    @classmethod
    def build(cls, local, ctx: dist.DistContext) -> Tuple[np.ndarray, "ShardedDict"]:
        """(global code of each key of the local dictionary ``local``, the dictionary)."""
        from .. import ingest
        if not ctx.is_distributed:
            return np.arange(len(local), dtype=np.int64), cls(local, [0, len(local)], ctx)
        blob, ends = local.keys_blob()
        owner = local.owners(ctx.world_size)
        rblob, rends = route_blob(blob, ends, owner, ctx)
        own = ingest.IdDict()
        local_codes = own.encode_blob(rblob, rends)
        sizes = all_gather_int(len(own), ctx)
        offsets = np.r_[0, np.cumsum(sizes)].astype(np.int64)
        back = _reply(local_codes + offsets[ctx.rank], owner, ctx)
        return back, cls(own, offsets, ctx)

    def lookup(self, local) -> np.ndarray:
        """Global codes of the keys of a local dictionary (-1 for keys nobody owns)."""
        if not self.ctx.is_distributed:
            blob, ends = local.keys_blob()
            return self.own.find_blob(blob, ends)
        blob, ends = local.keys_blob()
        owner = local.owners(self.ctx.world_size)
        rblob, rends = route_blob(blob, ends, owner, self.ctx)
        c = self.own.find_blob(rblob, rends)
        c = np.where(c >= 0, c + self.lo, -1)
        return _reply(c, owner, self.ctx)

    def all_keys_blob(self, keep: Optional[np.ndarray] = None,
                      to_main: bool = False) -> Optional[Tuple[np.ndarray, np.ndarray]]:
        """Every rank's keys in global code order as one (blob, ends) -- only the owned codes
        with ``keep[code - lo]`` when given; on rank 0 only (None elsewhere) with
        ``to_main``."""
        codes = np.arange(self.size, dtype=np.int64)
        if keep is not None:
            codes = codes[np.asarray(keep, dtype=bool)[:self.size]]
        blob, ends = self.own.keys_blob(codes)
        if not self.ctx.is_distributed:
            return blob, ends
        lens = np.diff(np.r_[0, ends])
        blobs = all_gather_var(blob, self.ctx)
        lenss = all_gather_var(lens, self.ctx)
        if to_main and not self.ctx.is_main:
            return None
        allb = np.concatenate(blobs) if blobs else np.zeros(0, np.uint8)
        alll = np.concatenate(lenss) if lenss else np.zeros(0, np.int64)
        return allb.astype(np.uint8, copy=False), np.cumsum(alll)


def route_tensors(owner: torch.Tensor, ctx: dist.DistContext, *cols: torch.Tensor
                  ) -> List[torch.Tensor]:
    """:func:`route` for device tensors of one length (int64 / float64 / int32 / float32
    columns packed into ONE all-to-all of 8-byte words): row j goes to rank ``owner[j]``."""
    if not ctx.is_distributed:
        return list(cols)
    W = ctx.world_size
    dev = _dev(ctx)
    owner = owner.to(dev)
    order = torch.argsort(owner, stable=True)
    counts = torch.bincount(owner, minlength=W).cpu().tolist()
    words = []
    for c in cols:
        c = c.to(dev)[order]
        if c.dtype in (torch.float64, torch.int64):
            words.append(c.contiguous().view(torch.int64))
        elif c.dtype == torch.float32:
            words.append(c.contiguous().view(torch.int32).to(torch.int64))
        else:
            words.append(c.to(torch.int64))
    packed = torch.stack(words, 1) if words else torch.zeros((len(order), 0), dtype=torch.int64,
                                                              device=dev)
    recv = _exchange(packed, counts, ctx)
    out = []
    for j, c in enumerate(cols):
        w = recv[:, j].contiguous()
        if c.dtype == torch.float64:
            out.append(w.view(torch.float64))
        elif c.dtype == torch.int64:
            out.append(w)
        elif c.dtype == torch.float32:
            out.append(w.to(torch.int32).view(torch.float32))
        else:
            out.append(w.to(c.dtype))
    return out
