"""Resident parsed rating history for the ALS batch layer.

Every generation the reference re-reads all past data from HDFS and re-parses it
(``[lambda]/batch/BatchUpdateFunction.java:103-130`` -> ``ALSUpdate.java:194-230``'s
``parsedToRatingRDD``).  Here the parse of a past part file is kept, keyed by the file's
identity (``layers.batch.read_past_data`` marks each file's byte range of the past-data buffer
with ``(path, size, mtime)``), and only ranges never seen before -- the new interval, and an
interval's part file the first time it is read back -- go through the text parser.

A cached segment holds its undecayed parse with *segment-local* ID dictionaries: the columns
(local user / item codes as int32, strength fp64, timestamp int64 with a marker for lines
without one) live on the training device.  A generation merges the segments' dictionaries
into the build's global ones in segment order (``IdDict.merge_from``) -- which reproduces
exactly the codes one parse of the concatenated text assigns, since both are first-appearance
order -- and remaps each segment's codes with one device gather.  Decay, the zero threshold
and the time-ordered aggregation then run on the merged columns as before, so a generation's
ratings are bit-identical with and without the cache.

Segments whose key no longer appears among a generation's past data (aged out by
``max-age-data-hours``) are dropped.

The new interval is parsed as an unkeyed segment; its parse is also remembered under a hash
of its bytes (xxh3-128), and when the part file the layer saves from those same bytes is read
back next generation (a keyed miss with the same hash) that parse is adopted -- so in steady
state every interval goes through the text parser exactly once.
"""

from __future__ import annotations

import ctypes
import logging
import os
from collections import OrderedDict
from typing import Optional, Tuple

import numpy as np
import torch

from ... import ingest
from ...textlines import TextLines

log = logging.getLogger(__name__)

__all__ = ["RatingsHistory"]

_NO_TS = -(1 << 62)    # parse marker of a line without a timestamp (same as models/als/batch)


_DEVICE_PARSE = os.environ.get("ORYX_ALS_DEVICE_PARSE", "1") != "0"


def _first_appearance_codes(v: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(int32 code per element, distinct values in code order) with codes numbered in order
    of first appearance -- the numbering a dictionary fed the elements in order gives."""
    n = int(v.numel())
    uniq, inv = torch.unique(v, sorted=True, return_inverse=True)
    first = torch.full((uniq.numel(),), n, dtype=torch.int64, device=v.device)
    first.scatter_reduce_(0, inv.long(), torch.arange(n, dtype=torch.int64, device=v.device),
                          reduce="amin", include_self=True)
    order = torch.argsort(first)
    rank = torch.empty_like(order)
    rank[order] = torch.arange(order.numel(), dtype=order.dtype, device=v.device)
    return rank[inv].to(torch.int32), uniq[order]


class _Segment:
    __slots__ = ("users", "items", "u", "i", "s", "ts", "nbytes")

    def __init__(self, users, items, u, i, s, ts, nbytes):
        self.users, self.items = users, items
        self.u, self.i, self.s, self.ts = u, i, s, ts
        self.nbytes = nbytes


class RatingsHistory:
    """Parse cache of keyed :class:`TextLines` segments (see the module docstring)."""

    def __init__(self, device: Optional[torch.device] = None):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._segs: "OrderedDict[tuple, _Segment]" = OrderedDict()
        # recent unkeyed parses (new intervals) by content hash, adopted when the same bytes
        # come back as a part file
        self._unkeyed: "OrderedDict[bytes, _Segment]" = OrderedDict()
        self.stats = {"hits": 0, "misses": 0, "hit_bytes": 0, "parsed_bytes": 0,
                      "adopted": 0}

    UNKEYED_MIN_BYTES = 1 << 20
    UNKEYED_KEEP = 4

    @staticmethod
    def _digest(buf, off: int, nbytes: int) -> Optional[bytes]:
        return ingest.content_digest(buf, off, nbytes)

    def __len__(self) -> int:
        return len(self._segs)

    def resident_bytes(self) -> int:
        segs = list(self._segs.values()) + list(self._unkeyed.values())
        return sum(int(sg.u.numel()) * (4 + 4 + 8 + 8) for sg in segs)

    def clear(self) -> None:
        """Drop every cached parse (keyed segments and remembered new intervals)."""
        self._segs.clear()
        self._unkeyed.clear()

    # ------------------------------------------------------------------ parse
    DEVICE_PARSE_MIN_BYTES = 4 << 20

    def _parse_range(self, buf, off: int, nbytes: int, n_lines: int) -> _Segment:
        if self.device.type == "cuda" and nbytes >= self.DEVICE_PARSE_MIN_BYTES and \
                _DEVICE_PARSE:
            sg = self._parse_range_device(buf, off, nbytes)
            if sg is not None:
                self.stats["device_parsed_bytes"] = \
                    self.stats.get("device_parsed_bytes", 0) + nbytes
                return sg
            self.stats["device_fallbacks"] = self.stats.get("device_fallbacks", 0) + 1
        users, items = ingest.IdDict(), ingest.IdDict()
        if isinstance(buf, np.ndarray):
            view = buf[off:off + nbytes]
            data = ctypes.cast(ctypes.c_void_p(view.ctypes.data), ctypes.c_char_p)
        else:
            data = bytes(buf[off:off + nbytes])
        u, i, s, ts = ingest._parse_ratings_buf(data, nbytes, n_lines + 1, users, items,
                                                _NO_TS, False)
        dev = self.device
        return _Segment(users, items,
                        torch.from_numpy(u.astype(np.int32)).to(dev),
                        torch.from_numpy(i.astype(np.int32)).to(dev),
                        torch.from_numpy(np.ascontiguousarray(s)).to(dev),
                        torch.from_numpy(np.ascontiguousarray(ts)).to(dev), nbytes)

    def _parse_range_device(self, buf, off: int, nbytes: int) -> Optional[_Segment]:
        """The range parsed on the GPU (``oryx_rating_lines``, csv.hip): the text goes to the
        device (smaller than its parse), one thread per line; the segment's user / item keys
        are numbered in first-appearance order there (unique values, their first line, sorted)
        and only the distinct keys come back to fill the segment's dictionaries.  Codes,
        strengths and timestamps are bitwise the host parser's; None (the caller parses on the
        host) when any line is not in the plain form with canonical decimal IDs below 2^24."""
        from ... import native
        if not native.kernels_available():
            return None
        lib = native.require_kernels()
        dev = self.device
        view = np.frombuffer(buf, dtype=np.uint8, count=nbytes, offset=off) \
            if not isinstance(buf, np.ndarray) else buf[off:off + nbytes]
        pad = ((nbytes + 15) // 16) * 16 + 16
        text = torch.empty(pad, dtype=torch.uint8, device=dev)
        text[:nbytes].copy_(torch.from_numpy(view))
        text[nbytes:].zero_()
        ends = torch.nonzero(text[:nbytes] == 10).flatten()
        if view[nbytes - 1] != 10:
            ends = torch.cat([ends, torch.full((1,), nbytes, dtype=torch.int64, device=dev)])
        n = int(ends.numel())
        starts = torch.empty_like(ends)
        starts[:1] = 0
        starts[1:] = ends[:-1] + 1
        uv = torch.empty(n, dtype=torch.int32, device=dev)
        iv = torch.empty(n, dtype=torch.int32, device=dev)
        sv = torch.empty(n, dtype=torch.float64, device=dev)
        tv = torch.empty(n, dtype=torch.int64, device=dev)
        bad = torch.empty(n, dtype=torch.uint8, device=dev)
        n_bad = torch.zeros(1, dtype=torch.int32, device=dev)
        native.check(lib.oryx_rating_lines(
            text.data_ptr(), starts.data_ptr(), ends.data_ptr(), n, _NO_TS, uv.data_ptr(),
            iv.data_ptr(), sv.data_ptr(), tv.data_ptr(), bad.data_ptr(), n_bad.data_ptr(),
            native.stream_ptr(dev)), "oryx_rating_lines")
        del text, starts, ends, bad
        if int(n_bad.item()):
            return None
        users, items = ingest.IdDict(), ingest.IdDict()
        cu, ku = _first_appearance_codes(uv)
        ci, ki = _first_appearance_codes(iv)
        users.encode_nums(ku.cpu().numpy())
        items.encode_nums(ki.cpu().numpy())
        return _Segment(users, items, cu, ci, sv, tv, nbytes)

    def parse_ratings(self, lines, users: ingest.IdDict, items: ingest.IdDict,
                      default_ts: int, device_out: bool = False):
        """Same results as ``ingest.parse_ratings(lines, users, items, default_ts)`` (codes in
        first-appearance order appended to ``users`` / ``items``), reusing the parse of every
        keyed segment seen before.  ``device_out``: the columns stay tensors on the history's
        device (user / item int64, strength fp64, timestamp int64) instead of host arrays."""
        if not isinstance(lines, TextLines):
            out = ingest.parse_ratings(lines, users, items, default_ts)
            if device_out and self.device.type == "cuda":
                return tuple(torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
                             for a in out)
            return out
        buf = lines.joined()
        off = 0
        keyed = set()
        cols = []
        for key, n_lines, nbytes in lines.segment_list():
            if nbytes == 0:
                continue
            sg = self._segs.get(key) if key is not None else None
            if sg is not None and sg.nbytes == nbytes:
                self.stats["hits"] += 1
                self.stats["hit_bytes"] += nbytes
                self._segs.move_to_end(key)
            else:
                dg = self._digest(buf, off, nbytes) \
                    if nbytes >= self.UNKEYED_MIN_BYTES else None
                sg = self._unkeyed.get(dg) if (dg is not None and key is not None) else None
                if sg is not None:
                    # this part file holds the bytes of an interval parsed as new data
                    self.stats["adopted"] += 1
                    self.stats["hit_bytes"] += nbytes
                    del self._unkeyed[dg]
                else:
                    sg = self._parse_range(buf, off, nbytes, n_lines)
                    self.stats["misses"] += 1
                    self.stats["parsed_bytes"] += nbytes
                    if key is None and dg is not None:
                        self._unkeyed[dg] = sg
                        while len(self._unkeyed) > self.UNKEYED_KEEP:
                            self._unkeyed.popitem(last=False)
                if key is not None:
                    self._segs[key] = sg
            if key is not None:
                keyed.add(key)
            off += nbytes
            mu = torch.from_numpy(users.merge_from(sg.users)).to(self.device)
            mi = torch.from_numpy(items.merge_from(sg.items)).to(self.device)
            if sg.u.numel():
                cols.append((mu[sg.u.long()], mi[sg.i.long()], sg.s, sg.ts))
        # aged-out part files (no longer among the past data) leave the cache -- also when
        # none of this generation's input is keyed (every past file aged out, or past data
        # without file identities): the cache must never pin segments nothing names
        for k in [k for k in self._segs if k not in keyed]:
            del self._segs[k]
        if not cols:
            e = np.zeros(0, dtype=np.int64)
            out = e, e.copy(), np.zeros(0, dtype=np.float64), e.copy()
            if device_out and self.device.type == "cuda":
                return tuple(torch.from_numpy(a).to(self.device) for a in out)
            return out
        u = torch.cat([c[0] for c in cols])
        i = torch.cat([c[1] for c in cols])
        s = torch.cat([c[2] for c in cols])
        ts = torch.cat([c[3] for c in cols])
        ts = torch.where(ts == _NO_TS, torch.full_like(ts, int(default_ts)), ts)
        if device_out and self.device.type == "cuda":
            return u, i, s, ts
        return u.cpu().numpy(), i.cpu().numpy(), s.cpu().numpy(), ts.cpu().numpy()
