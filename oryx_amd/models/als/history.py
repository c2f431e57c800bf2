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
from collections import OrderedDict
from typing import Optional, Tuple

import numpy as np
import torch

from ... import ingest
from ...textlines import TextLines

log = logging.getLogger(__name__)

__all__ = ["RatingsHistory"]

_NO_TS = -(1 << 62)    # parse marker of a line without a timestamp (same as models/als/batch)


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
    def _parse_range(self, buf, off: int, nbytes: int, n_lines: int) -> _Segment:
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

    def parse_ratings(self, lines, users: ingest.IdDict, items: ingest.IdDict,
                      default_ts: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """Same results as ``ingest.parse_ratings(lines, users, items, default_ts)`` (codes in
        first-appearance order appended to ``users`` / ``items``), reusing the parse of every
        keyed segment seen before."""
        if not isinstance(lines, TextLines):
            return ingest.parse_ratings(lines, users, items, default_ts)
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
            return e, e.copy(), np.zeros(0, dtype=np.float64), e.copy()
        u = torch.cat([c[0] for c in cols])
        i = torch.cat([c[1] for c in cols])
        s = torch.cat([c[2] for c in cols])
        ts = torch.cat([c[3] for c in cols])
        ts = torch.where(ts == _NO_TS, torch.full_like(ts, int(default_ts)), ts)
        return u.cpu().numpy(), i.cpu().numpy(), s.cpu().numpy(), ts.cpu().numpy()
