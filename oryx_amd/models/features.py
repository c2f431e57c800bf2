"""Feature rows of the k-means and RDF batch layers: native parse straight to a device matrix,
and the resident parsed history of past part files.

The reference parses every record of every generation inside Spark tasks
(``[mllib]/kmeans/KMeansUpdate.java:223-232`` ``parsedToVectorRDD``,
``[mllib]/rdf/RDFUpdate.java:228-260`` ``parseToLabeledPointRDD`` after
``getDistinctValues`` ``:207-225``).  Here one native, threaded pass
(``csrc/runtime/oryx_ingest.cpp`` ``oryx_csv_to_f32`` / ``_f64``) turns a buffer of CSV lines
into a float matrix -- numeric fields exactly parsed, empty numeric fields NaN -- and records
the byte spans of categorical fields, which are then encoded column by column with one
vectorised unique per column (codes in order of first appearance, as the reference's
encodings).

:class:`FeatureHistory` keeps each past part file's parse on the training device, keyed by
the file's identity (``layers.batch.read_past_data`` marks each part file's byte range with
``(path, size, mtime)``), with segment-local categorical codes; a generation merges the
segments' distinct values in segment order -- the first-appearance order one parse of the
concatenated text gives -- and remaps each segment's codes with one device gather.  The new
interval's parse is remembered under a hash of its bytes and adopted when the same bytes come
back as a part file, so in steady state every record is parsed once.

Lines the native parser does not take (quoted fields, backslash escapes, JSON arrays, a field
count other than the schema's) make the whole input go through the reference-compatible
Python parser instead (``utils.text.parse_input_line``).
"""

from __future__ import annotations

import ctypes
import logging
import os
import threading
import weakref
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ingest, native
from ..textlines import LineConcat, LineSelection, TextLines, _Lazy
from .schema import InputSchema

log = logging.getLogger(__name__)

__all__ = ["FeatureBlock", "FeatureHistory", "parse_features"]


@dataclass
class FeatureBlock:
    """Parsed feature rows: ``full`` [n, F] (numeric features as values, categorical ones as
    codes into ``values[f]``), on ``full.device``."""
    full: torch.Tensor
    values: Dict[int, List[str]] = field(default_factory=dict)

    def __len__(self) -> int:
        return int(self.full.shape[0])

    def predictors(self, schema: InputSchema) -> torch.Tensor:
        idx = list(schema.predictor_feature_indices)
        if idx and idx == list(range(idx[0], idx[0] + len(idx))):
            return self.full[:, idx[0]:idx[0] + len(idx)]
        return self.full[:, idx]

    def target(self, schema: InputSchema) -> torch.Tensor:
        if not schema.has_target():
            return torch.full((len(self),), float("nan"), dtype=self.full.dtype,
                              device=self.full.device)
        return self.full[:, schema.get_target_feature_index()]


@dataclass
class _Seg:
    full: torch.Tensor                 # categorical columns hold segment-local codes
    values: Dict[int, List[str]]       # categorical feature -> segment-local distinct values
    nbytes: int
    owned: bool = False                # ``full`` is this parse's own (not a cached tensor)
    ends: Optional[np.ndarray] = None  # the segment's '\n' offsets (when the parse had them)


def _buf_view(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return buf
    return np.frombuffer(bytes(buf), dtype=np.uint8)


def _native_block(buf: np.ndarray, off: int, nbytes: int, n_lines: int, schema: InputSchema,
                  dtype: torch.dtype) -> Optional[Tuple[np.ndarray, Dict[int, np.ndarray],
                                                       Dict[int, List[str]]]]:
    """(matrix [rows, F] with categorical columns as local codes, -, local distinct values) of
    bytes [off, off + nbytes) of ``buf``, or None when a line needs the general parser."""
    F = schema.get_num_features()
    is_num = np.array([0 if schema.is_categorical(f) else 1 for f in range(F)], dtype=np.uint8)
    cats = [f for f in range(F) if schema.is_categorical(f)]
    S = len(cats)
    out_col = np.arange(F, dtype=np.int32)
    np_dtype = np.float32 if dtype == torch.float32 else np.float64
    full = np.empty((max(n_lines, 1), F), dtype=np_dtype)
    span_off = np.empty((max(n_lines, 1), max(S, 1)), dtype=np.int64)
    span_len = np.empty((max(n_lines, 1), max(S, 1)), dtype=np.int32)
    lib = native.runtime()
    fn = lib.oryx_csv_to_f32 if np_dtype == np.float32 else lib.oryx_csv_to_f64
    base = buf.ctypes.data + off
    vp = ctypes.c_void_p
    got = fn(vp(base), int(nbytes), F, is_num.ctypes.data_as(vp), out_col.ctypes.data_as(vp), F,
             full.ctypes.data_as(vp), span_off.ctypes.data_as(vp), span_len.ctypes.data_as(vp),
             int(max(n_lines, 1)))
    if got < 0:
        return None
    n = int(got)
    full = full[:n]
    values, codes = _encode_spans(buf[off:off + nbytes], span_off[:n], span_len[:n], cats,
                                  np_dtype)
    for f in cats:
        full[:, f] = codes[f]
    return full, {}, values


def _encode_spans(seg: np.ndarray, span_off: np.ndarray, span_len: np.ndarray, cats,
                  np_dtype) -> Tuple[Dict[int, List[str]], Dict[int, np.ndarray]]:
    """Categorical codes of each span column (spans relative to ``seg``), in order of first
    appearance (empty = NaN): (distinct values, codes) per categorical feature."""
    n = span_off.shape[0]
    values: Dict[int, List[str]] = {}
    out_codes: Dict[int, np.ndarray] = {}
    if n and cats:
        # native: per-thread tables merged in row order (oryx_encode_spans)
        so = np.ascontiguousarray(span_off, dtype=np.int64)
        sl = np.ascontiguousarray(span_len, dtype=np.int32)
        S = so.shape[1]
        seg = np.ascontiguousarray(seg)
        lib = native.runtime()
        codes = np.empty(n, dtype=np.int64)
        first = np.empty(n, dtype=np.int64)
        for si, f in enumerate(cats):
            k = int(lib.oryx_encode_spans(seg.ctypes.data, so[:, si:].ctypes.data,
                                          sl[:, si:].ctypes.data, n, S, codes.ctypes.data,
                                          first.ctypes.data))
            rows = first[:k]
            o, ln = so[rows, si], sl[rows, si]
            values[f] = [bytes(seg[a:a + b]).decode("utf-8") for a, b in zip(o.tolist(),
                                                                            ln.tolist())]
            c = codes.astype(np_dtype)
            c[codes < 0] = np.nan
            out_codes[f] = c
        return values, out_codes
    for si, f in enumerate(cats):
        o = span_off[:, si]
        ln = span_len[:, si]
        L = int(ln.max()) if n else 0
        if L > 0:
            j = np.arange(L)
            g = seg[np.minimum(o[:, None] + j, max(len(seg) - 1, 0))]
            g[j >= ln[:, None]] = 0
            vals = np.ascontiguousarray(g).view("S%d" % L).ravel()
        else:
            vals = np.zeros(n, dtype="S1")
        uniq, first, inv = np.unique(vals, return_index=True, return_inverse=True)
        # local codes in order of first appearance (the reference's encoding order)
        order = np.argsort(first, kind="stable")
        rank = np.empty(len(uniq), dtype=np.int64)
        rank[order] = np.arange(len(uniq))
        codes = rank[inv.reshape(-1)].astype(np_dtype)
        names = [u.decode("utf-8") for u in uniq[order].tolist()]
        if "" in names:
            # an empty categorical value is missing (NaN), not a category
            e = names.index("")
            codes = np.where(codes == e, np.nan, np.where(codes > e, codes - 1, codes))
            names = names[:e] + names[e + 1:]
        out_codes[f] = codes
        values[f] = names
    return values, out_codes


def _device_ok(schema: InputSchema, device) -> bool:
    """The device parser applies: a GPU, the kernels built, not switched off (ORYX_GPU_CSV=0)."""
    import os
    if device.type != "cuda" or os.environ.get("ORYX_GPU_CSV", "1") == "0":
        return False
    return native.kernels_available()


_STAGE_BYTES = 64 << 20
_STAGES = 3


def h2d(buf: np.ndarray, off: int, nbytes: int, dst: torch.Tensor,
        staged: Optional[bool] = None) -> None:
    """``buf[off:off + nbytes]`` (pageable host memory) into ``dst[:nbytes]`` on the GPU.

    Plain ``copy_`` by default: the HIP runtime moves pageable memory at 56 GB/s on the
    MI355X box (profiles/r5_h2d_v2.json).  ``staged`` / ``ORYX_H2D_STAGED=1``: 64 MB pieces
    copied into pinned staging buffers by the native threads (``oryx_concat_buffers``) and
    DMA'd from there, the next piece's copy overlapping the current DMA -- measured at the same
    56 GB/s, so it stays off."""
    import os
    if staged is None:
        staged = os.environ.get("ORYX_H2D_STAGED", "0") == "1"
    src = buf[off:off + nbytes]
    if not staged or nbytes < 2 * _STAGE_BYTES or dst.device.type != "cuda":
        dst[:nbytes].copy_(torch.from_numpy(src))
        return
    lib = native.runtime()
    stream = torch.cuda.current_stream(dst.device)
    stages = [torch.empty(_STAGE_BYTES, dtype=torch.uint8, pin_memory=True)
              for _ in range(_STAGES)]
    events: List[Optional[torch.cuda.Event]] = [None] * _STAGES
    ptrs = np.zeros(1, dtype=np.uint64)
    lens = np.zeros(1, dtype=np.int64)
    base = src.ctypes.data
    for i, lo in enumerate(range(0, nbytes, _STAGE_BYTES)):
        n = min(_STAGE_BYTES, nbytes - lo)
        j = i % _STAGES
        if events[j] is not None:
            events[j].synchronize()          # the DMA out of this staging buffer is done
        ptrs[0] = base + lo
        lens[0] = n
        lib.oryx_concat_buffers(ptrs.ctypes.data, lens.ctypes.data, 1, stages[j].data_ptr())
        dst[lo:lo + n].copy_(stages[j][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        events[j] = ev
    # (the caching pinned allocator holds each staging block until its last copy completes)


# average line length from which the device parse takes a wave per line instead of a thread
# (ORYX_CSV_WIDE_MIN_BYTES; a huge value keeps the thread kernel), for up to WIDE_MAX_LINES
# lines (ORYX_CSV_WIDE_MAX_LINES).  At 256 "%.6f" values per line the wave kernel parses 10k
# lines in 67 us and 100k in 584 us, the thread kernel in 1043 / 1834 us
# (profiles/r6_csv_kernel_probe_v2.jsonl, scripts/csv_kernel_probe.py)
WIDE_LINE_MIN_BYTES = int(os.environ.get("ORYX_CSV_WIDE_MIN_BYTES", "192"))
WIDE_MAX_LINES = int(os.environ.get("ORYX_CSV_WIDE_MAX_LINES", str(1 << 62)))


def _device_block(buf: np.ndarray, off: int, nbytes: int, n_lines: int, schema: InputSchema,
                  dtype: torch.dtype, device, laps: Optional[Dict[str, float]] = None
                  ) -> Optional[Tuple[torch.Tensor, Dict[int, List[str]]]]:
    """Bytes [off, off + nbytes) of ``buf`` parsed on the device (``csv.hip``): the text goes
    to the GPU (smaller than its parse) and one thread per line parses it with the host
    parser's exact fast path; the [rows, F] matrix never exists on the host.  Lines outside
    that form are parsed on the host and their rows written in (bitwise the host parser's).
    Categorical fields come back as byte spans and are encoded on the host.  Returns (matrix,
    categorical values), or None when the caller should parse on the host instead."""
    import time
    t_last = [time.perf_counter()]

    def lap(name):
        if laps is not None:
            t = time.perf_counter()
            laps[name] = laps.get(name, 0.0) + t - t_last[0]
            t_last[0] = t

    F = schema.get_num_features()
    cats = [f for f in range(F) if schema.is_categorical(f)]
    S = len(cats)
    if nbytes == 0:
        return torch.zeros((0, F), dtype=dtype, device=device), {f: [] for f in cats}, \
            np.zeros(0, dtype=np.int64)
    # the line ends are found by the native threads while the text goes up to the device
    scan = _LineEnds(buf, off, nbytes, n_lines)
    text = torch.empty(((nbytes + 31) // 16) * 16, dtype=torch.uint8, device=device)
    h2d(buf, off, nbytes, text)
    lap("h2d")
    ends = scan.result()
    n = len(ends)
    if n == 0:
        return torch.zeros((0, F), dtype=dtype, device=device), {f: [] for f in cats}, ends
    d_ends = torch.from_numpy(ends).to(device)
    d_starts = torch.empty_like(d_ends)
    d_starts[0] = 0
    d_starts[1:] = d_ends[:-1] + 1
    lap("line_scan")
    out_col = torch.arange(F, dtype=torch.int32, device=device)
    is_num = torch.tensor([0 if f in cats else 1 for f in range(F)], dtype=torch.uint8,
                          device=device)
    out = torch.empty((n, F), dtype=dtype, device=device)
    sp_off = torch.empty((n, max(S, 1)), dtype=torch.int64, device=device)
    sp_len = torch.empty((n, max(S, 1)), dtype=torch.int32, device=device)
    bad = torch.empty(n, dtype=torch.uint8, device=device)
    n_bad = torch.zeros(1, dtype=torch.int32, device=device)
    lib = native.require_kernels()
    if nbytes >= WIDE_LINE_MIN_BYTES * n and n <= WIDE_MAX_LINES:
        # long lines: one wave per line (csv.hip csv_wide_kernel)
        slot = torch.tensor([cats.index(f) if f in cats else -1 for f in range(F)],
                            dtype=torch.int32, device=device)
        native.check(lib.oryx_csv_wide_lines_to_matrix(
            text.data_ptr(), d_starts.data_ptr(), d_ends.data_ptr(), n, F, out_col.data_ptr(),
            F, out.data_ptr(), int(dtype == torch.float64), slot.data_ptr(), sp_off.data_ptr(),
            sp_len.data_ptr(), S, bad.data_ptr(), n_bad.data_ptr(), native.stream_ptr(device)),
            "oryx_csv_wide_lines_to_matrix")
    else:
        native.check(lib.oryx_csv_lines_to_matrix(
            text.data_ptr(), d_starts.data_ptr(), d_ends.data_ptr(), n, F, is_num.data_ptr(),
            out_col.data_ptr(), F, out.data_ptr(), int(dtype == torch.float64),
            sp_off.data_ptr(), sp_len.data_ptr(), S, bad.data_ptr(), n_bad.data_ptr(),
            native.stream_ptr(device)), "oryx_csv_lines_to_matrix")
    values: Dict[int, List[str]] = {}
    bad_lines = int(n_bad.item())
    lap("kernel")
    if bad_lines:
        if S:
            return None     # (the host subset's local categories would need a re-encode)
        idx = torch.nonzero(bad).flatten().cpu().numpy()
        starts = np.empty(n, dtype=np.int64)
        starts[0] = 0
        starts[1:] = ends[:-1] + 1
        if (ends[idx] == starts[idx]).any():
            return None                 # an empty line: the host parser skips it (row count)
        sub = TextLines(buf[off:off + nbytes], n, ends).take(idx)
        got = _native_block(np.ascontiguousarray(sub.joined()), 0, sub.nbytes(), len(idx),
                            schema, dtype)
        if got is None or got[0].shape[0] != len(idx):
            return None
        out[torch.from_numpy(idx).to(device)] = torch.from_numpy(got[0]).to(device)
        lap("host_lines")
    if S:
        np_dtype = np.float32 if dtype == torch.float32 else np.float64
        values, codes = _encode_spans(buf[off:off + nbytes], sp_off.cpu().numpy(),
                                      sp_len.cpu().numpy(), cats, np_dtype)
        for f in cats:
            out[:, f] = torch.from_numpy(codes[f]).to(device)
        lap("categorical")
    return out, values, ends


def _python_block(lines: Sequence[str], schema: InputSchema, dtype: torch.dtype
                  ) -> Tuple[np.ndarray, Dict[int, List[str]]]:
    """The general parser (``parse_input_line``: quotes, escapes, JSON arrays)."""
    from ..utils import text
    F = schema.get_num_features()
    # (a CRLF line's CR is not part of its last field, as for the native parsers)
    rows = [text.parse_input_line(l[:-1] if l.endswith("\r") else l) for l in lines]
    rows = [r for r in rows if r is not None]
    np_dtype = np.float32 if dtype == torch.float32 else np.float64
    full = np.empty((len(rows), F), dtype=np_dtype)
    values: Dict[int, List[str]] = {}
    for f in range(F):
        col = [r[f] if f < len(r) else "" for r in rows]
        if schema.is_categorical(f):
            seen: Dict[str, int] = {}
            codes = []
            for v in col:
                if v == "":
                    codes.append(np.nan)
                    continue
                codes.append(seen.setdefault(v, len(seen)))
            full[:, f] = np.asarray(codes, dtype=np.float64)
            values[f] = list(seen.keys())
        elif schema.is_numeric(f):
            full[:, f] = [float(v) if v != "" else np.nan for v in col]
        else:
            full[:, f] = np.nan
    return full, values


def _merge(segs: List[_Seg], schema: InputSchema, device) -> FeatureBlock:
    F = schema.get_num_features()
    cats = [f for f in range(F) if schema.is_categorical(f)]
    if not segs:
        return FeatureBlock(torch.zeros((0, F), device=device), {f: [] for f in cats})
    if len(segs) > 1:
        full = torch.cat([sg.full for sg in segs])
    else:
        full = segs[0].full if segs[0].owned else segs[0].full.clone()
    values: Dict[int, List[str]] = {}
    for f in cats:
        index: Dict[str, int] = {}
        pos = 0
        for sg in segs:
            local = sg.values.get(f, [])
            remap = np.array([index.setdefault(v, len(index)) for v in local], dtype=np.float64)
            n = int(sg.full.shape[0])
            if len(local) and not np.array_equal(remap, np.arange(len(local))):
                col = full[pos:pos + n, f]
                ok = ~torch.isnan(col)
                m = torch.from_numpy(remap).to(device, full.dtype)
                col[ok] = m[col[ok].long()]
            pos += n
        values[f] = list(index.keys())
    return FeatureBlock(full, values)


def _select_rows(parent: _Seg, index: np.ndarray, cats: List[int], device) -> _Seg:
    """Rows ``index`` of a parsed block, categorical codes renumbered in their order of first
    appearance among those rows (what a parse of just those lines assigns)."""
    full = parent.full.index_select(0, torch.from_numpy(index).to(device))
    values: Dict[int, List[str]] = {}
    for f in cats:
        pv = parent.values.get(f, [])
        col = full[:, f]
        ok = ~torch.isnan(col)
        c = col[ok].long()
        if not pv or c.numel() == 0:
            values[f] = []
            continue
        n = c.numel()
        first = torch.full((len(pv),), n, dtype=torch.int64, device=device)
        first.scatter_reduce_(0, c, torch.arange(n, device=device), reduce="amin")
        present = torch.nonzero(first < n).flatten()
        order = present[torch.argsort(first[present])]
        remap = torch.full((len(pv),), -1, dtype=torch.int64, device=device)
        remap[order] = torch.arange(order.numel(), device=device)
        col[ok] = remap[c].to(full.dtype)
        values[f] = [pv[i] for i in order.tolist()]
    return _Seg(full, values, 0, owned=True)


class _Digest(threading.Thread):
    """``ingest.content_digest`` of a byte range on a thread of its own (the native hash runs
    without the GIL, beside the parse of the same bytes), and of the part files the batch
    layer saves it as (``textlines.part_edges``): ``result()`` -> (digest, [(edge0, edge1,
    digest)] or [])."""

    def __init__(self, buf: np.ndarray, off: int, nbytes: int):
        super().__init__(daemon=True)
        self._args = (buf, off, nbytes)
        self._out = None
        self._err: Optional[BaseException] = None
        self.start()

    def run(self) -> None:
        try:
            from ..textlines import part_edges
            buf, off, nbytes = self._args
            whole = ingest.content_digest(buf, off, nbytes)
            edges = part_edges(buf[off:off + nbytes])
            chunks = [(a, b, ingest.content_digest(buf, off + a, b - a))
                      for a, b in zip(edges[:-1], edges[1:])] if len(edges) > 2 else []
            self._out = (whole, chunks)
        except BaseException as e:   # re-raised in result()
            self._err = e

    def result(self):
        self.join()
        if self._err is not None:
            raise self._err
        return self._out


class _LineEnds(threading.Thread):
    """The ``'\n'`` offsets of ``buf[off:off + nbytes]`` (native threaded scan) on a thread of
    its own, beside the text's upload to the device."""

    def __init__(self, buf: np.ndarray, off: int, nbytes: int, n_lines: int):
        super().__init__(daemon=True)
        self._args = (buf, off, nbytes, n_lines)
        self._out: Optional[np.ndarray] = None
        self._err: Optional[BaseException] = None
        self.start()

    def run(self) -> None:
        try:
            buf, off, nbytes, n_lines = self._args
            lib = native.runtime()
            cap = max(1, n_lines or nbytes // 8)
            while True:
                ends = np.empty(cap, dtype=np.int64)
                got = lib.oryx_line_ends(ctypes.c_void_p(buf.ctypes.data + off), int(nbytes),
                                         ends.ctypes.data, cap)
                if got >= 0:
                    self._out = ends[:got]
                    return
                cap = -got
        except BaseException as e:   # re-raised in result()
            self._err = e

    def result(self) -> np.ndarray:
        self.join()
        if self._err is not None:
            raise self._err
        return self._out


# parse of the parent of LineSelections (the interval a train / test split selects from),
# shared by the train parse and the evaluation's test parse of one generation:
# (id(parent), schema key, device) -> (weak reference to the parent, its parse)
_SELECTION_PARENTS: "Dict[tuple, Tuple[weakref.ref, _Seg]]" = {}


def parse_features(lines, schema: InputSchema, device, dtype: torch.dtype = torch.float32,
                   history: Optional["FeatureHistory"] = None) -> FeatureBlock:
    """All records -> :class:`FeatureBlock` on ``device`` (see the module docstring)."""
    if history is not None:
        return history.parse(lines, schema, dtype)
    return FeatureHistory(device, keep=False).parse(lines, schema, dtype)


class FeatureHistory:
    """Parse cache of keyed :class:`TextLines` segments of feature rows (module docstring).
    ``keep=False``: a one-off parse (nothing is cached)."""

    UNKEYED_MIN_BYTES = 1 << 20
    UNKEYED_KEEP = 4

    def __init__(self, device=None, keep: bool = True):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.keep = keep
        self._segs: "OrderedDict[tuple, _Seg]" = OrderedDict()
        self._unkeyed: "OrderedDict[bytes, _Seg]" = OrderedDict()
        # part-file digest -> (digest of the unkeyed parse it is a byte range of, first row,
        # end row): a large interval is saved as several part files (layers/batch.py)
        self._unkeyed_chunks: Dict[bytes, Tuple[bytes, int, int]] = {}
        self._schema_key = None
        self.stats = {"hits": 0, "misses": 0, "hit_bytes": 0, "parsed_bytes": 0, "adopted": 0}

    def __len__(self) -> int:
        return len(self._segs)

    def resident_bytes(self) -> int:
        segs = list(self._segs.values()) + list(self._unkeyed.values())
        return sum(int(sg.full.numel()) * sg.full.element_size() for sg in segs)

    def clear(self) -> None:
        self._segs.clear()
        self._unkeyed.clear()
        self._unkeyed_chunks.clear()

    @staticmethod
    def _digest(buf: np.ndarray, off: int, nbytes: int) -> Optional[bytes]:
        return ingest.content_digest(buf, off, nbytes)

    def _parse_range(self, buf: np.ndarray, off: int, nbytes: int, n_lines: int,
                     schema: InputSchema, dtype) -> Optional[_Seg]:
        if _device_ok(schema, self.device):
            got = _device_block(buf, off, nbytes, n_lines, schema, dtype, self.device,
                                self.stats.setdefault("device_parse_s", {}))
            if got is not None:
                self.stats["device_parsed_bytes"] = \
                    self.stats.get("device_parsed_bytes", 0) + nbytes
                return _Seg(got[0], got[1], nbytes, ends=got[2])
        got = _native_block(buf, off, nbytes, n_lines, schema, dtype)
        if got is None:
            return None
        full, _, values = got
        return _Seg(torch.from_numpy(full).to(self.device), values, nbytes)

    def parse(self, lines, schema: InputSchema, dtype=torch.float32) -> FeatureBlock:
        key_s = (tuple(schema.feature_names), tuple(schema.is_categorical(f) for f in
                                                    range(schema.get_num_features())), dtype)
        if self._schema_key != key_s:
            self.clear()
            self._schema_key = key_s
        if not isinstance(lines, TextLines):
            lines = TextLines.from_strings([l for l in lines]) if len(lines) else \
                TextLines(b"", 0)
        parts = lines.parts if isinstance(lines, LineConcat) else [lines]
        segs: List[_Seg] = []
        keyed: set = set()
        for part in parts:
            sg = self._selection(part, schema, dtype, key_s, keyed) \
                if isinstance(part, LineSelection) else None
            if sg is not None:
                segs.append(sg)
                continue
            if isinstance(part, _Lazy):
                part = part.materialize()
            got = self._text_segs(part, schema, dtype, keyed)
            if got is None:
                # a line the native parser does not take: the general parser for all
                full, values = _python_block(list(lines), schema, dtype)
                blk = FeatureBlock(torch.from_numpy(full).to(self.device), {})
                blk.values = values
                return blk
            segs.extend(got)
        if self.keep:
            for k in [k for k in self._segs if k not in keyed]:
                del self._segs[k]
        return _merge(segs, schema, self.device)

    def _add_chunks(self, dg: bytes, sg: _Seg, chunks, buf: np.ndarray, off: int,
                    nbytes: int) -> None:
        """Remember the part files an unkeyed parse will come back as (row ranges by the
        segment's line ends)."""
        if not chunks:
            return
        ends = sg.ends
        if ends is None:
            ends = TextLines(buf[off:off + nbytes]).ends()
        if len(ends) != int(sg.full.shape[0]):
            return                     # (lines the parser dropped: rows and lines differ)
        for a, b, cdg in chunks:
            lo = int(np.searchsorted(ends, a, side="left"))
            hi = int(np.searchsorted(ends, b, side="left"))
            self._unkeyed_chunks[cdg] = (dg, lo, hi)

    def _drop_chunks(self, dg: bytes) -> None:
        for k in [k for k, v in self._unkeyed_chunks.items() if v[0] == dg]:
            del self._unkeyed_chunks[k]

    def _adopt_chunk(self, cdg: bytes, schema: InputSchema) -> _Seg:
        """A part file that is a byte range of a remembered unkeyed parse: its rows (codes
        renumbered as a parse of the file alone numbers them); the parse is released once its
        last part file is adopted."""
        dg, lo, hi = self._unkeyed_chunks.pop(cdg)
        parent = self._unkeyed[dg]
        cats = [f for f in range(schema.get_num_features()) if schema.is_categorical(f)]
        sg = _select_rows(parent, np.arange(lo, hi, dtype=np.int64), cats, self.device)
        if not any(v[0] == dg for v in self._unkeyed_chunks.values()):
            del self._unkeyed[dg]
        return sg

    def _selection(self, part: LineSelection, schema: InputSchema, dtype, key_s,
                   keyed: set) -> Optional[_Seg]:
        """A train / test selection: its rows of the parent's parse (parsed once per parent
        and shared through ``_SELECTION_PARENTS``), or None to parse its own text."""
        parent = part.parent
        if isinstance(parent, _Lazy) or not len(part):
            return None
        mk = (id(parent), key_s, str(self.device))
        hit = _SELECTION_PARENTS.get(mk)
        psg = hit[1] if hit is not None and hit[0]() is parent else None
        if psg is None:
            got = self._text_segs(parent, schema, dtype, keyed)
            if not got:
                return None
            blk = _merge(got, schema, self.device)
            if int(blk.full.shape[0]) != len(parent):
                return None       # (an empty line the parser skips: rows and lines differ)
            psg = _Seg(blk.full, blk.values, parent.nbytes())
            for k in [k for k, v in _SELECTION_PARENTS.items() if v[0]() is None]:
                del _SELECTION_PARENTS[k]
            ref = weakref.ref(parent, lambda _r, mk=mk: _SELECTION_PARENTS.pop(mk, None))
            _SELECTION_PARENTS[mk] = (ref, psg)
        else:
            self.stats["selection_hits"] = self.stats.get("selection_hits", 0) + 1
        cats = [f for f in range(schema.get_num_features()) if schema.is_categorical(f)]
        return _select_rows(psg, part.index, cats, self.device)

    def _text_segs(self, lines: TextLines, schema: InputSchema, dtype,
                   keyed: set) -> Optional[List[_Seg]]:
        """The parse of each byte segment of ``lines`` (cached ones reused, keyed ones added to
        ``keyed``), or None when a line needs the general parser."""
        buf = _buf_view(lines.joined())
        segs: List[_Seg] = []
        off = 0
        for key, n_lines, nbytes in lines.segment_list():
            if nbytes == 0:
                continue
            sg = self._segs.get(key) if (key is not None and self.keep) else None
            if sg is not None and sg.nbytes == nbytes:
                self.stats["hits"] += 1
                self.stats["hit_bytes"] += nbytes
                self._segs.move_to_end(key)
            else:
                dg, pending = None, None
                if self.keep and nbytes >= self.UNKEYED_MIN_BYTES:
                    if key is not None:     # (the adoption lookup needs it first)
                        dg = self._digest(buf, off, nbytes)
                    else:                   # (only stored: hashed beside the parse)
                        pending = _Digest(buf, off, nbytes)
                sg = self._unkeyed.get(dg) if (dg is not None and key is not None) else None
                if sg is not None:
                    self.stats["adopted"] += 1
                    self.stats["hit_bytes"] += nbytes
                    del self._unkeyed[dg]
                    self._drop_chunks(dg)
                elif dg is not None and key is not None and dg in self._unkeyed_chunks:
                    sg = self._adopt_chunk(dg, schema)
                    sg.nbytes = nbytes        # (cached under the part file's key from now on)
                    sg.owned = False
                    self.stats["adopted"] += 1
                    self.stats["hit_bytes"] += nbytes
                else:
                    sg = self._parse_range(buf, off, nbytes, n_lines, schema, dtype)
                    chunks = []
                    if pending is not None:
                        dg, chunks = pending.result()
                    if sg is None:
                        return None
                    self.stats["misses"] += 1
                    self.stats["parsed_bytes"] += nbytes
                    if key is None and dg is not None:
                        self._unkeyed[dg] = sg
                        self._add_chunks(dg, sg, chunks, buf, off, nbytes)
                        while len(self._unkeyed) > self.UNKEYED_KEEP:
                            old, _ = self._unkeyed.popitem(last=False)
                            self._drop_chunks(old)
                if key is not None and self.keep:
                    self._segs[key] = sg
            if key is not None:
                keyed.add(key)
            segs.append(sg)
            off += nbytes
        return segs
