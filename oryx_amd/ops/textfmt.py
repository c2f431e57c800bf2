"""Factor rows -> JSON array text, formatted where the rows live.

Model updates carry factor rows as JSON arrays of shortest round-trip floats (the reference
writes them with ``TextUtils.joinJSON``: ``[app-common]/als/ALSUtils`` callers in
``ALSUpdate.publishAdditionalModelData`` and ``ALSSpeedModelManager.java:182-215``).  Rows on
the GPU are converted by ``csrc/kernels/textfmt.hip`` (one wave per row, two launches) and only
the text crosses to the host; host rows use the native formatter of
``csrc/runtime/fastfloat.h``.  Both produce identical bytes.

:class:`RowText` holds the rows back to back (``blob``) with their end offsets; ``row(j)`` /
``rows()`` give Python strings, and the native message assemblers take the blob directly.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from .. import native

__all__ = ["RowText", "format_rows"]


@dataclass
class RowText:
    blob: object                # ASCII bytes or uint8 array, rows back to back
    ends: np.ndarray            # int64 [n]: end offset of row j

    def __len__(self) -> int:
        return len(self.ends)

    def rows(self) -> List[str]:
        text = str(memoryview(self.blob), "ascii")
        out, start = [], 0
        for e in self.ends.tolist():
            out.append(text[start:e])
            start = e
        return out

    def take(self, idx: np.ndarray) -> "RowText":
        """The rows ``idx`` (in that order) as a new :class:`RowText`."""
        idx = np.asarray(idx, dtype=np.int64)
        if len(idx) == 0:
            return RowText(b"", np.zeros(0, dtype=np.int64))
        starts = np.r_[0, self.ends[:-1]]
        buf = self.blob if isinstance(self.blob, np.ndarray) else \
            np.frombuffer(self.blob, dtype=np.uint8)
        lens = self.ends[idx] - starts[idx]
        parts = [buf[s:s + l] for s, l in zip(starts[idx].tolist(), lens.tolist())]
        return RowText(np.concatenate(parts).tobytes(), np.cumsum(lens))


def format_rows(mat) -> RowText:
    """JSON array text of every row of a 2-D float32 matrix (device tensor -> HIP kernels,
    host array / CPU tensor -> native host formatter)."""
    if isinstance(mat, torch.Tensor) and mat.device.type == "cuda":
        return _format_device(mat)
    if isinstance(mat, torch.Tensor):
        mat = mat.detach().numpy()
    from .. import ingest
    return ingest.format_float_rows_blob(np.asarray(mat, dtype=np.float32))


def _format_device(mat: torch.Tensor) -> RowText:
    m = mat.detach()
    if m.dtype != torch.float32:
        m = m.float()
    if m.dim() != 2:
        raise ValueError("need a 2-D matrix")
    if m.stride(1) != 1:
        m = m.contiguous()
    n, k = m.shape
    if n == 0:
        return RowText(b"", np.zeros(0, dtype=np.int64))
    lib = native.require_kernels()
    dev = m.device
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    stream = native.stream_ptr(dev)
    native.check(lib.oryx_format_rows_len(m.data_ptr(), n, k, m.stride(0), lens.data_ptr(),
                                          stream), "oryx_format_rows_len")
    ends = torch.cumsum(lens, 0, dtype=torch.int64)
    total = int(ends[-1])
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    native.check(lib.oryx_format_rows_text(m.data_ptr(), n, k, m.stride(0), ends.data_ptr(),
                                           lens.data_ptr(), out.data_ptr(), stream),
                 "oryx_format_rows_text")
    # pinned staging (torch's caching host allocator): one DMA, no page faults per call
    host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    host.copy_(out)
    return RowText(host.numpy(), ends.cpu().numpy())


_TEXT_WS = {}


def format_rows_and(mat: torch.Tensor, extra: torch.Tensor):
    """:func:`format_rows` of a device fp32 matrix with two host round trips in all: the
    text goes to a cached device buffer sized by the longest possible row (a float is at
    most 18 characters), and the row ends come back together with ``extra`` (a small device
    tensor, e.g. validity flags, returned as an int64 numpy array) before the one copy of the
    text.  Returns (RowText, extra on the host)."""
    m = mat.detach()
    if m.dtype != torch.float32 or m.dim() != 2 or m.stride(1) != 1 or m.device.type != "cuda":
        raise ValueError("need a row-contiguous 2-D float32 device matrix")
    n, k = m.shape
    if n == 0:
        return RowText(b"", np.zeros(0, dtype=np.int64)), extra.cpu().numpy().astype(np.int64)
    lib = native.require_kernels()
    dev = m.device
    stream = native.stream_ptr(dev)
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    native.check(lib.oryx_format_rows_len(m.data_ptr(), n, k, m.stride(0), lens.data_ptr(),
                                          stream), "oryx_format_rows_len")
    ends = torch.cumsum(lens, 0, dtype=torch.int64)
    bound = n * (19 * k + 2)
    ws = _TEXT_WS.get(dev)
    if ws is None or ws.numel() < bound:
        ws = torch.empty(bound, dtype=torch.uint8, device=dev)
        _TEXT_WS[dev] = ws
    native.check(lib.oryx_format_rows_text(m.data_ptr(), n, k, m.stride(0), ends.data_ptr(),
                                           lens.data_ptr(), ws.data_ptr(), stream),
                 "oryx_format_rows_text")
    small = torch.cat([ends, extra.reshape(-1).to(torch.int64)]).cpu().numpy()
    total = int(small[n - 1])
    host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    host.copy_(ws[:total])
    return RowText(host.numpy(), small[:n]), small[n:]


class DeviceRowText:
    """Rows formatted by :func:`format_rows_device`: the text still on the device, its row
    ends on the host, and a pinned host buffer of the text's size that :meth:`fetch` fills
    range by range (so a consumer can start on the first rows while later ones copy)."""

    def __init__(self, ws: torch.Tensor, ends: np.ndarray):
        self.ws = ws
        self.ends = ends
        total = int(ends[-1]) if len(ends) else 0
        self.host = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=True)
        self.blob = self.host.numpy()

    def fetch(self, ranges) -> None:
        """Copy the text of the row ranges [(lo, hi), ...] to the host buffer (one wait)."""
        for lo, hi in ranges:
            if hi <= lo:
                continue
            a = int(self.ends[lo - 1]) if lo else 0
            b = int(self.ends[hi - 1])
            if b > a:
                self.host[a:b].copy_(self.ws[a:b], non_blocking=True)
        torch.cuda.current_stream(self.ws.device).synchronize()

    def view(self, lo: int, hi: int) -> RowText:
        """RowText of rows [lo, hi) over the host buffer (offsets relative to row lo)."""
        a = int(self.ends[lo - 1]) if lo else 0
        return RowText(self.blob[a:int(self.ends[hi - 1]) if hi else a], self.ends[lo:hi] - a)


def format_rows_device(mat: torch.Tensor, extra: torch.Tensor, cache: Optional[dict] = None):
    """:func:`format_rows_and` without the text's copy: (DeviceRowText, extra on the host)
    after one small round trip (row ends + ``extra``).  ``cache``: the caller's own dict for
    the device text buffer (the text stays there while the caller fetches it, so it must not
    share the module's buffer with other formatting threads)."""
    m = mat.detach()
    if m.dtype != torch.float32 or m.dim() != 2 or m.stride(1) != 1 or m.device.type != "cuda":
        raise ValueError("need a row-contiguous 2-D float32 device matrix")
    n, k = m.shape
    lib = native.require_kernels()
    dev = m.device
    stream = native.stream_ptr(dev)
    lens = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    if n:
        native.check(lib.oryx_format_rows_len(m.data_ptr(), n, k, m.stride(0), lens.data_ptr(),
                                              stream), "oryx_format_rows_len")
    ends = torch.cumsum(lens[:n], 0, dtype=torch.int64)
    bound = max(n * (19 * k + 2), 1)
    wsc = cache if cache is not None else _TEXT_WS
    ws = wsc.get(dev)
    if ws is None or ws.numel() < bound:
        ws = torch.empty(bound, dtype=torch.uint8, device=dev)
        wsc[dev] = ws
    if n:
        native.check(lib.oryx_format_rows_text(m.data_ptr(), n, k, m.stride(0), ends.data_ptr(),
                                               lens.data_ptr(), ws.data_ptr(), stream),
                     "oryx_format_rows_text")
    small = torch.cat([ends, extra.reshape(-1).to(torch.int64)]).cpu().numpy()
    return DeviceRowText(ws, small[:n]), small[n:]


def format_csv(mat: torch.Tensor, pinned: bool = True) -> RowText:
    """CSV lines ``v0,v1,...\n`` of every row of a device float32 matrix (shortest round-trip
    float32 text, as :func:`format_rows`), formatted on the GPU; ``ends[r]`` is the end of row
    r's newline.  For generating batch-layer input (bench_batch.py)."""
    m = mat.detach()
    if m.dtype != torch.float32:
        m = m.float()
    if m.stride(1) != 1:
        m = m.contiguous()
    n, k = m.shape
    if n == 0:
        return RowText(b"", np.zeros(0, dtype=np.int64))
    lib = native.require_kernels()
    dev = m.device
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    stream = native.stream_ptr(dev)
    native.check(lib.oryx_format_csv_len(m.data_ptr(), n, k, m.stride(0), lens.data_ptr(),
                                         stream), "oryx_format_csv_len")
    ends = torch.cumsum(lens, 0, dtype=torch.int64)
    total = int(ends[-1])
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    native.check(lib.oryx_format_csv_text(m.data_ptr(), n, k, m.stride(0), ends.data_ptr(),
                                          lens.data_ptr(), out.data_ptr(), stream),
                 "oryx_format_csv_text")
    host = torch.empty(total, dtype=torch.uint8, pin_memory=pinned)
    host.copy_(out)
    return RowText(host.numpy(), ends.cpu().numpy())
