"""Device CSV kernels alone (csv.hip: one thread per line vs one wave per line) on k-means-
shaped lines (D "%.6f" values), timed with device events over repetitions, for several line
counts: where the parse time of a speed-layer micro-batch goes.

    python scripts/csv_kernel_probe.py [--dims 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", type=int, default=256)
    args = ap.parse_args()
    import numpy as np
    import torch
    from oryx_amd import native
    from oryx_amd.textlines import TextLines
    lib = native.require_kernels()
    dev = torch.device("cuda:0")
    g = np.random.default_rng(3)
    res = []
    for n in (1000, 10000, 100000):
        lines = [",".join("%.6f" % v for v in row) for row in g.standard_normal((n, args.dims))]
        tl = TextLines.from_strings(lines)
        buf = np.frombuffer(bytes(tl.joined()), dtype=np.uint8)
        nbytes = buf.nbytes
        text = torch.zeros(((nbytes + 31) // 16) * 16, dtype=torch.uint8, device=dev)
        text[:nbytes] = torch.from_numpy(buf).to(dev)
        ends = np.flatnonzero(buf == 10).astype(np.int64)
        d_ends = torch.from_numpy(ends).to(dev)
        d_starts = torch.empty_like(d_ends)
        d_starts[0] = 0
        d_starts[1:] = d_ends[:-1] + 1
        F = args.dims
        out_col = torch.arange(F, dtype=torch.int32, device=dev)
        is_num = torch.ones(F, dtype=torch.uint8, device=dev)
        slot = torch.full((F,), -1, dtype=torch.int32, device=dev)
        out = torch.empty((n, F), dtype=torch.float64, device=dev)
        sp_off = torch.empty((n, 1), dtype=torch.int64, device=dev)
        sp_len = torch.empty((n, 1), dtype=torch.int32, device=dev)
        bad = torch.empty(n, dtype=torch.uint8, device=dev)
        n_bad = torch.zeros(1, dtype=torch.int32, device=dev)
        st = native.stream_ptr(dev)

        def thread_k():
            return lib.oryx_csv_lines_to_matrix(
                text.data_ptr(), d_starts.data_ptr(), d_ends.data_ptr(), n, F, is_num.data_ptr(),
                out_col.data_ptr(), F, out.data_ptr(), 1, sp_off.data_ptr(), sp_len.data_ptr(),
                0, bad.data_ptr(), n_bad.data_ptr(), st)

        def wide_k():
            return lib.oryx_csv_wide_lines_to_matrix(
                text.data_ptr(), d_starts.data_ptr(), d_ends.data_ptr(), n, F, out_col.data_ptr(),
                F, out.data_ptr(), 1, slot.data_ptr(), sp_off.data_ptr(), sp_len.data_ptr(), 0,
                bad.data_ptr(), n_bad.data_ptr(), st)

        row = {"lines": n, "bytes": nbytes}
        for name, fn in (("thread", thread_k), ("wide", wide_k)):
            for _ in range(3):
                native.check(fn(), name)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            row[name + "_us"] = e0.elapsed_time(e1) / 20 * 1e3
        row["bad"] = int(n_bad.item())
        res.append(row)
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
