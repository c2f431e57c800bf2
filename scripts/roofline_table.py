"""Per-half-step roofline table of the ALS solve kernels from the rocprofv3 passes of
scripts/archive/r5_roofline.sh (rank 64 bf16 c2, rank 128 fp32; 25M ratings, 162,541 users, 59,047
items).  Writes profiles/r5_als_roofline.json and profiles/r5_als_roofline.md.

Half-steps: the solve kernel's dispatches alternate items, users (MLlib order) from the first
one on; every iteration of the run (warm-up, timed, phase breakdown) contributes.  Per
half-step the table gives the mean kernel time (unprofiled trace run), the MFMA FLOPs the
kernel executes (Gramian tiles per rating and the block LDL^T's K / trailing tiles per row,
counted from the kernel's loop structure), the HBM bytes (FETCH_SIZE x 1024 x 2: on gfx950
FETCH_SIZE reports half of what a wide coalesced stream fetches), MFMA and VALU busy from
the SQ counters, and achieved against the dense peaks (2.5 PFLOP/s bf16, 157 TFLOP/s fp32,
8 TB/s HBM3E).

Usage: python scripts/roofline_table.py [gpurun_out dir]
"""

import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
SIMDS = 1024                   # 256 CUs x 4
XCDS = 8
PEAK = {"bf16": 2.5e15, "fp32": 157e12, "hbm": 8e12}
RATINGS, USERS, ITEMS = 25_000_000, 162_541, 59_047


def _find(d, suffix):
    for base, _, files in os.walk(d):
        for f in files:
            if f.endswith(suffix):
                return os.path.join(base, f)
    raise FileNotFoundError(d + " " + suffix)


def _is_solve(name):
    return "als_solve_batch" in name


def counters(name):
    """{half: {counter: summed value}} of the solve kernel's dispatches."""
    per_dispatch = defaultdict(dict)
    kname = {}
    with open(_find(os.path.join(OUT, name), "counter_collection.csv")) as fh:
        for row in csv.DictReader(fh):
            if not _is_solve(row["Kernel_Name"]):
                continue
            d = int(row["Dispatch_Id"])
            per_dispatch[d][row["Counter_Name"]] = float(row["Counter_Value"])
            kname[d] = (row["Kernel_Name"], int(row["VGPR_Count"]), int(row["Accum_VGPR_Count"]),
                        int(row["LDS_Block_Size"]))
    out = {"items": defaultdict(float), "users": defaultdict(float)}
    n = {"items": 0, "users": 0}
    for j, d in enumerate(sorted(per_dispatch)):
        half = "items" if j % 2 == 0 else "users"
        n[half] += 1
        for c, v in per_dispatch[d].items():
            out[half][c] += v
    meta = next(iter(kname.values())) if kname else None
    return {h: {c: v / max(1, n[h]) for c, v in out[h].items()} for h in out}, meta


def times(name):
    """{half: mean solve-kernel ms} from an unprofiled kernel trace."""
    rows = []
    with open(_find(os.path.join(OUT, name), "kernel_trace.csv")) as fh:
        for row in csv.DictReader(fh):
            if _is_solve(row["Kernel_Name"]):
                rows.append((int(row["Dispatch_Id"]),
                             (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6))
    rows.sort()
    acc = {"items": [], "users": []}
    for j, (_, ms) in enumerate(rows):
        acc["items" if j % 2 == 0 else "users"].append(ms)
    return {h: sum(v) / len(v) for h, v in acc.items() if v}


def mfma_flops(k, split, rows):
    M = k // 16
    tiles = M * (M + 1) // 2
    gram = RATINGS * tiles * 16 * 16 * 2 * (3 if split else 1)     # bf16 MFMA
    # per row: K_j (M-1-p tiles of 4 MFMAs each, 16x16x4 fp32 = 2048 FLOPs) and the
    # trailing update (sum over p of (M-1-p)(M-p)/2 tiles x 4)
    k_t = sum(M - 1 - p for p in range(M))
    tr_t = sum((M - 1 - p) * (M - p) // 2 for p in range(M))
    solve = rows * (k_t + tr_t) * 4 * 2048
    useful = RATINGS * k * (k + 1) + rows * (k ** 3 / 3 + 2 * k * k)
    return gram, solve, useful


def table():
    res = {"how": __doc__.split("\n\n")[0], "configs": {}}
    for tag, k, split, prec in (("r64", 64, False, "bf16"), ("r128", 128, True, "fp32")):
        sq, meta = counters("roof_%s_sq" % tag)
        tcc, _ = counters("roof_%s_tcc" % tag)
        tm = times("roof_trace64" if tag == "r64" else "roof_trace")
        cfg = {"kernel": meta[0][:160] if meta else None,
               "vgpr": meta[1] if meta else None, "agpr": meta[2] if meta else None,
               "lds_bytes": meta[3] if meta else None, "half_steps": {}}
        for half, rows in (("items", ITEMS), ("users", USERS)):
            c = sq[half]
            active = c.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
            gram, solve, useful = mfma_flops(k, split, rows)
            ms = tm.get(half)
            fetch = tcc[half].get("FETCH_SIZE", 0.0) * 1024 * 2
            h = {
                "rows": rows, "ratings": RATINGS, "kernel_ms": ms,
                "mfma_flops_gramian": gram, "mfma_flops_solve": solve,
                "useful_flops": useful, "hbm_bytes_est": fetch,
                "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (SIMDS * active)
                if active else None,
                "valu_busy": 4 * c.get("SQ_ACTIVE_INST_VALU", 0.0) / (SIMDS * active)
                if active else None,
                "lds_bank_conflict_share": c.get("SQ_LDS_BANK_CONFLICT", 0.0) /
                max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0.0)),
                "counters": dict(c),
            }
            if ms:
                s = ms / 1e3
                h["gramian_tflops"] = gram / s / 1e12
                h["gramian_vs_bf16_peak"] = gram / s / PEAK["bf16"]
                h["solve_tflops_fp32"] = solve / s / 1e12
                h["hbm_tbps"] = fetch / s / 1e12
                h["hbm_vs_peak"] = fetch / s / PEAK["hbm"]
                # time floors: every MFMA at its dense peak, every byte at HBM peak
                h["floor_ms_mfma"] = (gram / PEAK["bf16"] + solve / PEAK["fp32"]) * 1e3
                h["floor_ms_hbm"] = fetch / PEAK["hbm"] * 1e3
            cfg["half_steps"][half] = h
        res["configs"]["rank%d_%s" % (k, prec)] = cfg
    return res


def markdown(res):
    lines = ["# ALS solve kernels: per-half-step roofline (round 5)", "",
             res["how"], "",
             "| config | half-step | kernel ms | MFMA TFLOP/s (Gramian, bf16) | vs bf16 peak | "
             "solve MFMA TFLOP/s (fp32) | HBM TB/s (est) | MFMA busy | VALU busy | "
             "MFMA floor ms | HBM floor ms |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    for name, cfg in res["configs"].items():
        for half, h in cfg["half_steps"].items():
            f = lambda v, d=3: ("%.*f" % (d, v)) if isinstance(v, (int, float)) else "-"
            lines.append("| %s | %s | %s | %s | %s | %s | %s | %s | %s | %s | %s |" % (
                name, half, f(h.get("kernel_ms")), f(h.get("gramian_tflops"), 1),
                f(h.get("gramian_vs_bf16_peak")), f(h.get("solve_tflops_fp32"), 1),
                f(h.get("hbm_tbps"), 2), f(h.get("mfma_busy")), f(h.get("valu_busy")),
                f(h.get("floor_ms_mfma")), f(h.get("floor_ms_hbm"))))
    lines += ["", "Kernels: " + "; ".join("%s: %s (VGPR %s, AGPR %s, LDS %s B)" % (
        n, c["kernel"], c["vgpr"], c["agpr"], c["lds_bytes"]) for n, c in res["configs"].items())]
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    r = table()
    with open(os.path.join(ROOT, "profiles", "r5_als_roofline.json"), "w") as fh:
        json.dump(r, fh, indent=1)
    md = markdown(r)
    with open(os.path.join(ROOT, "profiles", "r5_als_roofline.md"), "w") as fh:
        fh.write(md)
    print(md)
