#!/usr/bin/env python3
"""Per-kernel register / spill / LDS / occupancy table of one .hip file (gfx950).

usage: python scripts/kernel_resources.py csrc/kernels/als.hip
"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
       "-munsafe-fp-atomics", "-I", "csrc/kernels", "-c", src, "-o", "/tmp/_kr.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: ([A-Za-z \[\]/]+): (.*?) \[-Rpass", line)
    if not m:
        continue
    key, val = m.group(1).strip(), m.group(2).strip()
    if key == "Function Name":
        cur = {"name": subprocess.run(["c++filt", val], capture_output=True,
                                      text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[key] = val
cols = ["VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "SGPRs Spill", "LDS Size [bytes/block]",
        "Occupancy [waves/SIMD]"]
print("%-60s %5s %5s %5s %6s %6s %7s %4s" % ("kernel", "vgpr", "agpr", "sgpr", "vspill",
                                             "sspill", "lds", "occ"))
for r in rows:
    n = re.sub(r"\(anonymous namespace\)::", "", r["name"])[:60]
    print("%-60s %5s %5s %5s %6s %6s %7s %4s" % ((n,) + tuple(r.get(c, "?") for c in cols)))
