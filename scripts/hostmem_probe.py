"""Host memory costs behind the batch layer's "release" phases (r5_bb_*_phases: k-means frees
~35 GB of text per generation in ~2 s): first-touch faults and frees of an 8 GB buffer,
numpy's allocator vs an anonymous mapping with MADV_HUGEPAGE, touched by 1 or 16 threads.

Usage: python scripts/hostmem_probe.py [GB]   (one JSON line)
"""

import json
import mmap
import sys
import threading
import time

import numpy as np

GB = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
N = int(GB * (1 << 30))


def _read(p):
    try:
        return open(p).read().strip()
    except OSError as e:
        return str(e)


def touch(a, threads):
    step = 4096
    per = -(-len(a) // threads)
    per = -(-per // step) * step

    def run(lo):
        a[lo:min(len(a), lo + per):step] = 1

    ts = [threading.Thread(target=run, args=(lo,)) for lo in range(0, len(a), per)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


def case(kind, threads):
    t0 = time.perf_counter()
    if kind == "numpy":
        a = np.empty(N, dtype=np.uint8)
        m = None
    else:
        m = mmap.mmap(-1, N, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        if kind == "mmap_huge":
            m.madvise(mmap.MADV_HUGEPAGE)
        a = np.frombuffer(m, dtype=np.uint8)
    t1 = time.perf_counter()
    touch(a, threads)
    t2 = time.perf_counter()
    del a
    if m is not None:
        m.close()
    t3 = time.perf_counter()
    return {"kind": kind, "threads": threads, "alloc_s": round(t1 - t0, 4),
            "touch_s": round(t2 - t1, 4), "free_s": round(t3 - t2, 4)}


def main():
    out = {"gb": GB, "thp_enabled": _read("/sys/kernel/mm/transparent_hugepage/enabled"),
           "thp_defrag": _read("/sys/kernel/mm/transparent_hugepage/defrag"),
           "memtotal": _read("/proc/meminfo").split("\n")[0], "cases": []}
    for kind in ("numpy", "mmap", "mmap_huge"):
        for threads in (1, 16):
            out["cases"].append(case(kind, threads))
            print(json.dumps(out["cases"][-1]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
