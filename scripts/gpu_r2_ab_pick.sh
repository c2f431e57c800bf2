#!/bin/bash
# Same-box A/B of the kernel library: this tree's build vs oryx_amd/_native/liboryx_kernels_abold.so
# (built from another revision), alternating three times.  Extra args go to bench.py.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OLD=$PWD/oryx_amd/_native/liboryx_kernels_abold.so
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --speed-events 0 "$@" > gpurun_out/ab_new_$r.log 2>&1 || exit 1
  ORYX_KERNELS_SO=$OLD timeout -k 10 200 python bench.py --steps 10 --warmup 3 --speed-events 0 "$@" > gpurun_out/ab_old_$r.log 2>&1 || exit 1
  echo "new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$r.log)  old $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$r.log)"
done
