#!/bin/bash
# Per-half-step roofline counters of the ALS solve kernels: rank 64 bf16 (c2) and rank 128
# fp32 at 25M ratings.  Two rocprofv3 --pmc passes per configuration (8 SQ + GRBM; TCC
# FETCH_SIZE + GRBM), each its own run; plus a kernel trace for the per-dispatch times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
TCC="FETCH_SIZE GRBM_GUI_ACTIVE"
run() {  # name counters args...
  local name=$1 ctrs=$2; shift 2
  rm -rf gpurun_out/roof_$name
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/roof_$name -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/roof_$name.log 2>&1 || { echo "pass $name failed"; tail -20 gpurun_out/roof_$name.log; exit 1; }
  echo "pass $name ok"
}
run r64_sq "$SQ" --steps 2 --warmup 1 --speed-events 0
run r64_tcc "$TCC" --steps 2 --warmup 1 --speed-events 0
run r128_sq "$SQ" --steps 2 --warmup 1 --speed-events 0 --rank-k 128 --precision fp32
run r128_tcc "$TCC" --steps 2 --warmup 1 --speed-events 0 --rank-k 128 --precision fp32
rm -rf gpurun_out/roof_trace
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/roof_trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --speed-events 0 --rank-k 128 --precision fp32 > gpurun_out/roof_trace.log 2>&1 || { tail -20 gpurun_out/roof_trace.log; exit 1; }
rm -rf gpurun_out/roof_trace64
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/roof_trace64 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --speed-events 0 > gpurun_out/roof_trace64.log 2>&1 || { tail -20 gpurun_out/roof_trace64.log; exit 1; }
echo done
