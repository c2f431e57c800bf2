#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log | grep -o '"speed_layer_update_ms.*'
timeout -k 10 400 python bench_rdf.py --steps 2 --warmup 1 > gpurun_out/bench_rdf.log 2>&1 || { tail -20 gpurun_out/bench_rdf.log; exit 1; }
tail -1 gpurun_out/bench_rdf.log | grep -o '"ms_per_step[^,]*\|"speed_layer_update_ms[^,]*'
bash scripts/gpu_r2_km.sh
