#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log | grep -o '"speed_layer_update_ms.*'
for ro in 1 0; do
  ORYX_RDF_ROW_ORDER=$ro timeout -k 10 400 python bench_rdf.py --steps 3 --warmup 1 > gpurun_out/bench_rdf_ro$ro.log 2>&1 || { tail -20 gpurun_out/bench_rdf_ro$ro.log; exit 1; }
  echo "row_order=$ro"; tail -1 gpurun_out/bench_rdf_ro$ro.log | grep -o '"ms_per_step[^,]*\|"speed_layer_update_ms[^,]*'
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rdf3 -o run --output-format csv -- python3 bench_rdf.py --steps 3 --warmup 1 > gpurun_out/prof_rdf3.log 2>&1 || { tail -20 gpurun_out/prof_rdf3.log; exit 1; }
bash scripts/gpu_r2_km.sh
