#!/bin/bash
# k-means assign A/B on one GPU: kernel tests, then bench_kmeans for each configuration
# "RT:WAVES:EPI" in CONFIGS (RT 0 = 64-point B-operand kernel with WAVES-wave blocks and the
# packed (EPI 1) or plain epilogue, RT 2 = the 32-point A-operand kernel), a kernel-trace of
# the default and (PMC=1) SQ counters of both epilogues (pmc_km1 = packed, pmc_km0 = plain).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_km.log 2>&1 || { tail -30 gpurun_out/t_km.log; exit 1; }
tail -2 gpurun_out/t_km.log
for cfg in ${CONFIGS:-0:4:1 0:4:0 0:8:1 2:4:0}; do
  IFS=: read -r rt nw epi <<< "$cfg"
  log=gpurun_out/bkm_${rt}_${nw}_${epi}.log
  ORYX_KMEANS_RT=$rt ORYX_KMEANS_WAVES=$nw ORYX_KMEANS_EPI=$epi timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 > $log 2>&1 || { tail -30 $log; exit 1; }
  echo "$cfg $(tail -1 $log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["tflops"])')"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [[ ${PROF:-1} == 1 ]]; then
  rm -rf gpurun_out/prof_km
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o km --output-format csv -- python3 bench_kmeans.py --steps 3 --warmup 1 > gpurun_out/prof_km.log 2>&1 || { tail -30 gpurun_out/prof_km.log; exit 1; }
  find gpurun_out/prof_km -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/km_kernel_stats.csv
  cut -c1-150 gpurun_out/km_kernel_stats.csv | head -4
fi
if [[ ${PMC:-0} == 1 ]]; then
  for epi in 1 0; do
    nw=$epi
    rm -rf gpurun_out/pmc_km$nw
    ORYX_KMEANS_EPI=$epi timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_km$nw -o run --output-format csv -- python3 bench_kmeans.py --steps 1 --warmup 0 > gpurun_out/pmc_km$nw.log 2>&1 || { tail -20 gpurun_out/pmc_km$nw.log; exit 1; }
  done
fi
