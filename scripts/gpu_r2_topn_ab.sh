#!/bin/bash
# Same-box A/B of the top-N scan: in-tree library (pipelined loads) vs ab/liboryx_kernels_old.so.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "50 1000000 0.3" "250 20000000 1.0"; do
  set -- $cfg
  for v in new old; do
    if [[ $v == old ]]; then export ORYX_KERNELS_SO=$PWD/ab/liboryx_kernels_old.so; else unset ORYX_KERNELS_SO; fi
    timeout -k 10 500 python -u bench_serving.py --features $1 --items $2 --sample-rate $3 --workers 1,4 --requests 200 --warmup 20 > gpurun_out/ab_topn_${1}_$v.jsonl 2> gpurun_out/ab_topn_${1}_$v.err || { tail -20 gpurun_out/ab_topn_${1}_$v.err; exit 1; }
    echo "$v $1 $2 $3: $(grep -o '"value": [0-9.]*\|"mean_latency_ms": [0-9.]*\|"workers": [0-9]*' gpurun_out/ab_topn_${1}_$v.jsonl | tr '\n' ' ')"
  done
done
