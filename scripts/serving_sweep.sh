#!/bin/bash
# /recommend sweep over BASELINE.md's published (features, items, sample-rate) rows on one GPU.
# usage: bash scripts/serving_sweep.sh "50:1000000:0.3 250:20000000:1.0 ..."
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
CONFIGS=${1:-"50:1000000:0.3 250:1000000:0.3 50:5000000:0.3 250:5000000:0.3 50:20000000:0.3 250:20000000:0.3 50:1000000:1.0 250:20000000:1.0"}
for c in $CONFIGS; do
  IFS=: read f n s <<< "$c"
  echo "== features=$f items=$n sample=$s"
  timeout -k 10 600 python bench_serving.py --features $f --items $n --sample-rate $s \
      --workers ${WORKERS:-2} --requests ${REQS:-300} --warmup 20 \
      > gpurun_out/serving_${f}_${n}_${s}.json 2> gpurun_out/serving_${f}_${n}_${s}.err \
    || { tail -20 gpurun_out/serving_${f}_${n}_${s}.err; exit 1; }
  cat gpurun_out/serving_${f}_${n}_${s}.json
done
