#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_als_trainer.py tests/test_forced_collectives.py -m gpu > gpurun_out/r5_graph_tests.log 2>&1 || { tail -40 gpurun_out/r5_graph_tests.log; exit 1; }
tail -2 gpurun_out/r5_graph_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --speed-events 0 --steps 10 --warmup 3 > gpurun_out/r5_bench64_graph$i.json 2>gpurun_out/r5_bench64_graph.err || { tail -20 gpurun_out/r5_bench64_graph.err; exit 1; }
done
ORYX_ALS_GRAPH=0 timeout -k 10 300 python -u bench.py --speed-events 0 --steps 10 --warmup 3 > gpurun_out/r5_bench64_nograph.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --speed-events 0 --steps 5 --warmup 2 --rank-k 128 --precision fp32 > gpurun_out/r5_bench128_graph.json 2>/dev/null || exit 1
echo done
