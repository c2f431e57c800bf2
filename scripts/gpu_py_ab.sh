#!/bin/bash
# Same-box A/B of two versions of oryx_amd/ops/rdf.py (ab/rdf_old.py vs ab/rdf_new.py) on
# bench_rdf, after the RDF GPU tests; swaps the file in the box's scratch copy only.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rdf.py tests/test_app_its.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_rdf.log 2>&1 || { tail -30 gpurun_out/pytest_rdf.log; exit 1; }
tail -1 gpurun_out/pytest_rdf.log
for i in 1 2 3; do for v in new old; do
  cp ab/rdf_$v.py oryx_amd/ops/rdf.py
  timeout -k 10 400 python bench_rdf.py --steps 10 --warmup 2 --speed-events 1000 > gpurun_out/ab_rdf_$v.log 2>&1 || { tail -20 gpurun_out/ab_rdf_$v.log; exit 1; }
  echo "rdf $v $(tail -1 gpurun_out/ab_rdf_$v.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
cp ab/rdf_new.py oryx_amd/ops/rdf.py
