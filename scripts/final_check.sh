#!/bin/bash
# Pre-commit / round-end check.  On the CPU container (default): the CPU test suite, the
# gfx950 build check and the host-code sanitizers.  With --gpu (run under gpurun on an
# MI355X box): the GPU tests, smoke(), and the 1-GPU ALS and RDF benches.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ "${1:-}" != "--gpu" ]; then
  timeout -k 10 1800 python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider \
    > gpurun_out/final_cpu_tests.log 2>&1 || { echo "CPU tests failed"; tail -40 gpurun_out/final_cpu_tests.log; exit 1; }
  tail -1 gpurun_out/final_cpu_tests.log
  timeout -k 10 1200 python -c "import __graft_entry__ as g; g.build(); print('build ok')" \
    || { echo "build failed"; exit 1; }
  timeout -k 10 1800 bash scripts/sanitize_runtime.sh > gpurun_out/final_sanitize.log 2>&1 \
    || { echo "sanitizers failed"; tail -40 gpurun_out/final_sanitize.log; exit 1; }
  echo "cpu checks ok"
  exit 0
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/final_pytest_gpu.log 2>&1 || { echo tests failed; tail -40 gpurun_out/final_pytest_gpu.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 1
timeout -k 10 400 python -u bench_rdf.py > gpurun_out/final_bench_rdf.json 2> gpurun_out/final_bench_rdf.err || exit 1
echo done
