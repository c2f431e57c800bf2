set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_pytest_gpu_v6.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_pytest_gpu_v6.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke_v6.log 2>&1 || { tail -20 gpurun_out/r4_smoke_v6.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench_v6.json 2> gpurun_out/r4_bench_v6.err || exit 1
timeout -k 10 400 python -u bench_rdf.py > gpurun_out/r4_bench_rdf_v13.json 2> gpurun_out/r4_bench_rdf_v13.err || exit 1
echo done
