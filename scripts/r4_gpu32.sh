set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_pytest_gpu_v4.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_pytest_gpu_v4.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke_v4.log 2>&1 || { tail -20 gpurun_out/r4_smoke_v4.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench_v5.json 2> gpurun_out/r4_bench_v5.err || exit 1
timeout -k 10 400 python -u bench_kmeans.py > gpurun_out/r4_bench_kmeans_v7.json 2> gpurun_out/r4_bench_kmeans_v7.err || exit 1
timeout -k 10 400 python -u bench_rdf.py > gpurun_out/r4_bench_rdf_v10.json 2> gpurun_out/r4_bench_rdf_v10.err || exit 1
echo done
