set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_km.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_km.log; exit 1; }
timeout -k 10 400 python -u bench_kmeans.py > gpurun_out/r4_bench_kmeans_v2.json 2> gpurun_out/r4_bench_kmeans_v2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profkm2 -o run --output-format csv -- python3 bench_kmeans.py --steps 5 --warmup 2 --speed-events 0 > gpurun_out/profkm2.log 2>&1 || exit 1
timeout -k 10 400 python -u bench_batch.py --test-fraction 0.1 > gpurun_out/r4_bb_als_tf01_v2.json 2> gpurun_out/r4_bb_als_tf01_v2.err || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench_v3.json 2> gpurun_out/r4_bench_v3.err || exit 1
echo done
