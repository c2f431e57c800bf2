set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_km4.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_km4.log; exit 1; }
timeout -k 10 400 python -u bench_kmeans.py --speed-events 0 > gpurun_out/r4_bench_kmeans_v6.json 2> gpurun_out/r4_bench_kmeans_v6.err || exit 1
ORYX_KM_SEGSUM_VEC=0 timeout -k 10 400 python -u bench_kmeans.py --speed-events 0 > gpurun_out/r4_bench_kmeans_v6_scalar.json 2>> gpurun_out/r4_bench_kmeans_v6.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profkm6 -o run --output-format csv -- python3 bench_kmeans.py --steps 5 --warmup 2 --speed-events 0 > gpurun_out/profkm6.log 2>&1 || exit 1
echo done
