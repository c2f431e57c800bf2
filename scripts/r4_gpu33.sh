set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rdf.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_rdf6.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_rdf6.log; exit 1; }
timeout -k 10 400 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_v11.json 2> gpurun_out/r4_bench_rdf_v11.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profrdf11 -o run --output-format csv -- python3 bench_rdf.py --steps 3 --warmup 1 --speed-events 0 > gpurun_out/profrdf11.log 2>&1 || exit 1
echo done
