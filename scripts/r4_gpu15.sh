set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3 4; do
  ORYX_KM_FULL_VARIANT=$v timeout -k 10 120 python -u scripts/km_full_variants.py >> gpurun_out/r4_km_full_variants.jsonl 2>> gpurun_out/r4_km_full_variants.err || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_rdf.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_rdf2.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_rdf2.log; exit 1; }
timeout -k 10 400 python -u bench_rdf.py > gpurun_out/r4_bench_rdf_v4.json 2> gpurun_out/r4_bench_rdf_v4.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profrdf4 -o run --output-format csv -- python3 bench_rdf.py --steps 3 --warmup 1 --speed-events 0 > gpurun_out/profrdf4.log 2>&1 || exit 1
echo done
