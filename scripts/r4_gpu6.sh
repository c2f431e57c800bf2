set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r4_gpu_tests.log; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || exit 1
timeout -k 10 300 python scripts/speed_under_load.py > gpurun_out/r4_speed_under_load.json 2> gpurun_out/r4_speed_under_load.err || exit 1
timeout -k 10 300 env ORYX_FORCE_COLLECTIVES=1 python bench_batch.py --ratings 25000000 --generations 3 > gpurun_out/r4_bb_forced_g3.json 2> gpurun_out/r4_bb_forced_g3.err || exit 1
timeout -k 10 600 python -u bench_serving.py --items 20000000 --features 250 --sample-rate 1.0 --workers 1,4 --requests 200 --warmup 20 --rescorer > gpurun_out/r4_serving_rescorer.jsonl 2> gpurun_out/r4_serving_rescorer.err || exit 1
echo done
