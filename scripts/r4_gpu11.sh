set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py tests/test_als_serving.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_km.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_km.log; exit 1; }
timeout -k 10 400 python -u bench_kmeans.py > gpurun_out/r4_bench_kmeans.json 2> gpurun_out/r4_bench_kmeans.err || exit 1
timeout -k 10 400 python -u bench_rdf.py > gpurun_out/r4_bench_rdf.json 2> gpurun_out/r4_bench_rdf.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --speed-events 0 > gpurun_out/prof64.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof128 -o run --output-format csv -- python3 bench.py --rank-k 128 --precision fp32 --steps 5 --warmup 2 --speed-events 0 > gpurun_out/prof128.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc64 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --speed-events 0 > gpurun_out/pmc64.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc128 -o run --output-format csv -- python3 bench.py --rank-k 128 --precision fp32 --steps 3 --warmup 1 --speed-events 0 > gpurun_out/pmc128.log 2>&1 || exit 1
timeout -k 10 600 python -u bench_batch.py --app kmeans > gpurun_out/r4_bb_kmeans.json 2> gpurun_out/r4_bb_kmeans.err || exit 1
echo done
