set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench_batch.py --test-fraction 0.1 > gpurun_out/r4_bb_als_tf01_v3.json 2> gpurun_out/r4_bb_als_tf01_v3.err || exit 1
timeout -k 10 400 python -u bench_batch.py > gpurun_out/r4_bb_single_v2.json 2> gpurun_out/r4_bb_single_v2.err || exit 1
echo done
