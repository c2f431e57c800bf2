set -o pipefail
mkdir -p gpurun_out
df -h /tmp /dev/shm > gpurun_out/r4_df.txt 2>&1; free -g >> gpurun_out/r4_df.txt 2>&1; nproc >> gpurun_out/r4_df.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r4_gpu_tests.log; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || exit 1
timeout -k 10 300 python scripts/bench_log_append.py > gpurun_out/r4_log_append.jsonl 2>&1 || exit 1
timeout -k 10 300 python bench_batch.py --ratings 25000000 --test-fraction 0.1 > gpurun_out/r4_bb_single_tf.json 2> gpurun_out/r4_bb_single_tf.err || exit 1
timeout -k 10 300 python bench_batch.py --ratings 25000000 > gpurun_out/r4_bb_single.json 2> gpurun_out/r4_bb_single.err || exit 1
timeout -k 10 400 python bench_batch.py --app rdf --points 6250000 > gpurun_out/r4_bb_rdf.json 2> gpurun_out/r4_bb_rdf.err || exit 1
timeout -k 10 300 python bench.py --emulate-world 8 --emulate-rank 0 --steps 10 --warmup 3 > gpurun_out/r4_emul_c2_w8.json 2> gpurun_out/r4_emul_c2_w8.err || exit 1
timeout -k 10 400 python -u bench_serving.py --items 20000000 --features 250 --sample-rate 1.0 --workers 1,4 --requests 200 --warmup 20 --rescorer > gpurun_out/r4_serving_rescorer.jsonl 2> gpurun_out/r4_serving_rescorer.err || exit 1
echo done
