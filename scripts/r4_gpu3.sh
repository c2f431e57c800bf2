set -o pipefail
mkdir -p gpurun_out
ORYX_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench_batch.py --ratings 25000000 --generations 3 > gpurun_out/r4_bb_forced_g3.json 2> gpurun_out/r4_bb_forced_g3.err || exit 1
ORYX_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench_batch.py --ratings 25000000 --test-fraction 0.1 > gpurun_out/r4_bb_forced_tf.json 2> gpurun_out/r4_bb_forced_tf.err || exit 1
timeout -k 10 300 python bench_batch.py --ratings 25000000 --test-fraction 0.1 > gpurun_out/r4_bb_single_tf.json 2> gpurun_out/r4_bb_single_tf.err || exit 1
timeout -k 10 300 python bench_batch.py --ratings 25000000 > gpurun_out/r4_bb_single.json 2> gpurun_out/r4_bb_single.err || exit 1
echo done
