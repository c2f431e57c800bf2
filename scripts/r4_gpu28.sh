set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m cProfile -o gpurun_out/bb_tf01.prof bench_batch.py --test-fraction 0.1 > gpurun_out/r4_bb_als_tf01_prof.json 2> gpurun_out/r4_bb_als_tf01_prof.err || exit 1
python - > gpurun_out/bb_tf01_prof.txt <<'PY'
import pstats
p = pstats.Stats("gpurun_out/bb_tf01.prof")
p.sort_stats("cumulative").print_stats(70)
p.sort_stats("tottime").print_stats(40)
PY
echo done
