set -o pipefail
mkdir -p gpurun_out
for t in 8 32 128; do
ORYX_TOPN_TILES_PER_WAVE=$t timeout -k 10 300 python -u scripts/topn_bench.py --items 1000000 --features 50 --sample-rate 0.3 > gpurun_out/r4_topn_1m_50_tpw$t.jsonl 2>&1 || exit 1
done
for t in 8 32; do
ORYX_TOPN_TILES_PER_WAVE=$t timeout -k 10 400 python -u scripts/topn_bench.py --items 20000000 --features 250 --sample-rate 1.0 --reps 20 > gpurun_out/r4_topn_20m_250_tpw$t.jsonl 2>&1 || exit 1
done
ORYX_TOPN_BF16=0 timeout -k 10 400 python -u scripts/topn_bench.py --items 20000000 --features 250 --sample-rate 1.0 --reps 20 > gpurun_out/r4_topn_20m_250_fp32.jsonl 2>&1 || exit 1
echo done
