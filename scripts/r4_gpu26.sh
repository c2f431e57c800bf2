set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench_serving.py --items 20000000 --features 250 --time-to-ready > gpurun_out/r4_serving_ttr_20m_250_v2.json 2> gpurun_out/r4_serving_ttr_20m_250_v2.err || exit 1
echo done
