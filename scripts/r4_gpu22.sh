set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_v9.json 2> gpurun_out/r4_bench_rdf_v9.err || exit 1
timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_v9b.json 2>> gpurun_out/r4_bench_rdf_v9.err || exit 1
rocm-smi --showclocks --showpower --showuse > gpurun_out/r4_smi.txt 2>&1 || true
echo done
