set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rdf.py tests/test_kmeans.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_rdf.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_rdf.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profkm -o run --output-format csv -- python3 bench_kmeans.py --steps 5 --warmup 2 --speed-events 0 > gpurun_out/profkm.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profrdf -o run --output-format csv -- python3 bench_rdf.py --steps 3 --warmup 1 --speed-events 0 > gpurun_out/profrdf.log 2>&1 || exit 1
timeout -k 10 400 python -u bench_rdf.py > gpurun_out/r4_bench_rdf_v2.json 2> gpurun_out/r4_bench_rdf_v2.err || exit 1
for s in default 6250,3125 4096,2048 8192,4096 3072,1536; do
  if [ $s = default ]; then e=""; else e="ORYX_ALS_SPLIT=$s"; fi
  env $e timeout -k 10 200 python bench.py --emulate-world 8 --emulate-rank 0 --steps 10 --warmup 3 > gpurun_out/r4_emul_c2_w8_split_$s.json 2> gpurun_out/r4_emul_split.err || exit 1
done
timeout -k 10 900 python -u bench_serving.py --items 20000000 --features 250 --time-to-ready > gpurun_out/r4_serving_ttr_20m_250.json 2> gpurun_out/r4_serving_ttr_20m_250.err || exit 1
echo done
