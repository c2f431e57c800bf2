set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_v8.json 2> gpurun_out/r4_bench_rdf_v8.err || exit 1
for pc in 8192 32768 65536; do
  ORYX_RDF_PIECE=$pc timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_piece_$pc.json 2>> gpurun_out/r4_bench_rdf_sweep.err || exit 1
done
echo done
