set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_ab2_views.json 2> gpurun_out/r4_bench_rdf_ab.err || exit 1
ORYX_RDF_BUILD_NOGC=1 timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_ab2_nogc.json 2>> gpurun_out/r4_bench_rdf_ab.err || exit 1
ORYX_RDF_ROUTE_LDS=0 timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_ab2_noroute.json 2>> gpurun_out/r4_bench_rdf_ab.err || exit 1
echo done
