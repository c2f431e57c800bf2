set -o pipefail
mkdir -p gpurun_out
ORYX_RDF_STAGE_STEPS=8 timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_rdf_ab_sparse8.json 2> gpurun_out/r4_rdf_ab.err || exit 1
ORYX_RDF_STAGE_STEPS=8 ORYX_RDF_STAGE_SPARSE=0 timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_rdf_ab_dense8.json 2>> gpurun_out/r4_rdf_ab.err || exit 1
timeout -k 10 300 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_rdf_ab_default2.json 2>> gpurun_out/r4_rdf_ab.err || exit 1
echo done
