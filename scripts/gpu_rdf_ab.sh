#!/bin/bash
# RDF level-histogram A/B on one GPU: kernel tests, bench_rdf with the row-staged histogram
# (ORYX_RDF_HIST=1, default) and the direct-gather kernel (0), and (PROF=1) a kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rdf.py tests/test_kmeans.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_rdf.log 2>&1 || { tail -30 gpurun_out/t_rdf.log; exit 1; }
tail -2 gpurun_out/t_rdf.log
for h in ${HISTS:-1 0}; do for pc in ${PIECES:-16384}; do
  ORYX_RDF_PIECE=$pc ORYX_RDF_HIST=$h timeout -k 10 400 python bench_rdf.py --steps 2 --warmup 1 --speed-events 2000 > gpurun_out/brdf$h.log 2>&1 || { tail -30 gpurun_out/brdf$h.log; exit 1; }
  echo "hist=$h piece=$pc $(tail -1 gpurun_out/brdf$h.log | cut -c1-300)"; done
done
if [[ ${PROF:-1} == 1 ]]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  rm -rf gpurun_out/prof_rdf
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rdf -o rdf --output-format csv -- python3 bench_rdf.py --steps 1 --warmup 1 --speed-events 2000 > gpurun_out/prof_rdf.log 2>&1 || { tail -30 gpurun_out/prof_rdf.log; exit 1; }
  find gpurun_out/prof_rdf -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/rdf_kernel_stats.csv
  cut -c1-160 gpurun_out/rdf_kernel_stats.csv | head -8
fi
