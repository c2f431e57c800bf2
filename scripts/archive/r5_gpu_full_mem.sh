#!/bin/bash
# Full GPU suite + smoke, then the host-memory probe and a k-means / RDF generation with the
# reaper-thread host buffers (oryx_amd/hostbuf.py).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
bash scripts/r5_gpu_full.sh $TAG || exit 1
timeout -k 10 200 python -u scripts/hostmem_probe.py 8 > gpurun_out/r5_hostmem_$TAG.jsonl 2>&1 || { tail -5 gpurun_out/r5_hostmem_$TAG.jsonl; exit 1; }
tail -1 gpurun_out/r5_hostmem_$TAG.jsonl
timeout -k 10 400 python -u bench_batch.py --app kmeans --generations 2 > gpurun_out/r5_bb_kmeans_hb_$TAG.json 2> gpurun_out/r5_bb_kmeans_hb_$TAG.err || { tail -20 gpurun_out/r5_bb_kmeans_hb_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --app rdf --generations 2 > gpurun_out/r5_bb_rdf_hb_$TAG.json 2> gpurun_out/r5_bb_rdf_hb_$TAG.err || { tail -20 gpurun_out/r5_bb_rdf_hb_$TAG.err; exit 1; }
echo done
