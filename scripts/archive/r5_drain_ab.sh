#!/bin/bash
# Drain A/B on a k-means generation (22.5 GB of text over 8 partitions): per-partition
# buffers + concatenation, one buffer, one buffer prefaulted by 16 threads.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
for v in old one pre; do
  case $v in
    old) E="ORYX_DRAIN_ONE_BUFFER=0" ;;
    one) E="ORYX_DRAIN_ONE_BUFFER=1" ;;
    pre) E="ORYX_DRAIN_ONE_BUFFER=1 ORYX_DRAIN_PREFAULT=1" ;;
  esac
  env $E timeout -k 10 300 python -u bench_batch.py --app kmeans --generations 1 > gpurun_out/r5_drain_${v}_$TAG.json 2> gpurun_out/r5_drain_${v}_$TAG.err || { tail -20 gpurun_out/r5_drain_${v}_$TAG.err; exit 1; }
  python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=r['phase_s']; print(sys.argv[2], 'gen %.3f drain %.3f save_data %.3f update %.3f' % (r['generation_s'], p['layer_drain'], p['layer_save_data'], p['layer_update']))" gpurun_out/r5_drain_${v}_$TAG.json $v
done
echo done
