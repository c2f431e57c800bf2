#!/bin/bash
# Serving time-to-ready at scale (20M items x 250 features from the
# update topic) plus HBM held by the loaded model.  $1 items (default 20000000).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ITEMS=${1:-20000000}
df -h /tmp /dev/shm . 2>&1 | tee gpurun_out/ttr_df.txt
free -g | tee -a gpurun_out/ttr_df.txt
# the log needs ~2.8 KB per row: pick a filesystem with room for it (the overlay /tmp
# reported 79 GB free but failed a write part-way through the 20M-row log)
DIR=$(python - "$ITEMS" <<'PY'
import os, shutil, sys
need = int(sys.argv[1]) * 2900 * 1.15
for d in ("/dev/shm", "/tmp", os.getcwd()):
    try:
        if shutil.disk_usage(d).free > need:
            print(d); break
    except OSError:
        pass
else:
    print("")
PY
)
if [ -z "$DIR" ]; then echo "no filesystem with room for $ITEMS rows"; exit 1; fi
echo "log dir: $DIR"
( while sleep 30; do echo "tick $(date +%T)"; done ) &
TICK=$!
ORYX_TTR_DIR=$DIR timeout -k 10 1000 python bench_serving.py --time-to-ready --items $ITEMS \
    --users 100000 --features 250 > gpurun_out/ttr_$ITEMS.log 2>&1
RC=$?
kill $TICK
tail -1 gpurun_out/ttr_$ITEMS.log
exit $RC
