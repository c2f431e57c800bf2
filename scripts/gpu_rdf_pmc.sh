#!/bin/bash
# SQ counters of the RDF level histogram (one bench_rdf forest)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_rdf
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d gpurun_out/pmc_rdf -o run --output-format csv -- python3 bench_rdf.py --steps 1 --warmup 0 --speed-events 100 > gpurun_out/pmc_rdf.log 2>&1 || { tail -20 gpurun_out/pmc_rdf.log; exit 1; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/pmc_rdf/run_counter_collection.csv')))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[r['Kernel_Name'][:60]][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0))[:6]:
    print(k, {c: '%.3g' % x for c, x in v.items()})
PY
