#!/bin/bash
# One parametrised GPU-box session (replaces the per-experiment one-off scripts).
#
#   bash scripts/gpu.sh STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the chain stops at the first failure
# (never retried).  Output goes to gpurun_out/<step>.log (JSON lines to .json).  Environment
# variables pass through (e.g. ORYX_ALS_VARIANT=3 bash scripts/gpu.sh bench).
#
#   tests[=EXPR]        pytest -m gpu (EXPR: a -k expression)
#   smoke               __graft_entry__.smoke()
#   bench[=ARGS]        bench.py --steps 20 --warmup 5 [ARGS, comma separated]
#   halfstep[=V]        scripts/als_kernel_bench.py (per half-step ms) with ORYX_ALS_VARIANT=V
#   hs[=ARGS]           scripts/als_kernel_bench.py ARGS (e.g. hs=--rank-k,128,--precision,fp32);
#                       ORYX_KERNELS_SO / ORYX_ALS_* from the environment (A/B of builds)
#   phases[=V]          scripts/als_phase_profile.py (per-phase cycles) with ORYX_ALS_VARIANT=V
#   batch[=ARGS]        bench_batch.py --ratings 25000000 [ARGS]
#   kmeans[=PREC]       bench_kmeans.py --precision PREC (fp32)
#   rdf                 bench_rdf.py
#   serving[=ARGS]      bench_serving.py [ARGS]
#   sil                 scripts/silhouette_probe.py (MFMA vs VALU silhouette, 100k x 256, k = 1000)
#   traffic[=RATE]      bench_traffic.py 20M items x 250, LSH sample rate RATE (0.3), speed layer live
#   prof=NAME:CMD       rocprofv3 --kernel-trace --stats of CMD (e.g. prof=als:bench.py,--steps,5)
#   pmc=NAME:CTRS:CMD   one rocprofv3 --pmc pass (CTRS comma separated) of CMD
#   env=K=V             export K=V for the following steps (env=K= unsets K)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTEST="python -u -m pytest -x -v --timeout 150 --timeout-method thread"

fail() { echo "== FAILED: $1"; tail -30 "$2"; exit 1; }
args() { echo "$1" | tr ',' ' '; }
tag() { echo "$1" | tr -c 'a-zA-Z0-9\n' '_'; }

for step in "$@"; do
  name=${step%%=*}
  val=""
  [[ $step == *=* ]] && val=${step#*=}
  echo "== $step"
  case $name in
    tests)
      out=gpurun_out/tests${val:+_sel}.log
      if [[ -n $val ]]; then
        timeout -k 10 900 $PYTEST tests -m gpu -k "$val" > $out 2>&1 || fail "$step" $out
      else
        timeout -k 10 1100 $PYTEST tests -m gpu > $out 2>&1 || fail "$step" $out
      fi
      tail -2 $out ;;
    smoke)
      out=gpurun_out/smoke.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out 2>&1 || fail "$step" $out
      tail -2 $out ;;
    bench)
      out=gpurun_out/bench${val:+_$(tag "$val")}${ORYX_FORCE_COLLECTIVES:+_forced}.json
      timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 $(args "$val") > $out 2> gpurun_out/bench.err || fail "$step" gpurun_out/bench.err
      tail -1 $out | cut -c1-3000 ;;
    halfstep)
      out=gpurun_out/halfstep_v${val:-default}.json
      ORYX_ALS_VARIANT=${val:-${ORYX_ALS_VARIANT:-5}} timeout -k 10 400 python -u scripts/als_kernel_bench.py --reps 7 > $out 2> $out.err || fail "$step" $out.err
      cat $out ;;
    hs)
      out=gpurun_out/hs_$(tag "${val:-default}")${ORYX_KERNELS_SO:+_$(basename $ORYX_KERNELS_SO .so)}.json
      timeout -k 10 300 python -u scripts/als_kernel_bench.py --reps 5 $(args "$val") > $out 2> $out.err || fail "$step" $out.err
      cut -c1-400 $out ;;
    phases)
      out=gpurun_out/phases_v${val:-default}.json
      ORYX_ALS_VARIANT=${val:-${ORYX_ALS_VARIANT:-5}} timeout -k 10 400 python -u scripts/als_phase_profile.py > $out 2> $out.err || fail "$step" $out.err
      cat $out ;;
    batch)
      out=gpurun_out/bench_batch.json
      timeout -k 10 900 python -u bench_batch.py --ratings 25000000 $(args "$val") > $out 2> gpurun_out/bench_batch.err || fail "$step" gpurun_out/bench_batch.err
      tail -1 $out | cut -c1-2000 ;;
    kmeans)
      out=gpurun_out/bench_kmeans_${val:-fp32}.json
      timeout -k 10 400 python -u bench_kmeans.py --steps 5 --warmup 2 --precision ${val:-fp32} > $out 2> $out.err || fail "$step" $out.err
      tail -1 $out | cut -c1-1500 ;;
    rdf)
      out=gpurun_out/bench_rdf.json
      timeout -k 10 400 python -u bench_rdf.py --steps 3 --warmup 1 $(args "$val") > $out 2> $out.err || fail "$step" $out.err
      tail -1 $out | cut -c1-1500 ;;
    serving)
      out=gpurun_out/bench_serving.jsonl
      timeout -k 10 1100 python -u bench_serving.py $(args "$val") > $out 2> $out.err || fail "$step" $out.err
      cut -c1-400 $out ;;
    sil)
      out=gpurun_out/silhouette${val:+_$(tag "$val")}.json
      timeout -k 10 300 python -u scripts/silhouette_probe.py > $out 2> $out.err || fail "$step" $out.err
      cat $out ;;
    traffic)
      out=gpurun_out/traffic_20m_250_lsh$(tag "${val:-0.3}").json
      timeout -k 10 600 python -u bench_traffic.py --items 20000000 --users 500000 --features 250 --sample-rate ${val:-0.3} > $out 2> $out.err || fail "$step" $out.err
      tail -1 $out | cut -c1-1500 ;;
    prof)
      pname=${val%%:*}; cmd=$(args "${val#*:}")
      rm -rf gpurun_out/prof_$pname
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$pname -o run --output-format csv -- python3 $cmd > gpurun_out/prof_$pname.log 2>&1 || fail "$step" gpurun_out/prof_$pname.log
      find gpurun_out/prof_$pname -name "*kernel_stats.csv" | head -1 | xargs -I{} head -16 {} | cut -c1-220 ;;
    pmc)
      pname=${val%%:*}; rest=${val#*:}; ctrs=$(args "${rest%%:*}"); cmd=$(args "${rest#*:}")
      rm -rf gpurun_out/pmc_$pname
      timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $ctrs -d gpurun_out/pmc_$pname -o run --output-format csv -- python3 $cmd > gpurun_out/pmc_$pname.log 2>&1 || fail "$step" gpurun_out/pmc_$pname.log
      find gpurun_out/pmc_$pname -name "*counter_collection.csv" | head -1 | xargs -I{} head -3 {} | cut -c1-300 ;;
    env)
      kv=$val; k=${kv%%=*}; v=${kv#*=}
      if [[ -n $v ]]; then export "$k=$v"; else unset "$k"; fi ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
