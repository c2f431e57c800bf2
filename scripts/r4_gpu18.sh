set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rdf.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_rdf3.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_rdf3.log; exit 1; }
timeout -k 10 400 python -u bench_rdf.py --speed-events 0 > gpurun_out/r4_bench_rdf_v5.json 2> gpurun_out/r4_bench_rdf_v5.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES -d gpurun_out/pmcrdf1 -o run --output-format csv -- python3 bench_rdf.py --steps 1 --warmup 1 --speed-events 0 > gpurun_out/pmcrdf1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES -d gpurun_out/pmcrdf2 -o run --output-format csv -- python3 bench_rdf.py --steps 1 --warmup 1 --speed-events 0 > gpurun_out/pmcrdf2.log 2>&1 || exit 1
echo done
