set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES -d gpurun_out/pmckm1 -o run --output-format csv -- python3 bench_kmeans.py --steps 3 --warmup 1 --speed-events 0 > gpurun_out/pmckm1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES -d gpurun_out/pmckm2 -o run --output-format csv -- python3 bench_kmeans.py --steps 3 --warmup 1 --speed-events 0 > gpurun_out/pmckm2.log 2>&1 || exit 1
echo done
