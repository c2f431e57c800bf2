set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_als_kernel.py tests/test_als_trainer.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_als.log 2>&1 || { tail -30 gpurun_out/t_als.log; exit 1; }
tail -2 gpurun_out/t_als.log
ORYX_ALS_VARIANT=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/b0.log 2>&1 || { tail -30 gpurun_out/b0.log; exit 1; }
ORYX_ALS_VARIANT=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/b1.log 2>&1 || { tail -30 gpurun_out/b1.log; exit 1; }
python -c "
import json
for f in ['gpurun_out/b0.log','gpurun_out/b1.log']:
    r=json.loads(open(f).read().strip().splitlines()[-1]); print(f, r['value'], r['ms_per_step'], r['solve_failures'])
"
timeout -k 10 300 python scripts/als_phase_profile.py > gpurun_out/phase.log 2>&1 || { tail -30 gpurun_out/phase.log; exit 1; }
cat gpurun_out/phase.log | tail -30
