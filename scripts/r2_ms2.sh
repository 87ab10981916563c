#!/bin/bash
# graph cache + interleaved calibration: runtime/multigpu/schedule GPU tests, then driver-shaped benches
set -o pipefail
mkdir -p gpurun_out
T=${1:-ms}
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_multigpu_gpu.py tests/test_schedules_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_b${rep}.json 2> gpurun_out/${T}_b${rep}.err || { echo "bench failed"; tail -20 gpurun_out/${T}_b${rep}.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('rep$rep', d['ms_per_step'], d['value'], d['config'].get('plan_autotune',{}).get('timings_ms'))" gpurun_out/${T}_b${rep}.json
done
