#!/bin/bash
# multi-step graph check: new GPU test, then driver-shaped bench with k=1 vs k=8 vs k=20 (same box)
set -o pipefail
mkdir -p gpurun_out
T=${1:-ms}
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -x -q --timeout 120 --timeout-method thread \
  -k "multi_step or captured_step" > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for rep in 1 2; do
  for k in 1 8 20; do
    MNIST_AMD_GRAPH_STEPS=$k timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_k${k}_${rep}.json 2> gpurun_out/${T}_k${k}_${rep}.err || { echo "bench k=$k failed"; tail -20 gpurun_out/${T}_k${k}_${rep}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('k=$k rep$rep', d['ms_per_step'], d['value'])" gpurun_out/${T}_k${k}_${rep}.json
  done
done
for k in 1 8; do
  MNIST_AMD_GRAPH_STEPS=$k timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > gpurun_out/${T}_long_k${k}.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('long k=$k', d['ms_per_step'], d['value'])" gpurun_out/${T}_long_k${k}.json
done
