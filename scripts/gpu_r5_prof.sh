#!/bin/bash
# Round-5 measurement pass (one gpurun call):  scripts/gpu_r5_prof.sh TAG
# benches of every BASELINE-relevant config, kernel-time profiles and the one-shot latency breakdown.
# Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5prof}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
B="timeout -k 10 180 python bench.py"
J="$OUT/bench.jsonl"
E="$OUT/bench.err"
echo "numerics + schedules" &&
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py tests/test_schedules_gpu.py tests/test_gpu_runtime.py tests/test_multigpu_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_subset.txt" 2>&1 &&
echo "benches" &&
$B --gpus 1 --steps 20 --warmup 5 >> $J 2>> $E &&
$B --gpus 1 --steps 20 --warmup 5 >> $J 2>> $E &&
$B --steps 2000 --warmup 50 >> $J 2>> $E &&
$B --model mlp --dtype bf16 --batch 8192 --steps 1000 --warmup 50 >> $J 2>> $E &&
$B --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 50 >> $J 2>> $E &&
$B --batch 128 --steps 2000 --warmup 50 >> $J 2>> $E &&
$B --batch 128 --dtype fp32 --steps 2000 --warmup 50 >> $J 2>> $E &&
$B --dtype fp32 --steps 200 --warmup 10 >> $J 2>> $E &&
$B --batch 1024 --steps 1000 --warmup 50 >> $J 2>> $E &&
$B --model mlp --dtype fp32 --batch 8192 --steps 500 --warmup 20 >> $J 2>> $E &&
echo "one-shot latency" &&
timeout -k 10 180 python scripts/diag/oneshot_lat.py > "$OUT/oneshot_lat.txt" 2>&1 &&
echo "kernel profiles" &&
timeout -k 10 1200 bash scripts/prof_configs.sh "$TAG/k" lenet mlp8k mlp128 lenet128 lenet128f lenetf > "$OUT/prof.log" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
