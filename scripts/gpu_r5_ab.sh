#!/bin/bash
# Round 5: A/B of one environment switch on the BASELINE configs it touches, after the schedule / numerics tests.
#   scripts/gpu_r5_ab.sh TAG VAR "CONFIG ..."   (CONFIG = model:dtype:batch:steps)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5ab}; VAR=$2; CONFIGS=$3
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
echo "tests" &&
timeout -k 10 900 python -u -m pytest tests/test_schedules_gpu.py tests/test_native_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || exit 1
echo "A/B"
for r in 1 2; do
  for c in $CONFIGS; do
    IFS=: read -r m d b n <<< "$c"
    for v in 1 0; do
      env "$VAR=$v" timeout -k 10 180 python bench.py --no-eval --model "$m" --dtype "$d" --batch "$b" --steps "$n" --warmup 50 >> "$OUT/ab_${m}_${d}_${b}_${v}.jsonl" 2>> "$OUT/ab.err" || exit 1
    done
  done
done
echo "rc=0"
