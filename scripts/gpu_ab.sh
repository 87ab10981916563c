#!/bin/bash
# One GPU A/B session of a change:  scripts/gpu_ab.sh TAG "PYTEST -k EXPR|-" "BENCH ARGS" ENV_A ENV_B ...
# 1. the GPU tests selected by EXPR (test_native_gpu + test_schedules_gpu; "-" = skip),
# 2. in-kernel phase stamps under each env variant, 3. interleaved bench A/B (scripts/ab_env.sh).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=$1; SEL=$2; ARGS=$3; shift 3
mkdir -p "$OUT"
cd "$ROOT" || exit 1
if [ "$SEL" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py tests/test_schedules_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "$SEL" > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
  tail -1 "$OUT/${TAG}_pytest.log"
fi
i=0
for kv in "$@"; do
  [ "$kv" = "-" ] && kv=""
  env $kv timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_$i.log" 2>&1 || exit 1
  i=$((i+1))
done
bash scripts/ab_env.sh "$TAG" "$ARGS" "$@"
