#!/bin/bash
# Round 5: like gpu_r5_soab.sh, with extra variant builds: scripts/gpu_r5_ab3.sh TAG "bench args;..." [variant.so ...]
# (numerics / schedule tests on the working tree's _C; then, per config, new, each variant, old, twice)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5ab3}; CONFIGS=$2; shift 2
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
AB=$(ls pytorch_ddp_mnist_amd/_C_ab*.so | head -1)
echo "tests" &&
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py tests/test_schedules_gpu.py tests/test_loaders.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || exit 1
for v in "$@"; do
  echo "tests $v"
  MNIST_AMD_C_PATH=$v timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py tests/test_schedules_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_$(basename $v .so).txt" 2>&1 || exit 1
done
echo "A/B"
IFS=';' read -ra CS <<< "$CONFIGS"
for r in 1 2; do
  i=0
  for c in "${CS[@]}"; do
    timeout -k 10 180 python bench.py --no-eval $c >> "$OUT/ab_${i}_new.jsonl" 2>> "$OUT/ab.err" || exit 1
    for v in "$@"; do
      MNIST_AMD_C_PATH=$v timeout -k 10 180 python bench.py --no-eval $c >> "$OUT/ab_${i}_$(basename $v .so).jsonl" 2>> "$OUT/ab.err" || exit 1
    done
    MNIST_AMD_C_PATH=$AB timeout -k 10 180 python bench.py --no-eval $c >> "$OUT/ab_${i}_old.jsonl" 2>> "$OUT/ab.err" || exit 1
    i=$((i+1))
  done
done
echo "rc=0"
