#!/bin/bash
# Round 5: last-arriver update tails -- the MLP weight gradient's (head.hip wgrad_tail) and the LeNet small-batch
# conv update's (lenet.hip conv_tail): numerics + bitwise tests, the guard-region store audit, then interleaved
# A/B runs against the separate reduce + SGD kernel (MNIST_AMD_WGRAD_TAIL=0 / MNIST_AMD_CONV_TAIL=0).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5tail}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
T="timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread"
echo "tests" &&
$T tests/test_schedules_gpu.py -k "tail" > "$OUT/pytest_tail.txt" 2>&1 &&
$T tests/test_guard_gpu.py > "$OUT/pytest_guard.txt" 2>&1 &&
echo "A/B" &&
for r in 1 2; do
  for t in 1 0; do
    MNIST_AMD_WGRAD_TAIL=$t timeout -k 10 180 python bench.py --model mlp --dtype bf16 --no-eval --batch 8192 --steps 2000 --warmup 50 >> "$OUT/ab_mlp8192_tail$t.jsonl" 2>> "$OUT/ab.err" || exit 1
    MNIST_AMD_WGRAD_TAIL=$t timeout -k 10 180 python bench.py --model mlp --dtype bf16 --no-eval --batch 4096 --steps 2000 --warmup 50 >> "$OUT/ab_mlp4096_tail$t.jsonl" 2>> "$OUT/ab.err" || exit 1
    MNIST_AMD_CONV_TAIL=$t timeout -k 10 180 python bench.py --model lenet5 --dtype bf16 --no-eval --batch 128 --steps 5000 --warmup 200 >> "$OUT/ab_lenet128bf16_tail$t.jsonl" 2>> "$OUT/ab.err" || exit 1
    MNIST_AMD_CONV_TAIL=$t timeout -k 10 180 python bench.py --model lenet5 --dtype fp32 --no-eval --batch 128 --steps 5000 --warmup 200 >> "$OUT/ab_lenet128fp32_tail$t.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
done
rc=$?
echo "rc=$rc"
exit $rc
