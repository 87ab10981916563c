#!/bin/bash
# Round 5: MLP weight-gradient tail update (head.hip wgrad_tail) -- numerics, then an interleaved A/B against the
# separate reduce + SGD kernel (MNIST_AMD_WGRAD_TAIL=0) on MLP bf16 B=8192 and B=4096, then kernel stats.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5tail}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
B="timeout -k 10 180 python bench.py --model mlp --dtype bf16 --no-eval"
echo "tests" &&
timeout -k 10 900 python -u -m pytest tests/test_schedules_gpu.py tests/test_native_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/pytest.txt" 2>&1 &&
echo "A/B" &&
for r in 1 2; do
  for t in 1 0; do
    MNIST_AMD_WGRAD_TAIL=$t $B --batch 8192 --steps 2000 --warmup 50 >> "$OUT/ab_8192_tail$t.jsonl" 2>> "$OUT/ab.err" || exit 1
    MNIST_AMD_WGRAD_TAIL=$t $B --batch 4096 --steps 2000 --warmup 50 >> "$OUT/ab_4096_tail$t.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
done &&
echo "profile" &&
timeout -k 10 600 bash scripts/prof_configs.sh "$TAG/k" mlp8k > "$OUT/prof.log" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
