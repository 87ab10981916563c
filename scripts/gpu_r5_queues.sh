#!/bin/bash
# Round 5: does the fork/join cost of a captured two-stream graph depend on the hardware-queue count?
# fork_join micro-benchmark and the concurrent / serial LeNet B=8192 step (--plan fixed) per GPU_MAX_HW_QUEUES.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5queues}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
for q in 2 8 4; do
  for c in 1 0; do
    GPU_MAX_HW_QUEUES=$q MNIST_AMD_CONCURRENT=$c timeout -k 10 180 python bench.py --no-eval --plan fixed --steps 2000 --warmup 50 >> "$OUT/bench_q${q}_c${c}.jsonl" 2>> "$OUT/bench.err" || exit 1
  done
done
echo "rc=0"
