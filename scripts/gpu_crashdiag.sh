#!/bin/bash
# Round-5 crash diagnosis (VERDICT r4 "next round" item 1) on one leased GPU, from the repo root:
#   scripts/gpu_crashdiag.sh TAG
# 1. the command that failed on the driver's box (GPUTEST_r04: bench.py --gpus 2 --comm gloo --model mlp --dtype fp32
#    --batch 128), every launch synchronised and checked (MNIST_AMD_SYNC_DEBUG=1), each rank's stderr in its own file,
#    native backtrace + faulthandler on a host fault;
# 2. the same without the per-launch sync (the driver's timing);
# 3. the full GPU suite (-x, per-test timeout), then smoke().
# Every step has its own time limit; the chain stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-crashdiag}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export MNIST_AMD_SEGV_TRACE=1 PYTHONFAULTHANDLER=1
CMD="bench.py --gpus 2 --comm gloo --model mlp --dtype fp32 --batch 128 --steps 4 --warmup 2 --no-eval --digest"
echo "step 1: sync-debug run" &&
MNIST_AMD_SYNC_DEBUG=1 timeout -k 10 240 python -u $CMD --rank-logs "$OUT/ranks_sync" > "$OUT/sync.out" 2> "$OUT/sync.err" &&
echo "step 2: plain run" &&
timeout -k 10 240 python -u $CMD --rank-logs "$OUT/ranks_plain" > "$OUT/plain.out" 2> "$OUT/plain.err" &&
echo "step 3: GPU suite" &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 &&
echo "step 4: smoke" &&
timeout -k 10 180 python -u __graft_entry__.py smoke > "$OUT/smoke.txt" 2>&1 &&
echo "step 5: bench (driver shape)" &&
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
rc=$?
echo "rc=$rc"
tail -3 "$OUT/pytest_gpu.txt" 2>/dev/null
exit $rc
