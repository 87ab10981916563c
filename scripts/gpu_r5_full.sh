#!/bin/bash
# Round 5: the whole GPU suite + smoke + driver-shape bench on the current tree, then short A/B runs
# (extra arguments: "ab" to also run the MLP FC batch-split A/B).  scripts/gpu_r5_full.sh TAG [ab]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5full}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export MNIST_AMD_SEGV_TRACE=1 PYTHONFAULTHANDLER=1
echo "suite" &&
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 &&
echo "smoke" &&
timeout -k 10 180 python -u __graft_entry__.py smoke > "$OUT/smoke.txt" 2>&1 &&
echo "bench" &&
timeout -k 10 180 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err" &&
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 >> "$OUT/bench.jsonl" 2>> "$OUT/bench.err"
rc=$?
if [ $rc -eq 0 ] && [ "$2" = "ab" ]; then
  echo "A/B"
  for r in 1 2; do
    for s in 16 8 32; do
      MNIST_AMD_FC_SPLITS=$s timeout -k 10 180 python bench.py --model mlp --dtype bf16 --no-eval --batch 8192 --steps 2000 --warmup 50 >> "$OUT/ab_mlp8192_splits$s.jsonl" 2>> "$OUT/ab.err" || { rc=1; break 2; }
    done
  done
fi
echo "rc=$rc"
tail -3 "$OUT/pytest_gpu.txt"
exit $rc
