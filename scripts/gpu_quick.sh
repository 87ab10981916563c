#!/bin/bash
# Quick GPU check of a change: the native numerics tests, stamps (kernel gaps), driver-shape benches.
#   scripts/gpu_quick.sh TAG [extra bench args]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-quick}; shift
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1 &&
timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps.log" 2>&1 &&
STAMP_MODEL=mlp timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_mlp.log" 2>&1 &&
for i in 1 2; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-eval "$@" >> "$OUT/${TAG}_bench.jsonl" || exit 1; done &&
timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-eval "$@" >> "$OUT/${TAG}_bench.jsonl" &&
timeout -k 10 120 python bench.py --model mlp --steps 1000 --warmup 50 --no-eval >> "$OUT/${TAG}_bench.jsonl" &&
timeout -k 10 120 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 50 --no-eval >> "$OUT/${TAG}_bench.jsonl"
rc=$?; echo "rc=$rc"; exit $rc
