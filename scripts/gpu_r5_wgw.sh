#!/bin/bash
# Round 5: the FC weight gradient on conv_bwd's spare waves (conv_bwd_wg_kernel) -- bitwise test, then interleaved
# A/B of the pinned schedules (--plan fixed) and the calibrated default, then a kernel trace of the new schedule.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5wgw}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
B="timeout -k 10 180 python bench.py --no-eval"
echo "test" &&
timeout -k 10 900 python -u -m pytest tests/test_schedules_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -k "wgwaves" > "$OUT/pytest_wgw.txt" 2>&1 &&
echo "A/B" &&
for r in 1 2; do
  MNIST_AMD_CONCURRENT=1 $B --plan fixed --steps 2000 --warmup 50 >> "$OUT/ab_conc.jsonl" 2>> "$OUT/ab.err" &&
  MNIST_AMD_WGWAVES=1 MNIST_AMD_CONCURRENT=0 $B --plan fixed --steps 2000 --warmup 50 >> "$OUT/ab_wgw.jsonl" 2>> "$OUT/ab.err" &&
  $B --steps 2000 --warmup 50 >> "$OUT/ab_auto.jsonl" 2>> "$OUT/ab.err" &&
  $B --batch 2048 --steps 2000 --warmup 50 >> "$OUT/ab_auto2048.jsonl" 2>> "$OUT/ab.err" || exit 1
done &&
cd /tmp && export TMPDIR=/tmp &&
MNIST_AMD_WGWAVES=1 MNIST_AMD_CONCURRENT=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace_wgw" -o run --output-format csv -- python3 "$ROOT/bench.py" --no-eval --plan fixed --steps 40 --warmup 10 > "$OUT/trace_wgw.log" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
