#!/bin/bash
# Round 5: where the concurrent LeNet step loses time between kernels -- a fork/join micro-benchmark in a captured
# graph, then kernel traces of the concurrent and serial schedules at B=8192 (--plan fixed: no calibration).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5gaps}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 120 python -u scripts/diag/fork_join.py > "$OUT/fork_join.txt" 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
MNIST_AMD_CONCURRENT=1 timeout -k 10 240 rocprofv3 --kernel-trace -d "$OUT/conc" -o run --output-format csv -- python3 "$ROOT/bench.py" --no-eval --plan fixed --steps 40 --warmup 10 > "$OUT/conc.log" 2>&1 &&
MNIST_AMD_CONCURRENT=0 timeout -k 10 240 rocprofv3 --kernel-trace -d "$OUT/serial" -o run --output-format csv -- python3 "$ROOT/bench.py" --no-eval --plan fixed --steps 40 --warmup 10 > "$OUT/serial.log" 2>&1 &&
MNIST_AMD_CONCURRENT=1 timeout -k 10 180 python3 "$ROOT/bench.py" --no-eval --plan fixed --steps 2000 --warmup 50 > "$OUT/conc_bench.jsonl" 2>&1 &&
MNIST_AMD_CONCURRENT=0 timeout -k 10 180 python3 "$ROOT/bench.py" --no-eval --plan fixed --steps 2000 --warmup 50 > "$OUT/serial_bench.jsonl" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
