#!/bin/bash
# Multi-GPU-path checks on one GPU: emulation / watchdog / autotune / schedule tests, then benches.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-mg}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
PT="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 300 $PT tests/test_multigpu_gpu.py -k "autotune or emulation" > "$OUT/${TAG}_pytest1.log" 2>&1 &&
timeout -k 10 900 $PT tests/test_schedules_gpu.py tests/test_gpu_runtime.py > "$OUT/${TAG}_pytest2.log" 2>&1 &&
timeout -k 10 300 $PT tests/test_multigpu_gpu.py -k watchdog > "$OUT/${TAG}_pytest3.log" 2>&1 &&
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/${TAG}_bench.log" 2>&1 &&
timeout -k 10 120 python bench.py --steps 300 --warmup 20 --comm-world1 --no-eval >> "$OUT/${TAG}_bench.log" 2>&1 &&
timeout -k 10 120 python bench.py --steps 300 --warmup 20 --no-eval >> "$OUT/${TAG}_bench.log" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
