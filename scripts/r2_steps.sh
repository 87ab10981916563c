#!/bin/bash
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 120 python scripts/step_times.py --warmup 5 --steps 60 > "$OUT/steps.log" 2>&1 &&
timeout -k 10 120 python scripts/step_times.py --warmup 200 --steps 60 >> "$OUT/steps.log" 2>&1 &&
timeout -k 10 120 python scripts/step_times.py --warmup 5 --steps 60 --idle-ms 50 >> "$OUT/steps.log" 2>&1
echo rc=$?
