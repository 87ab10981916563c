#!/bin/bash
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/hoist_pytest.log" 2>&1 || { tail -30 "$OUT/hoist_pytest.log"; exit 1; }
tail -1 "$OUT/hoist_pytest.log"
bash scripts/ab_bench.sh base
