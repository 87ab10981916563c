#!/bin/bash
# numerics gate, then same-box A/B (ab_multi.sh) of the given variants
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_gpu.py tests/test_schedules_gpu.py > "$OUT/ab_pytest.log" 2>&1 || { tail -30 "$OUT/ab_pytest.log"; exit 1; }
tail -1 "$OUT/ab_pytest.log"
bash scripts/ab_multi.sh "$@"
