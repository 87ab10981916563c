#!/bin/bash
# GPU runtime + numerics gate, then driver-shape / long A/B vs ab/base (deferred join and friends)
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dj}; shift
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_runtime.py tests/test_native_gpu.py tests/test_schedules_gpu.py > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
bash scripts/r3_driver_ab.sh "${TAG}ab" "$@"
