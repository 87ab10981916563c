#!/bin/bash
# streaming-store A/B: numerics gate, kernel-boundary stamps of base and current, driver-shape + long benches
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-nt}
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_gpu.py tests/test_schedules_gpu.py > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
(cd ab/base && timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_base.log" 2>&1) || exit 1
timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_cur.log" 2>&1 || exit 1
grep boundaries "$OUT/${TAG}_stamps_base.log" "$OUT/${TAG}_stamps_cur.log"
grep "span" "$OUT/${TAG}_stamps_base.log" "$OUT/${TAG}_stamps_cur.log"
bash scripts/r3_driver_ab.sh "${TAG}ab" -
