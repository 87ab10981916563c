#!/bin/bash
# Quick A/B loop: numerics tests, long bench, stamps, kernel stats.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-q}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_gpu.py tests/test_schedules_gpu.py > "$OUT/${TAG}_pytest.log" 2>&1 &&
timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-eval > "$OUT/${TAG}_bench.log" 2>&1 &&
timeout -k 10 120 python bench.py --steps 20 --warmup 5 >> "$OUT/${TAG}_bench.log" 2>&1 &&
timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps.log" 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- python3 "$OUT/../bench.py" --steps 20 --warmup 5 --no-eval > "$OUT/${TAG}_prof.log" 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
