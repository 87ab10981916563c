#!/bin/bash
# Round-2 GPU check: GPU tests, driver-shaped bench, kernel stats, two PMC passes.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-r2}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1 &&
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> "$OUT/${TAG}_bench.log" 2>&1 || exit 1; done &&
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-eval >> "$OUT/${TAG}_bench.log" 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- python3 "$OUT/../bench.py" --steps 20 --warmup 5 --no-eval > "$OUT/${TAG}_prof.log" 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
