#!/bin/bash
# One GPU session: numerics tests, headline bench, reference-config bench, kernel profile.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-run}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -q -x > "$OUT/${TAG}_pytest.log" 2>&1 &&
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > "$OUT/${TAG}_bench.log" 2>&1 &&
timeout -k 10 300 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 50 >> "$OUT/${TAG}_bench.log" 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- python3 "$OUT/../bench.py" --steps 20 --warmup 5 > "$OUT/${TAG}_prof.log" 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
