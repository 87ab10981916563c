#!/bin/bash
# Round 5: localise the MLP weight-gradient tail's difference (scripts/diag/tail_diag.py), eager and graph.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r5_taildiag}
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 300 python -u scripts/diag/tail_diag.py --batch 4096 --steps 3 > "$OUT/mlp4096.txt" 2>&1 &&
timeout -k 10 300 python -u scripts/diag/tail_diag.py --batch 128 --steps 3 --model lenet5 > "$OUT/lenet128.txt" 2>&1 &&
timeout -k 10 300 python -u scripts/diag/tail_diag.py --batch 128 --steps 3 --model lenet5 --dtype fp32 > "$OUT/lenet128f.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
