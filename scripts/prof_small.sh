#!/bin/bash
# Kernel profiles of the small-batch reference configs (MLP fp32 B=128, LeNet fp32 B=128).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-small}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 300 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 50 --no-eval > "$OUT/${TAG}_bench.log" 2>&1 &&
timeout -k 10 300 python bench.py --model lenet5 --dtype fp32 --batch 128 --steps 2000 --warmup 50 --no-eval >> "$OUT/${TAG}_bench.log" 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof_mlp" -o run --output-format csv -- python3 "$OUT/../bench.py" --model mlp --dtype fp32 --batch 128 --steps 50 --warmup 5 --no-eval > "$OUT/${TAG}_prof.log" 2>&1) &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof_lenet" -o run --output-format csv -- python3 "$OUT/../bench.py" --model lenet5 --dtype fp32 --batch 128 --steps 50 --warmup 5 --no-eval >> "$OUT/${TAG}_prof.log" 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
