#!/bin/bash
# One GPU session of the current tree (run through gpurun from the repo root):
#   scripts/gpu_session.sh TAG [pytest-selector]
# GPU tests, the driver-shape headline bench, the reference-MLP bench (Dropout 0.2 in the step), and the
# world-1 communicator bench (comm_profile).  Every GPU step has its own time limit and the chain stops at
# the first failure; results land in gpurun_out/TAG_*.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-run}
SEL=${2:-tests}
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1 &&
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/${TAG}_bench.jsonl" 2> "$OUT/${TAG}_bench.err" &&
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 >> "$OUT/${TAG}_bench.jsonl" 2>> "$OUT/${TAG}_bench.err" &&
timeout -k 10 180 python bench.py --steps 2000 --warmup 50 >> "$OUT/${TAG}_bench.jsonl" 2>> "$OUT/${TAG}_bench.err" &&
timeout -k 10 180 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 50 >> "$OUT/${TAG}_bench.jsonl" 2>> "$OUT/${TAG}_bench.err" &&
timeout -k 10 180 python bench.py --model mlp --dtype bf16 --batch 8192 --steps 1000 --warmup 50 >> "$OUT/${TAG}_bench.jsonl" 2>> "$OUT/${TAG}_bench.err" &&
timeout -k 10 180 python bench.py --comm-world1 --steps 200 --warmup 20 >> "$OUT/${TAG}_bench.jsonl" 2>> "$OUT/${TAG}_bench.err" &&
timeout -k 10 180 python bench.py --comm-world1 --model mlp --dtype bf16 --steps 200 --warmup 20 >> "$OUT/${TAG}_bench.jsonl" 2>> "$OUT/${TAG}_bench.err"
rc=$?
echo "rc=$rc"
exit $rc
