#!/bin/bash
# Round-2 evidence package of the current tree: GPU tests, driver-shaped + long benches (LeNet, MLP),
# kernel stats, 4 PMC passes + table.  Outputs gpurun_out/${TAG}_*; copy the summaries to profiles/.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-fin}
cd "$ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
: > "$OUT/${TAG}_bench.jsonl"
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --steps 2000 --warmup 100 >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 100 >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --model mlp --dtype fp32 --batch 128 --steps 20 --warmup 5 >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --model mlp --dtype bf16 --batch 8192 --steps 1000 --warmup 50 >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --model mlp --dtype bf16 --batch 8192 --steps 20 --warmup 5 >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --dtype fp32 --steps 200 --warmup 20 >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
python scripts/summarize.py bench "$OUT/${TAG}_bench.jsonl"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-eval > "$OUT/${TAG}_prof.log" 2>&1) || exit 1
python scripts/summarize.py stats "$OUT/${TAG}_prof/run_kernel_stats.csv" 8
bash scripts/pmc_final.sh "${TAG}pmc" || exit 1
python scripts/pmc_table.py "$OUT/${TAG}pmc" > "$OUT/${TAG}_pmc_table.md" && cat "$OUT/${TAG}_pmc_table.md"
