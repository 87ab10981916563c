#!/bin/bash
# driver-shaped LeNet x3, MLP fp32 B=128 and MLP bf16 B=8192 benches, kernel stats of the MLP small step
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-mlp}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/${T}_drv$i.json 2>/dev/null || exit 1
  python scripts/summarize.py bench $OUT/${T}_drv$i.json; done
timeout -k 10 120 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 100 > $OUT/${T}_mlp128.json 2>&1 || exit 1
python scripts/summarize.py bench $OUT/${T}_mlp128.json
timeout -k 10 120 python bench.py --model mlp --dtype bf16 --batch 8192 --steps 1000 --warmup 50 > $OUT/${T}_mlp8k.json 2>&1 || exit 1
python scripts/summarize.py bench $OUT/${T}_mlp8k.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${T}_prof" -o run --output-format csv -- python3 "$OUT/../bench.py" --model mlp --dtype fp32 --batch 128 --steps 200 --warmup 10 --no-eval > "$OUT/${T}_prof.log" 2>&1) || exit 1
python scripts/summarize.py stats "$OUT/${T}_prof/run_kernel_stats.csv" 8
