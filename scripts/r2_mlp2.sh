#!/bin/bash
# MLP small-batch path: GPU numerics + runtime tests, MLP/LeNet benches, MLP kernel stats
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-mlp2}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_gpu.py tests/test_gpu_runtime.py tests/test_schedules_gpu.py > $OUT/${T}_pytest.log 2>&1 || { tail -40 $OUT/${T}_pytest.log; exit 1; }
tail -1 $OUT/${T}_pytest.log
for i in 1 2; do
timeout -k 10 120 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 100 > $OUT/${T}_mlp128_$i.json 2>&1 || exit 1
python scripts/summarize.py bench $OUT/${T}_mlp128_$i.json
done
timeout -k 10 120 python bench.py --model mlp --dtype bf16 --batch 8192 --steps 1000 --warmup 50 > $OUT/${T}_mlp8k.json 2>&1 || exit 1
python scripts/summarize.py bench $OUT/${T}_mlp8k.json
timeout -k 10 120 python bench.py --steps 2000 --warmup 100 --no-eval > $OUT/${T}_lenet.json 2>&1 || exit 1
python scripts/summarize.py bench $OUT/${T}_lenet.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${T}_prof" -o run --output-format csv -- python3 "$OUT/../bench.py" --model mlp --dtype fp32 --batch 128 --steps 200 --warmup 10 --no-eval > "$OUT/${T}_prof.log" 2>&1) || exit 1
python scripts/summarize.py stats "$OUT/${T}_prof/run_kernel_stats.csv" 6
