#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-mlp3}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -k "fused or multi_step" > $OUT/${T}_pytest.log 2>&1 || { tail -40 $OUT/${T}_pytest.log; exit 1; }
tail -1 $OUT/${T}_pytest.log
timeout -k 10 120 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 100 > $OUT/${T}_mlp128.json 2>&1 || exit 1
python scripts/summarize.py bench $OUT/${T}_mlp128.json
STAMP_MODEL=mlp STAMP_DTYPE=fp32 STAMP_BATCH=128 timeout -k 10 120 python scripts/stamps.py > $OUT/${T}_stamps.log 2>&1 || { tail $OUT/${T}_stamps.log; exit 1; }
cat $OUT/${T}_stamps.log | grep -v amdgpu.ids
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${T}_prof" -o run --output-format csv -- python3 "$OUT/../bench.py" --model mlp --dtype fp32 --batch 128 --steps 200 --warmup 10 --no-eval > "$OUT/${T}_prof.log" 2>&1) || exit 1
python scripts/summarize.py stats "$OUT/${T}_prof/run_kernel_stats.csv" 4
