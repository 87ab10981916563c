#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-st}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -k "lookahead or fused" > $OUT/${T}_pytest.log 2>&1 || { grep -v "^  File" $OUT/${T}_pytest.log | tail -30; exit 1; }
tail -1 $OUT/${T}_pytest.log
STAMP_MODEL=mlp STAMP_DTYPE=fp32 STAMP_BATCH=128 timeout -k 10 120 python scripts/stamps.py > $OUT/${T}_stamps.log 2>&1 || { tail $OUT/${T}_stamps.log; exit 1; }
grep -v amdgpu.ids $OUT/${T}_stamps.log
for i in 1 2; do
timeout -k 10 120 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 100 > $OUT/${T}_mlp128_$i.json 2>&1 || exit 1
python scripts/summarize.py bench $OUT/${T}_mlp128_$i.json
done
