#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-st2}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_gpu.py tests/test_gpu_runtime.py -k "mlp or fused or replay or determinism" > $OUT/${T}_pytest.log 2>&1 || { grep -v "^  File" $OUT/${T}_pytest.log | tail -30; exit 1; }
tail -1 $OUT/${T}_pytest.log
STAMP_MODEL=mlp STAMP_DTYPE=fp32 STAMP_BATCH=128 timeout -k 10 120 python scripts/stamps.py > $OUT/${T}_stamps.log 2>&1 || { tail $OUT/${T}_stamps.log; exit 1; }
grep -v amdgpu.ids $OUT/${T}_stamps.log
timeout -k 10 120 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 100 > $OUT/${T}_mlp128.json 2>&1 || exit 1
python scripts/summarize.py bench $OUT/${T}_mlp128.json
