#!/bin/bash
# MLP small-batch (reference config) A/B: GPU runtime + numerics gate, then base vs current, interleaved
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-mlp}
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_runtime.py tests/test_native_gpu.py > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
for rep in 1 2 3; do
  for v in base cur; do
    d=.; [ $v = base ] && d=ab/base
    (cd $d && timeout -k 10 200 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 100 --no-eval > "$OUT/${TAG}_${v}_$rep.log" 2>/dev/null) || exit 1
    echo "$v 2000 $(python scripts/summarize.py bench $OUT/${TAG}_${v}_$rep.log)"
    (cd $d && timeout -k 10 200 python bench.py --model mlp --dtype fp32 --batch 128 --steps 20 --warmup 5 > "$OUT/${TAG}_${v}_d$rep.log" 2>/dev/null) || exit 1
    echo "$v 20   $(python scripts/summarize.py bench $OUT/${TAG}_${v}_d$rep.log)"
  done
done
(STAMP_MODEL=mlp STAMP_DTYPE=fp32 STAMP_BATCH=128 timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps.log" 2>&1) || exit 1
tail -12 "$OUT/${TAG}_stamps.log"
