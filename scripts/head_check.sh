#!/bin/bash
# Head-kernel iteration: native numerics tests, phase stamps, headline + MLP benches.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-head}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
timeout -k 10 120 python scripts/stamps.py || exit 1
for args in "" "--model mlp --dtype fp32 --batch 128" "--model mlp --dtype bf16 --batch 8192"; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-eval $args > "$OUT/${TAG}_b.log" 2>&1 || { cat "$OUT/${TAG}_b.log"; exit 1; }
  echo "$(python scripts/summarize.py bench $OUT/${TAG}_b.log)"
done
