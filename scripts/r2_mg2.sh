#!/bin/bash
# Multi-GPU path on one GPU, current tree: world-1 RCCL benches (calibration of join / split / split_r16),
# the same without a communicator, and the 2-rank replica test (skipped unless >= 2 GPUs).
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-mg}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
: > "$OUT/${TAG}_bench.jsonl"
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 20 --comm-world1 --no-eval >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py --steps 300 --warmup 20 --no-eval >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --comm-world1 --plan split --no-eval >> "$OUT/${TAG}_bench.jsonl" 2>/dev/null || exit 1
python - "$OUT/${TAG}_bench.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    c = d["config"]
    print(d["ms_per_step"], round(d["value"] / 1e6, 2), "M img/s |", c["comm"][:70], "|", (c.get("plan_autotune") or {}).get("timings_ms"))
PY
timeout -k 10 300 python -u -m pytest -q --timeout 280 --timeout-method thread tests/test_multirank_gpu.py > "$OUT/${TAG}_pytest.log" 2>&1; tail -1 "$OUT/${TAG}_pytest.log"
