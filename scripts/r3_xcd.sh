#!/bin/bash
# XCD-contiguous mapping: full GPU suite, stamps (boundaries, per-phase, dispatch check), driver A/B vs ab/base
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-xcd}
cd "$ROOT" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
(cd ab/base && timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_base.log" 2>&1) || exit 1
timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_cur.log" 2>&1 || exit 1
grep -E "boundaries|span|stage X|XCD g" "$OUT/${TAG}_stamps_base.log" "$OUT/${TAG}_stamps_cur.log"
bash scripts/r3_driver_ab.sh "${TAG}ab" -
