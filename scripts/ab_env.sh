#!/bin/bash
# A/B a runtime knob on the headline bench: ab_env.sh TAG "ENV=A" "ENV=B" ... (2000 steps each, interleaved twice)
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for rep in 1 2; do
  i=0
  for kv in "$@"; do
    env $kv timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-eval ${BENCH_ARGS} > "$OUT/${TAG}_${i}_${rep}.log" 2>&1 || exit 1
    echo "$kv rep$rep $(python scripts/summarize.py bench $OUT/${TAG}_${i}_${rep}.log)"
    i=$((i+1))
  done
done
