#!/bin/bash
# A/B runtime knobs on one box: ab_env.sh TAG "BENCH ARGS" "ENV=A [ENV2=..]" "ENV=B" ...   ("-" = no env)
# Each variant runs twice, interleaved; one summary line per run is printed (and kept in gpurun_out/TAG_ab.txt).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=$1; ARGS=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for rep in 1 2; do
  i=0
  for kv in "$@"; do
    [ "$kv" = "-" ] && kv=""
    env $kv timeout -k 10 200 python bench.py --no-eval $ARGS > "$OUT/${TAG}_${i}_${rep}.log" 2>&1 || { cat "$OUT/${TAG}_${i}_${rep}.log" | tail -5; exit 1; }
    echo "[$kv] rep$rep $(python scripts/summarize.py bench $OUT/${TAG}_${i}_${rep}.log)" | tee -a "$OUT/${TAG}_ab.txt"
    i=$((i+1))
  done
done
