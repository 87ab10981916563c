#!/bin/bash
# Same-box A/B: current tree vs ab/<name> (see ab_prepare.sh), interleaved, 2000 steps each.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
NAME=${1:-base}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-eval "$@" > "$OUT/ab_cur_$rep.log" 2>&1 || exit 1
  echo "cur   rep$rep $(python scripts/summarize.py bench $OUT/ab_cur_$rep.log)"
  (cd "ab/$NAME" && timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-eval "$@" > "$OUT/ab_${NAME}_$rep.log" 2>&1) || exit 1
  echo "$NAME rep$rep $(python scripts/summarize.py bench $OUT/ab_${NAME}_$rep.log)"
done
