#!/bin/bash
# Same-box A/B of several builds: ab_multi.sh "cur lds r1k" [bench args]   (cur = this tree, X = ab/X)
# 3 interleaved reps of the 2000-step bench per variant, then one rocprofv3 --stats run per variant.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
VARS=$1; shift
cd "$ROOT" || exit 1
dir() { if [ "$1" = cur ]; then echo "$ROOT"; else echo "$ROOT/ab/$1"; fi; }
for rep in 1 2 3; do
  for v in $VARS; do
    (cd "$(dir $v)" && timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --no-eval "$@" > "$OUT/abm_${v}_$rep.log" 2>&1) || exit 1
    echo "$v rep$rep $(python scripts/summarize.py bench $OUT/abm_${v}_$rep.log)"
  done
done
for v in $VARS; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/abm_${v}_prof" -o run --output-format csv -- python3 "$(dir $v)/bench.py" --steps 50 --warmup 10 --no-eval "$@" > "$OUT/abm_${v}_prof.log" 2>&1) || exit 1
  echo "== $v"; python scripts/summarize.py stats "$OUT/abm_${v}_prof/run_kernel_stats.csv" 5
done
