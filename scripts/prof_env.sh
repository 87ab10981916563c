#!/bin/bash
# Kernel-time profile per env setting: prof_env.sh TAG "ENV=A" "ENV=B" ...
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for kv in "$@"; do
  env $kv timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_$i" -o run --output-format csv -- python3 "$OUT/../bench.py" --steps 30 --warmup 5 --no-eval ${BENCH_ARGS} > "$OUT/${TAG}_$i.log" 2>&1 || { echo "fail $kv"; exit 1; }
  echo "== $kv"; python3 "$OUT/../scripts/summarize.py" stats "$OUT/${TAG}_$i/run_kernel_stats.csv" 5
  i=$((i+1))
done
