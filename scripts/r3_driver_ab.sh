#!/bin/bash
# Driver-shape A/B (bench.py --gpus 1 --steps 20 --warmup 5, the harness's command) of ab/base vs the
# current tree and env variants, interleaved; then the same variants at 2000 steps.
#   r3_driver_ab.sh TAG "ENV=A" "ENV=B" ...      ("-" = no env change)
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd "$ROOT" || exit 1
run() {  # name dir env steps warmup
  local name=$1 dir=$2 kv=$3 st=$4 wu=$5
  local log="$OUT/${TAG}_${name}_${st}.log"
  if [ "$kv" = "-" ]; then kv="MNIST_AMD_NOP=1"; fi
  (cd "$dir" && env $kv timeout -k 10 200 python bench.py --gpus 1 --steps $st --warmup $wu >> "$log" 2>/dev/null) || return 1
  echo "$name st=$st $(python "$ROOT/scripts/summarize.py" bench "$log" | tail -1)"
}
for rep in 1 2 3; do
  run base ab/base - 20 5 || exit 1
  i=0
  for kv in "$@"; do run "v$i" . "$kv" 20 5 || exit 1; i=$((i+1)); done
done
for rep in 1 2; do
  run base ab/base - 2000 50 || exit 1
  i=0
  for kv in "$@"; do run "v$i" . "$kv" 2000 50 || exit 1; i=$((i+1)); done
done
