#!/bin/bash
# Same-box A/B of build or runtime variants (the one A/B driver; replaces the round-4/5 session scripts).
#
#   scripts/ab.sh TAG [-t "TEST FILES"] [-r REPS] "BENCH ARGS" VARIANT [VARIANT ...]
#
# VARIANT: "-" (as is) or space-separated env assignments, e.g. "MNIST_AMD_CONCURRENT=0" or
#          "MNIST_AMD_C_PATH=pytorch_ddp_mnist_amd/_C_ab.cpython-310-x86_64-linux-gnu.so" (a previous revision's
#          extension built on the CPU host by scripts/build_ab.sh).
# -t: pytest files run once per variant (under its env, -m gpu) before any bench; a failure ends the call.
# -r: rounds (default 2); every round runs every variant once, in order, so variants interleave on the box.
# Each bench line is summarised (ms/step, img/s, calibration timings) into gpurun_out/TAG_ab.txt.
# Every GPU step has its own time limit and the chain stops at the first failure (no retries).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=$1; shift
TESTS=""; REPS=2
while [ $# -gt 0 ]; do
  case $1 in
    -t) TESTS=$2; shift 2 ;;
    -r) REPS=$2; shift 2 ;;
    *) break ;;
  esac
done
ARGS=$1; shift
mkdir -p "$OUT"
cd "$ROOT" || exit 1
if [ -n "$TESTS" ]; then
  i=0
  for kv in "$@"; do
    [ "$kv" = "-" ] && kv=""
    env $kv timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 240 --timeout-method thread \
      > "$OUT/${TAG}_pytest_$i.txt" 2>&1 || { echo "tests failed under [$kv]"; tail -20 "$OUT/${TAG}_pytest_$i.txt"; exit 1; }
    echo "[$kv] $(tail -1 "$OUT/${TAG}_pytest_$i.txt")" | tee -a "$OUT/${TAG}_ab.txt"
    i=$((i+1))
  done
fi
for rep in $(seq 1 "$REPS"); do
  i=0
  for kv in "$@"; do
    [ "$kv" = "-" ] && kv=""
    log="$OUT/${TAG}_${i}_${rep}.log"
    env $kv timeout -k 10 240 python bench.py --no-eval $ARGS > "$log" 2>&1 || { tail -5 "$log"; exit 1; }
    echo "[$kv] rep$rep $(python scripts/summarize.py bench "$log")" | tee -a "$OUT/${TAG}_ab.txt"
    i=$((i+1))
  done
done
echo "rc=0"
