#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-st}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for tw in 0 1; do
  if [ $tw = 1 ]; then export MNIST_AMD_HEAD_TWICE=1; fi
  timeout -k 10 120 python scripts/stamps.py > $OUT/${T}_stamps_$tw.log 2>&1 || { tail $OUT/${T}_stamps_$tw.log; exit 1; }
  echo "== twice $tw"; grep -A 10 "^head" $OUT/${T}_stamps_$tw.log
done
