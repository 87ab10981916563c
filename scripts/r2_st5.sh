#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-st}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for ab in 0 1; do
  MNIST_AMD_HEAD_ABLATE=$ab timeout -k 10 120 python scripts/stamps.py > $OUT/${T}_stamps_$ab.log 2>&1 || { tail $OUT/${T}_stamps_$ab.log; exit 1; }
  echo "== ablate $ab"; grep -A 10 "^head" $OUT/${T}_stamps_$ab.log
done
