#!/bin/bash
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for m in split recap_join join_split autotune; do
  MNIST_AMD_SEGV_TRACE=1 MNIST_AMD_TRACE=1 timeout -k 10 60 python -u scripts/diag_autotune.py $m >> "$OUT/diag.log" 2>&1 || { echo "FAIL $m rc=$?" >> "$OUT/diag.log"; exit 1; }
done
echo ok
