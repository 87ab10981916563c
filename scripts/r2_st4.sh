#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-st}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 120 python scripts/stamps.py > $OUT/${T}_stamps.log 2>&1 || { tail $OUT/${T}_stamps.log; exit 1; }
grep -v amdgpu.ids $OUT/${T}_stamps.log
