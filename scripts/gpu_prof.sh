#!/bin/bash
# Evidence pass of the current tree: phase stamps (LeNet fused default, MLP bf16) and the 4-pass PMC table of
# LeNet-5 bf16 / LeNet-5 fp32 / MLP bf16 at B=8192.   scripts/gpu_prof.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-prof}
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_lenet.log" 2>&1 &&
STAMP_MODEL=mlp timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_mlp.log" 2>&1 &&
BENCH_ARGS="" bash scripts/pmc_final.sh ${TAG}_pmc_lenet &&
BENCH_ARGS="--dtype fp32" bash scripts/pmc_final.sh ${TAG}_pmc_lenetf &&
BENCH_ARGS="--model mlp" bash scripts/pmc_final.sh ${TAG}_pmc_mlp
rc=$?; echo "rc=$rc"; exit $rc
