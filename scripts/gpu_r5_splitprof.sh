#!/bin/bash
# Round 5: where the fp32 split build (pytorch_ddp_mnist_amd/_C_split*.so) gains and loses -- per-kernel times
# (rocprofv3 --kernel-trace --stats) and per-phase stamps, exact build vs split build:
#   scripts/gpu_r5_splitprof.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5splitprof}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
SPLIT=$(cd "$ROOT" && ls "$ROOT"/pytorch_ddp_mnist_amd/_C_split*.so | head -1)
cd /tmp && export TMPDIR=/tmp
prof() {  # variant, name, bench args...
  local v=$1 name=$2; shift 2
  if [ "$v" = split ]; then export MNIST_AMD_C_PATH=$SPLIT; else unset MNIST_AMD_C_PATH; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/${v}_$name" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-eval "$@" > "$OUT/${v}_$name.log" 2>&1
}
for v in exact split; do
  prof $v f8192 --dtype fp32 --steps 50 --warmup 5 &&
  prof $v f1024 --dtype fp32 --batch 1024 --steps 200 --warmup 20 &&
  prof $v mlpf8192 --model mlp --dtype fp32 --batch 8192 --steps 200 --warmup 20 || { echo "prof $v failed"; exit 1; }
  if [ "$v" = split ]; then export MNIST_AMD_C_PATH=$SPLIT; else unset MNIST_AMD_C_PATH; fi
  (cd "$ROOT" && STAMP_DTYPE=fp32 timeout -k 10 120 python scripts/stamps.py > "$OUT/${v}_stamps_f8192.log" 2>&1 &&
   STAMP_DTYPE=fp32 STAMP_BATCH=1024 timeout -k 10 120 python scripts/stamps.py > "$OUT/${v}_stamps_f1024.log" 2>&1) ||
    { echo "stamps $v failed"; exit 1; }
done
echo rc=0
