#!/bin/bash
# Kernel-time profiles (rocprofv3 --kernel-trace --stats, one run per config) and phase stamps of the
# BASELINE configs:  scripts/prof_configs.sh TAG [config ...]
#   configs: lenet (LeNet-5 bf16 B=8192, driver shape) | mlp8k (MLP bf16 B=8192, Dropout 0.2)
#            mlp128 (MLP fp32 B=128) | lenet128 (LeNet-5 bf16 B=128) | lenet128f (fp32 B=128)
#            lenetf (LeNet-5 fp32 B=8192) | stamps (head/conv stamps, concurrent vs serial schedule)
#            stampsmlp (MLP bf16 B=8192 head/wgrad stamps)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-prof}; shift
CONFIGS=${*:-lenet mlp8k}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
prof() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_$name" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-eval "$@" > "$OUT/${TAG}_$name.log" 2>&1
}
for c in $CONFIGS; do
  case $c in
    lenet) prof lenet --steps 20 --warmup 5 ;;
    mlp8k) prof mlp8k --model mlp --dtype bf16 --batch 8192 --steps 200 --warmup 20 ;;
    mlp128) prof mlp128 --model mlp --dtype fp32 --batch 128 --steps 500 --warmup 20 ;;
    lenet128) prof lenet128 --batch 128 --steps 500 --warmup 20 ;;
    lenet128f) prof lenet128f --dtype fp32 --batch 128 --steps 500 --warmup 20 ;;
    lenetf) prof lenetf --dtype fp32 --steps 50 --warmup 5 ;;
    stamps)
      (cd "$ROOT" && timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_conc.log" 2>&1 &&
       MNIST_AMD_CONCURRENT=0 timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_serial.log" 2>&1) ;;
    stampsmlp)
      (cd "$ROOT" && STAMP_MODEL=mlp STAMP_DTYPE=bf16 timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_mlp.log" 2>&1) ;;
    *) echo "unknown config $c"; false ;;
  esac || { echo "config $c failed"; exit 1; }
done
echo done
