#!/bin/bash
# Round 5: fp32 GEMMs as exact 3-part bf16 splits on 16x16x32 MFMAs (opt-in build -DMNIST_AMD_F32_SPLIT,
# pytorch_ddp_mnist_amd/_C_split*.so) against the exact fp32 MFMAs of the working tree's _C:
# MFMA issue rates, the fp32 numerics tests on the split build, then interleaved fp32 benches.
#   scripts/gpu_r5_split.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5split}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
SPLIT=$(ls pytorch_ddp_mnist_amd/_C_split*.so | head -1)
echo "mfma rates" &&
timeout -k 10 60 scripts/diag/mfma_rate > "$OUT/mfma_rate.txt" 2>&1 &&
echo "split-build numerics" &&
MNIST_AMD_C_PATH=$SPLIT timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -m gpu -x -v -k "fp32 or f32" --timeout 120 --timeout-method thread > "$OUT/pytest_split.txt" 2>&1
echo "pytest rc=$?" >> "$OUT/pytest_split.txt"
echo "A/B"
CS=("--dtype fp32 --batch 8192 --steps 300 --warmup 20" "--dtype fp32 --batch 1024 --steps 1000 --warmup 50"
    "--dtype fp32 --batch 128 --steps 3000 --warmup 100" "--model mlp --dtype fp32 --batch 128 --steps 3000 --warmup 100"
    "--model mlp --dtype fp32 --batch 8192 --steps 1000 --warmup 50")
for r in 1 2; do
  i=0
  for c in "${CS[@]}"; do
    timeout -k 10 180 python bench.py --no-eval $c >> "$OUT/ab_${i}_exact.jsonl" 2>> "$OUT/ab.err" || exit 1
    MNIST_AMD_C_PATH=$SPLIT timeout -k 10 180 python bench.py --no-eval $c >> "$OUT/ab_${i}_split.jsonl" 2>> "$OUT/ab.err" || exit 1
    i=$((i+1))
  done
done
echo "rc=0"
