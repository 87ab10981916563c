#!/bin/bash
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for v in 4 8 16; do
  MNIST_AMD_SPLIT_NWV=$v timeout -k 10 200 python bench.py --model mlp --dtype fp32 --batch 128 --steps 2000 --warmup 50 --no-eval > "$OUT/nwv_mlp_$v.log" 2>&1 || exit 1
  MNIST_AMD_SPLIT_NWV=$v timeout -k 10 200 python bench.py --model lenet5 --dtype fp32 --batch 128 --steps 2000 --warmup 50 --no-eval > "$OUT/nwv_lenet_$v.log" 2>&1 || exit 1
done
