#!/bin/bash
# conv_bwd MODE split: numerics + schedule equivalence, A/B of the split, kernel profile.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-split}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py tests/test_schedules_gpu.py -x -q --timeout 900 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -40 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -1 "$OUT/${TAG}_pytest.log"
bash scripts/ab_env.sh "${TAG}ab" MNIST_AMD_SPLIT_BWD=1 MNIST_AMD_SPLIT_BWD=0 || exit 1
bash scripts/prof_env.sh "${TAG}p" MNIST_AMD_SPLIT_BWD=1
