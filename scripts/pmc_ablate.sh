#!/bin/bash
# LDS counters of the conv kernels with phases ablated (attributes bank conflicts to phases).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-pa}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for m in ${ABL_SET:-0 1 2 4}; do
  MNIST_AMD_ABLATE=$m timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
    --kernel-trace --output-format csv -d "$OUT/${TAG}_$m" -o run -- python3 "$OUT/../bench.py" --steps 3 --warmup 1 --no-eval > "$OUT/${TAG}_$m.log" 2>&1 || { echo "fail $m"; exit 1; }
done
echo done
