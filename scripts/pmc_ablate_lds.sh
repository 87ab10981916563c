#!/bin/bash
# LDS bank-conflict attribution: one counter pass per conv-kernel phase ablation (MNIST_AMD_ABLATE bits).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-pmcab}; shift
cd /tmp && export TMPDIR=/tmp
for ab in "$@"; do
  MNIST_AMD_ABLATE=$ab timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    --kernel-trace --output-format csv -d "$OUT/${TAG}_$ab" -o run -- python3 "$OUT/../bench.py" --steps 3 --warmup 1 --no-eval > "$OUT/${TAG}_$ab.log" 2>&1 || { echo "fail $ab"; exit 1; }
  echo "== ABLATE=$ab"; python3 "$OUT/../scripts/summarize.py" pmc "$OUT/${TAG}_$ab/run_counter_collection.csv" | grep conv
done
