#!/bin/bash
# Hardware-counter pass (own run: --pmc with --kernel-trace only, as the pool requires).
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-pmc}
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/${TAG}_counters.txt" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  --kernel-trace --output-format csv -d "$OUT/${TAG}_a" -o run -- python3 "$OUT/../bench.py" --steps 3 --warmup 1 --no-eval "$@" > "$OUT/${TAG}_a.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM \
  --kernel-trace --output-format csv -d "$OUT/${TAG}_b" -o run -- python3 "$OUT/../bench.py" --steps 3 --warmup 1 --no-eval "$@" > "$OUT/${TAG}_b.log" 2>&1
echo "rc=$?"
