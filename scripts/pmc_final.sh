#!/bin/bash
# Hardware-counter table of the current tree: 4 passes, each its own rocprofv3 run (--pmc with
# --kernel-trace only, as the pool requires).  Program directly after "--".
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-pmcf}
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/${TAG}_$n" -o run -- \
    python3 "$OUT/../bench.py" --steps 3 --warmup 1 --no-eval $BENCH_ARGS > "$OUT/${TAG}_$n.log" 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT &&
run c FETCH_SIZE GRBM_GUI_ACTIVE &&
run d WRITE_SIZE GRBM_GUI_ACTIVE
rc=$?
echo "rc=$rc"
exit $rc
