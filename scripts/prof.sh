#!/bin/bash
# The one profiling driver (replaces prof_configs.sh, pmc_final.sh, prof_env.sh, prof_small.sh, gpu_prof.sh and the
# round-5 gpu_r5_* session scripts).  Run on the GPU box from the repo root:
#
#   scripts/prof.sh stats TAG [CONFIG ...]   rocprofv3 --kernel-trace --stats per BASELINE config
#   scripts/prof.sh pmc   TAG [CONFIG]       hardware counters, 5 passes (each its own --pmc run, --kernel-trace only),
#                                            then: python scripts/pmc_table.py gpurun_out/TAG_CONFIG [--model mlp]
#   scripts/prof.sh stamps TAG [CONFIG ...]  in-kernel wall-clock phase stamps (scripts/stamps.py)
#
# CONFIG: lenet (LeNet-5 bf16 B=8192, driver shape; default) | lenet_serial (same, serial schedule, no calibration)
#         mlp8k (MLP bf16 B=8192, Dropout 0.2) | mlp128 (MLP fp32 B=128) | lenet128 (bf16 B=128) | lenet128f (fp32
#         B=128) | lenetf (LeNet-5 fp32 B=8192)
# Extra environment for a variant: set it on the command line (e.g. MNIST_AMD_WGRAD_SK=1 scripts/prof.sh stats t lenet).
# Every step has its own time limit; the first failure ends the call (no retries).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
MODE=$1; TAG=${2:?tag}; shift 2
CONFIGS=${*:-lenet}
mkdir -p "$OUT"
args_of() {
  case $1 in
    lenet) echo "--steps 20 --warmup 5" ;;
    lenet_serial) echo "--steps 200 --warmup 20 --plan fixed" ;;
    mlp8k) echo "--model mlp --dtype bf16 --batch 8192 --steps 200 --warmup 20" ;;
    mlp128) echo "--model mlp --dtype fp32 --batch 128 --steps 500 --warmup 20" ;;
    lenet128) echo "--batch 128 --steps 500 --warmup 20" ;;
    lenet128f) echo "--dtype fp32 --batch 128 --steps 500 --warmup 20" ;;
    lenetf) echo "--dtype fp32 --steps 50 --warmup 5" ;;
    *) echo "unknown config $1" >&2; return 1 ;;
  esac
}
env_of() {  # per-config environment (the serial single-GPU schedule, pinned)
  [ "$1" = lenet_serial ] && echo "MNIST_AMD_CONCURRENT=0"
}
cd /tmp && export TMPDIR=/tmp
case $MODE in
  stats)
    for c in $CONFIGS; do
      A=$(args_of "$c") || exit 1
      env $(env_of "$c") timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_$c" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --no-eval $A > "$OUT/${TAG}_$c.log" 2>&1 || { echo "stats $c failed"; exit 1; }
      python3 "$ROOT/scripts/summarize.py" stats "$OUT/${TAG}_$c/run_kernel_stats.csv" 8
    done ;;
  pmc)
    c=${CONFIGS%% *}
    A=$(args_of "$c") || exit 1
    A=$(echo "$A" | sed -E 's/--steps [0-9]+/--steps 3/; s/--warmup [0-9]+/--warmup 1/')
    run() {
      local n=$1; shift
      env $(env_of "$c") timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/${TAG}_${c}_$n" -o run -- \
        python3 "$ROOT/bench.py" --no-eval $A > "$OUT/${TAG}_${c}_$n.log" 2>&1
    }
    run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
    run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT &&
    run c FETCH_SIZE GRBM_GUI_ACTIVE &&
    run d WRITE_SIZE GRBM_GUI_ACTIVE &&
    run e SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
      || { echo "pmc pass failed"; exit 1; } ;;
  stamps)
    cd "$ROOT" || exit 1
    for c in $CONFIGS; do
      case $c in
        lenet) E="" ;;
        lenet_serial) E="MNIST_AMD_CONCURRENT=0" ;;
        mlp8k) E="STAMP_MODEL=mlp" ;;
        lenetf) E="STAMP_DTYPE=fp32" ;;
        mlp128) E="STAMP_MODEL=mlp STAMP_BATCH=128 STAMP_DTYPE=fp32" ;;
        lenet128) E="STAMP_BATCH=128" ;;
        *) echo "no stamps config $c"; exit 1 ;;
      esac
      env $E timeout -k 10 120 python scripts/stamps.py > "$OUT/${TAG}_stamps_$c.txt" 2>&1 || { echo "stamps $c failed"; exit 1; }
    done ;;
  *) echo "usage: scripts/prof.sh stats|pmc|stamps TAG [CONFIG ...]"; exit 2 ;;
esac
echo "rc=0"
