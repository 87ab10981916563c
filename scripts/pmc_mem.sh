#!/bin/bash
# Memory-hierarchy counters per kernel (own runs: --pmc + --kernel-trace only).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-pm}
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/${TAG}_$N" -o run -- python3 "$OUT/../bench.py" --steps 3 --warmup 1 --no-eval > "$OUT/${TAG}_$N.log" 2>&1
}
N=a run TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum &&
N=b run TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum &&
N=c run TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCC_EA0_RDREQ_DRAM_sum
echo "rc=$?"
