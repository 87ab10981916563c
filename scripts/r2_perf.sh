#!/bin/bash
# Perf iteration: numerics tests, driver-shaped + long bench, kernel stats, LDS/MFMA counter pass.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-perf}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
PT="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
timeout -k 10 600 $PT tests/test_native_gpu.py tests/test_schedules_gpu.py tests/test_multigpu_gpu.py -k "not watchdog" > "$OUT/${TAG}_pytest.log" 2>&1 &&
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/${TAG}_bench.log" 2>&1 &&
timeout -k 10 120 python bench.py --steps 20 --warmup 5 >> "$OUT/${TAG}_bench.log" 2>&1 &&
timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-eval >> "$OUT/${TAG}_bench.log" 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- python3 "$OUT/../bench.py" --steps 20 --warmup 5 --no-eval > "$OUT/${TAG}_prof.log" 2>&1) &&
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$OUT/${TAG}_pmcb" -o run -- python3 "$OUT/../bench.py" --steps 3 --warmup 1 --no-eval > "$OUT/${TAG}_pmcb.log" 2>&1)
rc=$?
echo "rc=$rc"
exit $rc
