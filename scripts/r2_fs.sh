#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
T=${1:-fs}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_runtime.py -k "forward_split or multi_step or captured" > $OUT/${T}_pytest.log 2>&1 || { grep -v "^  File" $OUT/${T}_pytest.log | tail -30; exit 1; }
tail -1 $OUT/${T}_pytest.log
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/${T}_drv$i.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'], d['config']['plan'], d['config'].get('plan_autotune',{}).get('timings_ms'))" $OUT/${T}_drv$i.json
done
timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --no-eval > $OUT/${T}_long.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('long', d['ms_per_step'], d['value'], d['config']['plan'])" $OUT/${T}_long.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${T}_prof" -o run --output-format csv -- python3 "$OUT/../bench.py" --steps 50 --warmup 10 --no-eval > "$OUT/${T}_prof.log" 2>&1) || exit 1
python scripts/summarize.py stats "$OUT/${T}_prof/run_kernel_stats.csv" 7
