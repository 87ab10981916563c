#!/bin/bash
# Step-schedule check on one GPU: GPU tests of the runtime, then the headline bench with the serial /
# concurrent schedules, with and without a world-1 RCCL communicator (multi-GPU schedule on one GPU).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-sched}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1 || { tail -30 "$OUT/${TAG}_pytest.log"; exit 1; }
tail -2 "$OUT/${TAG}_pytest.log"
for kv in "MNIST_AMD_CONCURRENT=0" "MNIST_AMD_CONCURRENT=1"; do
  for extra in "" "--comm-world1" ; do
    env $kv timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-eval $extra > "$OUT/${TAG}_b.log" 2>&1 || { cat "$OUT/${TAG}_b.log"; exit 1; }
    echo "$kv $extra $(python scripts/summarize.py bench $OUT/${TAG}_b.log)"
  done
done
MNIST_AMD_MG_SCHED=split timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-eval --comm-world1 > "$OUT/${TAG}_b.log" 2>&1 || { cat "$OUT/${TAG}_b.log"; exit 1; }
echo "split --comm-world1 $(python scripts/summarize.py bench $OUT/${TAG}_b.log)"
