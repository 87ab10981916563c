#!/bin/bash
# Phase ablation of the LeNet conv kernels: per-kernel time with phases skipped (diagnostic only; WRONG
# results).  Needs the ablation build, made on the CPU host BEFORE the GPU call, and the normal build back
# afterwards:
#   MNIST_AMD_BUILD_DEFINES=-DMNIST_AMD_ABLATION_BUILD python -m pytorch_ddp_mnist_amd.ops.build
#   ... gpurun -- scripts/ablate.sh TAG ...
#   python -m pytorch_ddp_mnist_amd.ops.build
# (the normal build refuses MNIST_AMD_ABLATE / MNIST_AMD_HEAD_ABLATE)
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-abl}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for m in ${ABL_SET:-0 1 2 4 8 16 32 64 128 256 512 1016}; do
  MNIST_AMD_ABLATE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_$m" -o run --output-format csv -- python3 "$OUT/../bench.py" --steps 20 --warmup 3 --no-eval > "$OUT/${TAG}_$m.log" 2>&1 || { echo "fail $m"; exit 1; }
done
echo done
