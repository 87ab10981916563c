#!/bin/bash
# Build the native _C extension of another git revision as pytorch_ddp_mnist_amd/_C_ab.so (CPU host, before a
# GPU call), for same-box A/B runs against the working tree's build:
#   scripts/build_ab.sh REV [NAME]      (NAME: module name, default _C_ab)
#   gpurun -- 'bash scripts/ab.sh TAG "--steps 2000 --warmup 50" "MNIST_AMD_C_PATH=pytorch_ddp_mnist_amd/_C_ab.so" "-"'
set -e
REV=${1:?revision}
NAME=${2:-_C_ab}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" csrc | tar -x -C "$TMP"
SUF=$(python3 -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
python3 -m pytorch_ddp_mnist_amd.ops.build --only _C --csrc "$TMP/csrc" --out "$ROOT/pytorch_ddp_mnist_amd/$NAME$SUF"
rm -rf "$TMP"
echo "built $REV -> pytorch_ddp_mnist_amd/$NAME$SUF"
