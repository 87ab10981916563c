#!/bin/bash
# Build a git ref into ab/<name>/ (source + its own in-tree .so) for same-box A/B benches:
#   scripts/ab_prepare.sh HEAD base   ->   on the box: (cd ab/base && python bench.py ...)
set -e
REF=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$ROOT/ab/$NAME" && mkdir -p "$ROOT/ab/$NAME"
git -C "$ROOT" archive "$REF" | tar -x -C "$ROOT/ab/$NAME"
(cd "$ROOT/ab/$NAME" && python -m pytorch_ddp_mnist_amd.ops.build > /dev/null)
echo "ab/$NAME <- $(git -C "$ROOT" rev-parse --short "$REF")"
