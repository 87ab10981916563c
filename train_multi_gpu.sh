#!/bin/bash
# One process per GPU on one node (reference train_multi_gpu.sh used the deprecated
# torch.distributed.launch; torch.distributed.run passes --local-rank / LOCAL_RANK, both accepted).
NPROC=${NPROC:-8}
python -m torch.distributed.run --nnodes=1 --nproc-per-node="$NPROC" --master-addr 127.0.0.1 \
    --master-port "${MASTER_PORT:-29500}" ddp_tutorial_multi_gpu.py "$@"
