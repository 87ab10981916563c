"""Single-node multi-GPU DDP training (reference: ddp_tutorial_multi_gpu.py; train_multi_gpu.sh).

One process per GPU, launched by ``torch.distributed.run``/``launch``.  Accepts ``--local_rank``,
the dashed ``--local-rank`` newer launchers pass (survey Q5) and ``LOCAL_RANK``; rank/world come
from the launcher environment.  batch_size=128 per rank, epochs=10, DistributedSampler(seed=42)
order, rank-0 ``model.pt`` — as upstream.  The step runs on the native MI355X trainer: hand-written
CDNA4 kernels, gradients all-reduced by the native RCCL communicator over xGMI.  Without a GPU it
falls back to the torch-CPU engine over gloo (so the script stays runnable for plumbing tests).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from pytorch_ddp_mnist_amd.config import configure_gpu_tutorial  # noqa: E402
from pytorch_ddp_mnist_amd.engine.runner import run  # noqa: E402

if __name__ == "__main__":
    cfg = configure_gpu_tutorial()
    cfg.data_format = "idx" if cfg.data_format == "auto" else cfg.data_format
    if cfg.local_rank is not None:
        os.environ.setdefault("LOCAL_RANK", str(cfg.local_rank))
    if torch.cuda.device_count() == 0 and cfg.device in ("cuda", "auto"):
        print("[ddp_tutorial_multi_gpu] no GPU visible: running the torch-CPU engine over gloo", file=sys.stderr)
        cfg.device = "cpu"
    cfg.parallel = int(os.environ.get("WORLD_SIZE", "1")) > 1
    run(cfg, entry="ddp_tutorial_multi_gpu")
