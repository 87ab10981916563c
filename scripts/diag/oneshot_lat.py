"""World-1 latency of the one-shot all-reduce kernel (graph-replayed, median) by block count and size."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.ops.native import load_c  # noqa: E402
from pytorch_ddp_mnist_amd.parallel.oneshot import time_oneshot  # noqa: E402

C = load_c()
dev = torch.device("cuda", 0)
for nblk in (4, 16, 64):
    o = C.OneShotAllReduce(0, 1, 0, 61706, nblk)
    for n in (2572, 59134):
        ms = time_oneshot(o, n, dev, iters=200, warmup=20)
        print(f"nblk {nblk:3d}  count {n:6d}  {ms * 1000:7.2f} us", flush=True)
