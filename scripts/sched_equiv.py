"""Train a few LeNet-5 steps through the native step graph per variant and print parameter digests.

Used by tests/test_schedules_gpu.py to check that every step schedule gives bitwise-identical
parameters: serial / concurrent FC wgrad (MNIST_AMD_CONCURRENT, read once per process), conv_bwd
as two concurrent halves (MNIST_AMD_SPLIT_BWD), and with a world-1 RCCL communicator the JOIN and
SPLIT multi-GPU plans, with the default or a capped conv_bwd grid.  ``w2`` variants emulate the
1/W arithmetic of a 2-rank job on one GPU (world set to 2 on a world-1 communicator, so every
rank's "all-reduced" gradient is its own): they must equal a local run at half the learning rate
(x0.5 is exact in binary floating point).
Usage: python scripts/sched_equiv.py VARIANT [VARIANT ...]
  VARIANT = local | local_halflr | {join,split}[_b<blocks>][_w2]
"""
import argparse
import hashlib
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402
from pytorch_ddp_mnist_amd.ops.native import load_c  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--steps", type=int, default=4)
a = ap.parse_args()
x, y = make_split(4096, seed=7)
C = load_c()
order = torch.randperm(4096, generator=torch.Generator().manual_seed(1)).to(torch.int32)

for v in a.variants:
    lr = 0.025 if v == "local_halflr" else 0.05
    torch.manual_seed(0)
    tr = NativeTrainer("lenet5", "bf16", a.batch, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                       lr=lr, momentum=0.9, dropout=0.0, init=build_model("lenet5"))
    m = re.fullmatch(r"(join|split)(?:_b(\d+))?(_w2)?", v)
    if m:
        tr.attach_comm(C.RcclComm(C.RcclComm.make_unique_id(), 0, 1, 0), 2 if m.group(3) else 1,
                       plan=m.group(1), bwd_blocks=int(m.group(2) or 0))
        tr.broadcast_params(0)
    elif v.startswith("local_b"):
        tr.rt.set_bwd_blocks(int(v[7:]))
    elif v not in ("local", "local_halflr"):
        raise SystemExit(f"unknown variant {v}")
    tr.set_epoch_indices(order)
    for _ in range(a.steps):
        tr.step(a.batch, use_graph=True)
    tr.synchronize()
    print("digest", v, hashlib.sha256(tr.params.cpu().numpy().tobytes()).hexdigest(), flush=True)
