"""Train a few LeNet-5 steps through the native step graph and print a digest of the parameters.

Used by tests/test_schedules_gpu.py to check that every step schedule (serial / concurrent FC
wgrad, single-GPU fused update / world-1 RCCL join / split buckets) gives bitwise-identical
parameters: the schedules are selected by environment variables read once per process
(MNIST_AMD_CONCURRENT, MNIST_AMD_MG_SCHED), so each variant runs in its own interpreter.
Usage: python scripts/sched_equiv.py [--comm] [--batch B] [--steps K]
"""
import argparse
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402
from pytorch_ddp_mnist_amd.ops.native import load_c  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--comm", action="store_true", help="attach a world-1 RCCL communicator")
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--steps", type=int, default=4)
a = ap.parse_args()
x, y = make_split(4096, seed=7)
torch.manual_seed(0)
tr = NativeTrainer("lenet5", "bf16", a.batch, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                   lr=0.05, momentum=0.9, dropout=0.0, init=build_model("lenet5"))
if a.comm:
    C = load_c()
    tr.attach_comm(C.RcclComm(C.RcclComm.make_unique_id(), 0, 1, 0), 1)
    tr.broadcast_params(0)
tr.set_epoch_indices(torch.randperm(4096, generator=torch.Generator().manual_seed(1)).to(torch.int32))
for _ in range(a.steps):
    tr.step(a.batch, use_graph=True)
tr.synchronize()
print("digest", hashlib.sha256(tr.params.cpu().numpy().tobytes()).hexdigest())
