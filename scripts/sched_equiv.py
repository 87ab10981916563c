"""Train a few LeNet-5 steps through the native step graph per variant and print parameter digests.

Used by tests/test_schedules_gpu.py to check that every step schedule gives bitwise-identical
parameters: serial / concurrent FC wgrad (MNIST_AMD_CONCURRENT, read once per process), and with a
world-1 RCCL communicator the JOIN and
SPLIT multi-GPU plans, with the default or a capped conv_bwd grid.  ``w2`` variants emulate the
1/W arithmetic of a 2-rank job on one GPU (world set to 2 on a world-1 communicator, so every
rank's "all-reduced" gradient is its own): they must equal a local run at half the learning rate
(x0.5 is exact in binary floating point).
``_k<k>`` variants run the steps as ONE k-step graph (run_steps), whose steps may leave the aux
branch join to the next step's head; they must equal the same number of single-step graphs.
Usage: python scripts/sched_equiv.py [--model mlp|lenet5] [--dtype bf16|fp32] [--batch B] VARIANT [VARIANT ...]
  VARIANT = {local,local_halflr,join,split,overlap}[_g<groups>][_b<blocks>][_w2][_k<k>][_t<rows>]   (overlap: LeNet,
  world-1 one-shot; _t<rows>: one more step of a partial batch of <rows> rows after the full ones, eager launch;
  _g<groups>: the bucket groups of the FC units in ready order, "." between groups, e.g. split_g0.1.2)
"""
import argparse
import gc
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
from pytorch_ddp_mnist_amd.parallel.ddp import groups_to_buckets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--model", default="lenet5", choices=["lenet5", "mlp"])
ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
ap.add_argument("--dump", default=None, help="also save each variant's parameters to DUMP.<variant>.pt")
a = ap.parse_args()
N = max(4096, a.batch * (a.steps + 1))  # (4096 for the default shapes: their digests are unchanged)
x, y = make_split(N, seed=7)
C = load_c()
order = torch.randperm(N, generator=torch.Generator().manual_seed(1)).to(torch.int32)

for v in a.variants:
    m = re.fullmatch(r"(local_halflr|local|join|split|overlap)(?:_g([0-9.]+))?(?:_b(\d+))?(_w2)?(?:_k(\d+))?(?:_t(\d+))?", v)
    if not m:
        raise SystemExit(f"unknown variant {v}")
    kind, gspec = m.group(1), m.group(2)
    blocks, w2, k = int(m.group(3) or 0), bool(m.group(4)), int(m.group(5) or 0)
    tail_rows = int(m.group(6) or 0)
    lr = 0.025 if kind == "local_halflr" else 0.05
    torch.manual_seed(0)
    tr = NativeTrainer(a.model, a.dtype, a.batch, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                       lr=lr, momentum=0.9, dropout=0.0, init=build_model(a.model))
    if kind in ("join", "split"):
        tr.attach_comm(C.RcclComm(C.RcclComm.make_unique_id(), 0, 1, 0), 2 if w2 else 1, plan=kind,
                       bwd_blocks=blocks)
        if gspec:  # bucket groups of the FC units in ready order, e.g. "0.1.2" = three groups, "01.2" = two
            tr.set_buckets(groups_to_buckets(a.model, [[int(c) for c in part] for part in gspec.split(".")]))
        tr.broadcast_params(0)
    elif kind == "overlap":  # world-1 one-shot instances (identity sums), the 1/W of a 2-rank job with _w2
        fc, conv = C.OneShotAllReduce(0, 1, 0, tr.nparam), C.OneShotAllReduce(0, 1, 0, int(tr.rt.conv_params))
        tr.attach_overlap(fc, conv, 2 if w2 else 1)
        tr.set_plan("overlap", blocks)
    elif blocks:
        tr.rt.set_bwd_blocks(blocks)
    tr.set_epoch_indices(order)
    if k:
        tr.run_steps(a.steps, use_graph=True, k=k)
    else:
        for _ in range(a.steps):
            tr.step(a.batch, use_graph=True)
    if tail_rows:
        tr.step(tail_rows, use_graph=False)
    tr.synchronize()
    print("digest", v, hashlib.sha256(tr.params.cpu().numpy().tobytes()).hexdigest(), flush=True)
    if a.dump:
        torch.save(tr.params.cpu(), f"{a.dump}.{v}.pt")
    # deterministic teardown before the next variant, in DistContext.finalize's order (graphs -> trainer streams ->
    # communicator): left to the garbage collector, a previous variant's communicator could be destroyed in the
    # middle of the next variant's graph replays (a HIP-runtime segfault in hipGraphLaunch was seen that way)
    comm = tr.comm
    tr.close()
    if comm is not None:
        comm.destroy(60.0)
    del tr, comm
    gc.collect()
