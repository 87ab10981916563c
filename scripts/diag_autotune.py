"""Step-by-step probe of graph re-capture with RCCL nodes (prints after each step)."""
import os
import sys
import faulthandler
faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402
from pytorch_ddp_mnist_amd.ops.native import load_c  # noqa: E402


def p(*a):
    print(*a, flush=True)


mode = sys.argv[1]
C = load_c()
x, y = make_split(4096, seed=7)
tr = NativeTrainer("lenet5", "bf16", 512, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                   lr=0.05, momentum=0.9, dropout=0.0, init=build_model("lenet5"))
tr.set_epoch_indices(torch.arange(4096, dtype=torch.int32))
if mode != "nocomm":
    tr.attach_comm(C.RcclComm(C.RcclComm.make_unique_id(), 0, 1, 0), 1)
    tr.broadcast_params(0)
p("attached")
seq = {"recap_join": [0, 0], "split": [1], "join_split": [0, 1], "nocomm": [0, 1, 0], "autotune": []}[mode]
for k in seq:
    tr.rt.set_plan(k)
    p("set_plan", k)
    tr.capture()
    p("captured", k)
    for _ in range(3):
        with torch.cuda.stream(tr.stream):
            tr.step_ctr[0].zero_()
        tr.rt.replay(tr.stream.cuda_stream)
    tr.synchronize()
    p("replayed", k)
if mode == "autotune":
    tr.step(512)
    p("stepped")
    print(tr.autotune_plan(iters=4, warmup=1, log=p), flush=True)
    tr.step(512)
    tr.synchronize()
p("done", mode)
