"""Calibration vs steady state: time the single-GPU LeNet schedules three ways on one box --
interleaved k-step replays (time_schedules multi), interleaved single-step replays, and each schedule
alone in run_steps (the bench's timed path).   STAMP-free; python scripts/calib_probe.py [B] [dtype]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402
from pytorch_ddp_mnist_amd.parallel.ddp import local_plan_candidates  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16"
x, y = make_split(60000, seed=1)
dev = torch.device("cuda", 0)
tr = NativeTrainer("lenet5", dtype, B, torch.from_numpy(x.reshape(-1, 784)).to(dev), torch.from_numpy(y).to(dev),
                   device=dev, lr=0.05, momentum=0.9, dropout=0.0, init=build_model("lenet5"))
tr.set_epoch_indices(torch.randperm(60000, dtype=torch.int32)[: (60000 // B) * B])
cands = local_plan_candidates(fwd_head=tr.fwd_head_applies())
tr.run_steps(4)
tr.synchronize()
for rep in range(2):
    print("multi ", {k: round(v * 1000, 2) for k, v in tr.time_schedules(cands, multi=True).items()}, flush=True)
    print("single", {k: round(v * 1000, 2) for k, v in tr.time_schedules(cands, multi=False).items()}, flush=True)
    for name, c in cands.items():
        tr.apply_plan(c)
        tr.set_epoch_indices(torch.randperm(60000, dtype=torch.int32)[: (60000 // B) * B])
        n = max(8, min(400, 60000 // B - 8) // 8 * 8)
        tr.run_steps(min(8, 60000 // B - n))
        tr.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(tr.stream)
        tr.run_steps(n)
        b.record(tr.stream)
        tr.synchronize()
        print(f"alone {name}: {a.elapsed_time(b) / n * 1000:.2f} us/step ({n} steps)", flush=True)
