"""Why did the start-up calibration time the small-batch serial LeNet schedule slower than training runs it?

`time_schedules` timed LeNet bf16 B=128 serial at 38.5 us/step while `run_steps` ran the same schedule at
32.8 (profiles/r3_session3/NOTES.md).  This runs ONE of the two loops per process, so a kernel trace
(`rocprofv3 --kernel-trace --stats -- python scripts/calib_diag.py MODE`) shows, per kernel, what each
loop actually executes and how long it takes:

  calib  : time_schedules({"serial"}) -- the calibration's sample plan, serial candidate only
  calib2 : time_schedules({"serial", "concurrent"}) -- as autotune_plan runs it
  run    : apply_plan(serial) + run_steps, the training loop

Prints the per-step time the loop itself measured (events), plus the kernel count per step.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("mode", choices=["calib", "calib2", "run"])
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--steps", type=int, default=400)
ap.add_argument("--repeat", type=int, default=4, help="calibration calls (calib modes)")
a = ap.parse_args()

images, labels, idx, _, _ = bench.bench_data(1, 0, a.batch, a.steps + 64)
torch.manual_seed(0)
tr = NativeTrainer("lenet5", a.dtype, a.batch, images.cuda(), labels.cuda(), lr=0.05, momentum=0.9, dropout=0.0,
                   init=build_model("lenet5"), max_indices=idx.numel())
tr.set_epoch_indices(idx)
serial = {"concurrent": False}
if a.mode == "run":
    tr.apply_plan(serial)
    tr.run_steps(40, use_graph=True)  # warm-up: captures, clocks
    tr.synchronize()
    tr.set_epoch_indices(idx)
    st = tr.stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    tr.run_steps(a.steps, use_graph=True)
    e1.record(st)
    tr.synchronize()
    print(f"run serial: {e0.elapsed_time(e1) / a.steps * 1000:.2f} us/step over {a.steps} steps", flush=True)
else:
    cands = {"serial": serial} if a.mode == "calib" else {"serial": serial, "concurrent": {"concurrent": True}}
    for r in range(a.repeat):
        t0 = time.perf_counter()
        t = tr.time_schedules(cands)
        print(f"calib[{r}] " + " ".join(f"{k}={v * 1000:.2f}us" for k, v in t.items()) +
              f"  ({tr.last_timing}, {time.perf_counter() - t0:.2f} s)", flush=True)
