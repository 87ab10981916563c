"""Per-step GPU times of the bench step (events between graph replays) + host enqueue cost.

Answers: is a short timed region (driver: 20 steps after 5 warmup) slower per step than a long one,
and is it the GPU (clock ramp, first replays) or the host (graph-launch cost)?
Usage: python scripts/step_times.py [--warmup 5] [--steps 60] [--idle-ms 0]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.sampler import epoch_indices  # noqa: E402
from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--steps", type=int, default=60)
ap.add_argument("--batch", type=int, default=8192)
ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep between warmup and the timed steps")
a = ap.parse_args()
x, y = make_split(60000, seed=1)
reps = 2
images = torch.from_numpy(x.reshape(-1, 784)).cuda().repeat(reps, 1)
labels = torch.from_numpy(y).cuda().repeat(reps)
n = 60000 * reps
spe = n // a.batch
ne = -(-(a.warmup + a.steps) // spe)
idx = torch.cat([epoch_indices(n, 1, 0, e)[: spe * a.batch] for e in range(ne)]).to(torch.int32)
torch.manual_seed(0)
tr = NativeTrainer("lenet5", "bf16", a.batch, images, labels, lr=0.05, momentum=0.9, dropout=0.0,
                   init=build_model("lenet5"), max_indices=idx.numel())
tr.set_epoch_indices(idx)
for _ in range(a.warmup):
    tr.step(a.batch)
tr.synchronize()
if a.idle_ms:
    time.sleep(a.idle_ms / 1e3)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
t0 = time.perf_counter()
ev[0].record(tr.stream)
for i in range(a.steps):
    tr.step(a.batch)
    ev[i + 1].record(tr.stream)
t_enq = time.perf_counter() - t0
tr.synchronize()
t_all = time.perf_counter() - t0
d = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)]
print(f"warmup={a.warmup} steps={a.steps} host_enqueue={t_enq * 1e3:.3f} ms wall={t_all * 1e3:.3f} ms "
      f"gpu_sum={sum(d):.3f} ms")
print("per-step ms:", " ".join(f"{v:.4f}" for v in d))
for k in (20, a.steps):
    print(f"first {k}: mean {sum(d[:k]) / k:.4f} ms")
