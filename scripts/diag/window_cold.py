"""Why bench.py's 20-step window (after the start-up calibration and W = 5 warm-up steps) measures ~2 % slower per
step than the same 20-step window taken in the middle of a long run (scripts/diag/launch_lead.py): 20-step windows
timed exactly as bench.py's timed_region, in the bench's order and then after a controlled GPU idle gap.
  first      : calibration -> prepare_graphs -> 5 warm-up steps -> window   (bench.py)
  again      : the next window right after                                   (warm)
  idle<ms>   : host sleep (GPU idle) -> 5 warm-up steps -> window
  idle<ms>w50: host sleep -> 50 warm-up steps -> window
Usage: python scripts/diag/window_cold.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

B = 8192
dev = torch.device("cuda", 0)
x, y = make_split(60000, seed=1)
n_idx = 120 * B
idx = torch.randint(0, 60000, (n_idx,), dtype=torch.int32)
torch.manual_seed(0)
tr = NativeTrainer("lenet5", "bf16", B, torch.from_numpy(x.reshape(-1, 784)).to(dev), torch.from_numpy(y).to(dev),
                   device=dev, lr=0.05, momentum=0.9, dropout=0.0, init=build_model("lenet5"), max_indices=n_idx)
tr.set_epoch_indices(idx)
tr.autotune_plan()
tr.prepare_graphs()


def window(label, warm):
    tr.set_epoch_indices(idx)
    tr.run_steps(warm)
    tr.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run_steps(20)
    tr.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{label:14s} {dt / 20 * 1e3:.4f} ms/step", flush=True)


window("first", 5)
window("again", 5)
window("again", 5)
for ms in (1, 5, 20, 100):
    for w in (5, 50):
        time.sleep(ms / 1000)
        window(f"idle{ms}ms w{w}", w)
