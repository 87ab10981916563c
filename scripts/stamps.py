"""Per-phase wall-clock stamps of the fused head kernel (MNIST_AMD_STAMPS=1).

Runs the headline config (LeNet-5 bf16, B=8192) for a few steps, then prints, over the head
workgroups of the last step, the mean/min/max duration of each phase (stamp k -> k+1) and the
spread of workgroup start/end times.  The wall clock ticks at 100 MHz (10 ns).
"""
import os
import sys

os.environ["MNIST_AMD_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

B = int(os.environ.get("STAMP_BATCH", "8192"))
model = os.environ.get("STAMP_MODEL", "lenet5")
x, y = make_split(60000, seed=1)
dev = torch.device("cuda", 0)
tr = NativeTrainer(model, "bf16", B, torch.from_numpy(x.reshape(-1, 784)).to(dev), torch.from_numpy(y).to(dev),
                   device=dev, lr=0.05, momentum=0.9, dropout=0.0, init=build_model(model))
tr.set_epoch_indices(torch.randperm(60000, dtype=torch.int32)[: (60000 // B) * B])
tr.reset_metrics()
for _ in range(6):
    tr.step(B, use_graph=True)
tr.synchronize()
nblk = (B + 63) // 64
st = tr.stamps.view(-1, 16)[:nblk].cpu().numpy().astype(np.int64)
names = ["idx+stage X", "L1", "L2", "L3", "softmax", "dH2", "dH1", "dX"]
t0 = st[:, 0].min()
print(f"head workgroups: {nblk}; start spread {(st[:, 0].max() - t0) * 10 / 1000:.2f} us; "
      f"kernel span {(st[:, 8].max() - t0) * 10 / 1000:.2f} us")
for k, n in enumerate(names):
    d = (st[:, k + 1] - st[:, k]) * 10 / 1000.0
    print(f"  {n:12s} mean {d.mean():7.2f} us  min {d.min():7.2f}  max {d.max():7.2f}")
tot = (st[:, 8] - st[:, 0]) * 10 / 1000.0
print(f"  {'total':12s} mean {tot.mean():7.2f} us  min {tot.min():7.2f}  max {tot.max():7.2f}")
