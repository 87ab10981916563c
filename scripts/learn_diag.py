"""Diagnostic: per-epoch accuracy of the fused single-GPU step vs the phased step (same init/data)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_ddp_mnist_amd.data.synthetic import make_split
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
from pytorch_ddp_mnist_amd.models import build_model

model, dtype = sys.argv[1], sys.argv[2]
lr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.05
mom = float(sys.argv[4]) if len(sys.argv) > 4 else 0.9
modes = sys.argv[5].split(",") if len(sys.argv) > 5 else ["fused", "phased", "graph"]
x, y = make_split(4096, seed=7)
xt, yt = make_split(1024, seed=8)
torch.manual_seed(3)
m = build_model(model)
for mode in modes:
    tr = NativeTrainer(model, dtype, 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y), dropout=0.0,
                       init=m, lr=lr, momentum=mom)
    g = torch.Generator().manual_seed(0)
    for ep in range(3):
        idx = torch.randperm(len(y), generator=g).to(torch.int32)
        if mode == "graph":
            st = tr.train_epoch(idx)
        else:
            tr.set_epoch_indices(idx)
            tr.reset_metrics()
            for s in range(len(y) // 128):
                if mode == "fused":
                    tr.step(128, use_graph=False)
                else:
                    tr.forward_backward(128)
                    tr.optimizer_step(1.0)
            st = tr.read_metrics()
        ev = tr.evaluate(torch.from_numpy(xt.reshape(-1, 784)), torch.from_numpy(yt),
                         torch.arange(len(yt), dtype=torch.int32))
        print(mode, lr, mom, ep, f"train loss {st.mean_loss:.4f} acc {st.accuracy:.4f}  eval acc {ev.accuracy:.4f}", flush=True)
