"""Train YOUR OWN torch model with this framework's DDP + device loaders.

The reference's fixed models run on the native engine (``ddp_tutorial_*.py``); any other
``nn.Module`` uses the same building blocks the way a torch DDP script would:

    python examples/byo_model_ddp.py                                   # 1 process (GPU if present)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/byo_model_ddp.py   # 8 GPUs, RCCL
    python -m pytorch_ddp_mnist_amd.parallel.launch -n 2 --style torch -- \
        python examples/byo_model_ddp.py --device cpu                  # 2 CPU ranks, gloo

GPU: bucket all-reduces go over the native RCCL communicator on a side stream, batches come from
the native gather kernel over the HBM-resident dataset.  CPU: c10d gloo + torch indexing.
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_ddp_mnist_amd.data.loaders import create_data_loaders  # noqa: E402
from pytorch_ddp_mnist_amd.parallel import DistributedDataParallel  # noqa: E402
from pytorch_ddp_mnist_amd.parallel.comm import init_distributed  # noqa: E402


class MyNet(torch.nn.Module):
    """An arbitrary user model (not one of the native engine's two)."""

    def __init__(self):
        super().__init__()
        self.conv = torch.nn.Conv2d(1, 8, 3, padding=1)
        self.fc1 = torch.nn.Linear(8 * 14 * 14, 64)
        self.fc2 = torch.nn.Linear(64, 10)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv(x)), 2)
        return self.fc2(F.relu(self.fc1(x.flatten(1))))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--limit", type=int, default=6000, help="training samples (synthetic data)")
    ap.add_argument("--lr", type=float, default=0.05)
    a = ap.parse_args(argv)
    parallel = int(os.environ.get("WORLD_SIZE", "1")) > 1
    ctx = init_distributed(None, parallel=parallel, device=a.device)
    dev = ctx.device
    train, test = create_data_loaders(a.batch_size, ctx.world, ctx.rank, dev, fmt="synthetic", limit=a.limit,
                                      layout="image")
    torch.manual_seed(0)
    model = MyNet().to(dev)
    ddp = DistributedDataParallel(model, rccl=ctx.rccl) if ctx.world > 1 else model
    opt = torch.optim.SGD(ddp.parameters(), lr=a.lr, momentum=0.9)
    for epoch in range(a.epochs):
        train.sampler.set_epoch(epoch)
        ddp.train()
        for x, y in train:
            opt.zero_grad()
            F.cross_entropy(ddp(x), y).backward()
            opt.step()
        ddp.eval()
        correct = total = 0
        with torch.no_grad():
            for x, y in test:
                correct += int((model(x).argmax(1) == y).sum())
                total += y.numel()
        if ctx.rank == 0:
            print(f"Epoch={epoch}, top1={correct / total:.4f}", flush=True)
    ctx.finalize()
    return correct / total


if __name__ == "__main__":
    main()
