"""Where does the MLP weight-gradient tail update (head.hip wgrad_tail) differ from the separate reduce + SGD kernel?
One trainer per mode (MNIST_AMD_WGRAD_TAIL read at construction), identical init and batches; after each of a few
eager steps the gradient slab (grad = scale * sum of the partials, written by both paths) is compared per layer and
per 64 x 64 output tile.  Usage: python scripts/diag/tail_diag.py [--batch 4096] [--steps 3] [--model mlp|lenet5]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--model", default="mlp")
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--graph", action="store_true")
a = ap.parse_args()
var = "MNIST_AMD_WGRAD_TAIL" if a.model == "mlp" else "MNIST_AMD_CONV_TAIL"
N = a.batch * (a.steps + 1)
x, y = make_split(N, seed=7)
order = torch.randperm(N, generator=torch.Generator().manual_seed(1)).to(torch.int32)
grads, params = {}, {}
for mode in ("0", "1"):
    os.environ[var] = mode
    if a.model == "lenet5":
        os.environ["MNIST_AMD_CONCURRENT"] = "0"
    torch.manual_seed(0)
    tr = NativeTrainer(a.model, a.dtype, a.batch, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                       lr=0.05, momentum=0.9, dropout=0.0, init=build_model(a.model))
    tr.set_epoch_indices(order)
    grads[mode], params[mode] = [], []
    for s in range(a.steps):
        tr.step(a.batch, use_graph=a.graph)
        tr.synchronize()
        grads[mode].append(tr.grad.detach().cpu().clone())
        params[mode].append(tr.params.detach().cpu().clone())
        if s == 0 and mode == "1" and a.model == "mlp":
            slab1 = tr.slab_fc.detach().cpu().clone()
            nsplit = tr.rt.fc_splits
    tr.close()

if a.model == "mlp":
    # the tail mode's partials as they are in memory after step 0 (tile-major: split s, tile t, row nl, col kl at
    # s * ld + t * 4096 + nl * 64 + kl): their plain sum vs the separate kernel's gradient tells a wrong partial
    # (producer side) from a wrong read (the tail's loads)
    g0 = grads["0"][0]
    W1, B1 = 128 * 784, 128
    scale = 1.0 / a.batch
    print(f"slab rows {slab1.shape}, splits {nsplit}", flush=True)
    for (bn, bk) in [(0, 0), (1, 5), (0, 12)]:
        t = bn * 13 + bk
        part = slab1[:nsplit, t * 4096:(t + 1) * 4096].reshape(nsplit, 64, 64)
        tot = part.double().sum(0) * scale
        ref = torch.zeros(64, 64, dtype=torch.float64)
        for nl in range(64):
            n = bn * 64 + nl
            for kl in range(64):
                k = bk * 64 + kl
                if k < 784:
                    ref[nl, kl] = float(g0[n * 784 + k])
                elif k == 784:
                    ref[nl, kl] = float(g0[W1 + n])
        kmax = 784 - bk * 64 + 1 if bk == 12 else 64
        dd = (tot[:, :kmax] - ref[:, :kmax]).abs()
        got = grads["1"][0]
        gt = torch.zeros(64, kmax, dtype=torch.float64)
        for nl in range(64):
            n = bn * 64 + nl
            for kl in range(kmax):
                k = bk * 64 + kl
                gt[nl, kl] = float(got[n * 784 + k]) if k < 784 else float(got[W1 + n])
        dt = (gt - ref[:, :kmax]).abs()
        print(f"tile ({bn},{bk}): partial-sum vs sep max|d| {float(dd.max()):.3e}; tail grad vs sep max|d| "
              f"{float(dt.max()):.3e} (max|ref| {float(ref.abs().max()):.3e})", flush=True)
        bad = (dt > 1e-6 * float(ref.abs().max()) + 1e-12)
        print("   wrong per row (16-row groups) x 16-col quarter:", flush=True)
        for rg in range(4):
            print("     " + " ".join(f"{int(bad[rg * 16:(rg + 1) * 16, cq * 16:(cq + 1) * 16].sum()):4d}"
                                   for cq in range((kmax + 15) // 16)), flush=True)
        # the ratio tail / sep of a few wrong elements, and whether the tail equals a sum over a subset of splits
        idx = bad.nonzero()[:4]
        for nl, kl in idx.tolist():
            ps = part[:, nl, kl].double() * scale
            print(f"     ({nl},{kl}): sep {float(ref[nl, kl]):+.6e} tail {float(gt[nl, kl]):+.6e} partials*scale "
                  + " ".join(f"{float(v):+.3e}" for v in ps), flush=True)
    layers = [("W1", 0, 128, 784), ("b1", 128 * 784, 128, 1), ("W2", 128 * 785, 128, 128),
              ("b2", 128 * 785 + 128 * 128, 128, 1), ("W3", 128 * 785 + 128 * 129, 10, 128),
              ("b3", 128 * 785 + 128 * 129 + 1280, 10, 1)]
else:
    layers = [("conv", 0, 1, 2572), ("fc", 2572, 1, int(grads["0"][0].numel()) - 2572)]
for s in range(a.steps):
    g0, g1 = grads["0"][s], grads["1"][s]
    d = (g0 - g1).abs()
    print(f"step {s}: grad max|d| {float(d.max()):.3e} (max|g| {float(g0.abs().max()):.3e}), differing {int((d > 0).sum())}"
          f" of {d.numel()}; params differing {int((params['0'][s] != params['1'][s]).sum())}", flush=True)
    for name, off, n, k in layers:
        if off + n * k > d.numel():
            continue
        dd = d[off:off + n * k].view(n, k)
        gg = g0[off:off + n * k].view(n, k)
        print(f"   {name:5s} max|d| {float(dd.max()):.3e} rel {float(dd.max()) / max(float(gg.abs().max()), 1e-30):.3e}"
              f"  differing {int((dd > 0).sum())}/{dd.numel()}", flush=True)
        if k >= 64 and float(dd.max()) > 0:  # per 64 x 64 tile: share of differing elements
            rows = []
            for bn in range((n + 63) // 64):
                rows.append(" ".join(f"{int((dd[bn * 64:(bn + 1) * 64, bk * 64:(bk + 1) * 64] > 0).sum()):4d}"
                                     for bk in range((k + 63) // 64)))
            print("      differing per tile (rows = 64-row blocks):\n      " + "\n      ".join(rows), flush=True)
