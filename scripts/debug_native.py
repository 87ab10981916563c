"""Stage-by-stage comparison of the native head/conv kernels against torch (diagnostics)."""
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model, flatten_grads  # noqa: E402


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def main(model="mlp", dtype="fp32", B=128):
    torch.manual_seed(0)
    x, y = make_split(1024, 7)
    m = build_model(model)
    tr = NativeTrainer(model, dtype, 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y), dropout=0.0, init=m)
    idx = torch.arange(B, dtype=torch.int32)
    tr.set_epoch_indices(idx)
    tr.reset_metrics()
    tr.forward_backward(B)
    tr.synchronize()
    xb = (torch.from_numpy(x[:B]).float() / 255 - 0.1307) / 0.3081
    yb = torch.from_numpy(y[:B].astype(np.int64))
    L = [mod for mod in m if isinstance(mod, torch.nn.Linear)]
    if model == "mlp":
        X = xb.view(B, -1)
        print("xT", rel(tr.xT[:784, :B].t(), X))
    else:
        feats = m[:7](xb.view(B, 1, 28, 28))
        X = feats
        print("p2", rel(tr.p2[:B, :400], X))
        print("xT", rel(tr.xT[:400, :B].t(), X))
    X = X.detach().requires_grad_(True)
    h1 = torch.relu(L[0](X)); h1.retain_grad()
    h2 = torch.relu(L[1](h1)); h2.retain_grad()
    z = L[2](h2); z.retain_grad()
    loss = F.cross_entropy(z, yb)
    loss.backward()
    n1, n2 = L[0].out_features, L[1].out_features
    print("h1T", rel(tr.h1T[:n1, :B].t(), h1))
    print("h2T", rel(tr.h2T[:n2, :B].t(), h2))
    print("dy3T", rel(tr.dy3T[:10, :B].t() / B, z.grad))
    print("dy2T", rel(tr.dy2T[:n2, :B].t() / B, h2.grad * (h2 > 0)))
    print("dy1T", rel(tr.dy1T[:n1, :B].t() / B, h1.grad * (h1 > 0)))
    st = tr.read_metrics()
    print("loss", st.loss_sum / B, float(loss))
    if model == "lenet5":
        print("dp2", rel(tr.dp2[:B, :400] / B, X.grad))
    mm = build_model(model)
    mm.load_state_dict(m.state_dict())
    inp = xb.view(B, -1) if model == "mlp" else xb.view(B, 1, 28, 28)
    out = mm(inp)
    (F.nll_loss(out, yb) if model == "lenet5" else F.cross_entropy(out, yb)).backward()
    gref = flatten_grads(mm)
    g = tr.grads()
    off = 0
    for k, v in mm.state_dict().items():
        n = v.numel()
        print(f"grad {k:10s} rel {rel(g[off:off+n], gref[off:off+n]):.3e}  |g| {g[off:off+n].norm():.4e} |ref| {gref[off:off+n].norm():.4e}")
        off += n
    s = tr.slab_fc.cpu()
    print("slab rows", s.shape, "row norms", s.norm(dim=1)[:8])


if __name__ == "__main__":
    main(*(sys.argv[1:3]), *(int(a) for a in sys.argv[3:4]))
