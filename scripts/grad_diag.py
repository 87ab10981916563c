"""Per-layer gradient error of the native step vs torch fp32 (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
from test_native_gpu import make_trainer, rel_err, torch_grads  # noqa: E402
from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

model, dtype = sys.argv[1], sys.argv[2]
x, y = make_split(4096, seed=7)
for batch in [int(b) for b in sys.argv[3].split(",")]:
    torch.manual_seed(0)
    module = build_model(model)
    tr = make_trainer(model, dtype, max(128, batch), x, y, module)
    idx = torch.arange(batch, dtype=torch.int32) * 3 % len(y)
    tr.set_epoch_indices(idx)
    tr.reset_metrics()
    tr.forward_backward(batch)
    g = tr.grads()
    masks = None
    if model == "mlp" and os.environ.get("DIAG_MASKS"):
        masks = [(t[:128, :batch].float().cpu().T > 0).float() for t in (tr.h1T, tr.h2T)]
        print("mask zeros:", [int((mk == 0).sum()) for mk in masks])
    gref, _, _ = torch_grads(model, module, x[idx.numpy()], y[idx.numpy()], masks)
    off, parts = 0, []
    for k, v in module.state_dict().items():
        n = v.numel()
        d = (g[off:off + n] - gref[off:off + n]).view(v.shape)
        parts.append(f"{k}: {rel_err(g[off:off + n], gref[off:off + n]):.2e} maxabs {float(d.abs().max()):.2e}")
        if k == "0.weight":
            col = d.abs().sum(0)
            bad = torch.nonzero(col > col.median() * 20).view(-1).tolist()
            parts.append(f"   bad k cols: {bad[:20]} (n={len(bad)})")
            row = d.abs().sum(1)
            parts.append(f"   row err max/med: {float(row.max()):.2e}/{float(row.median()):.2e}")
        off += n
    print(f"B={batch} total {rel_err(g, gref):.2e}\n  " + "\n  ".join(parts), flush=True)

if os.environ.get("DIAG_DY1"):
    import torch.nn.functional as F
    batch = int(sys.argv[3].split(",")[0])
    torch.manual_seed(0)
    module = build_model(model)
    tr = make_trainer(model, dtype, max(128, batch), x, y, module)
    idx = torch.arange(batch, dtype=torch.int32) * 3 % len(y)
    tr.set_epoch_indices(idx)
    tr.forward_backward(batch)
    tr.synchronize()
    xb = (torch.from_numpy(x[idx.numpy()].reshape(-1, 784)).float() / 255 - 0.1307) / 0.3081
    yb = torch.from_numpy(y[idx.numpy()].astype("int64"))
    W0, b0, W3, b3, W5 = [v.float() for v in module.state_dict().values()]
    h1 = torch.relu(xb @ W0.T + b0)
    h2 = torch.relu(h1 @ W3.T + b3)
    z = h2 @ W5.T
    dz = torch.softmax(z, 1) - F.one_hot(yb, 10).float()
    dh2 = (dz @ W5) * (h2 > 0)
    dh1 = (dh2 @ W3) * (h1 > 0)
    got = tr.dy1T[:128, :batch].float().cpu().T
    gh1 = tr.h1T[:128, :batch].float().cpu().T
    err = (got - dh1).abs()
    print("h1 max err", float((gh1 - h1).abs().max()))
    print("dy1 max err", float(err.max()))
    bad = torch.nonzero(err > 1e-4)
    print("bad count", bad.shape[0])
    print("bad rows r:", sorted(set(bad[:, 0].tolist()))[:40])
    print("bad cols n:", sorted(set(bad[:, 1].tolist()))[:40])
    for r, n in bad[:8].tolist():
        print(r, n, float(got[r, n]), float(dh1[r, n]), float(h1[r, n]), float(gh1[r, n]))
