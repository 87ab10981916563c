"""Where the 20-step driver window loses ~50 us against long runs (LeNet-5 bf16 B=8192): the time of a K-step window
started from an idle, synchronised device, for several ways of cutting the K steps into graph launches, against
the per-step time of a long run.  Every variant runs the same kernels in the same order; the windows are
interleaved (15 rounds) and the median is reported.
  A  2 x 10-step graph                        (run_steps default)
  B  1-step graph, 10-step graph, 9-step graph (a short first launch: the GPU starts while the long one submits)
  C  4 x 5-step graph
  D  1-step graph, 19-step graph
plus the host time spent inside the first launch call, and the per-step time of 200-step windows.
Usage: python scripts/diag/launch_lead.py [batch]"""
import os
import statistics as st
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
LONG = 200
dev = torch.device("cuda", 0)
x, y = make_split(60000, seed=1)
n_idx = (LONG + 20) * B
idx = torch.randint(0, 60000, (n_idx,), dtype=torch.int32)
torch.manual_seed(0)
tr = NativeTrainer("lenet5", "bf16", B, torch.from_numpy(x.reshape(-1, 784)).to(dev), torch.from_numpy(y).to(dev),
                   device=dev, lr=0.05, momentum=0.9, dropout=0.0, init=build_model("lenet5"), max_indices=n_idx)
tr.set_epoch_indices(idx)
print("calibration:", tr.autotune_plan()["chosen"], flush=True)
tr.prepare_graphs(10, extra=(9, 5, 19))
tr.set_epoch_indices(idx)
tr.run_steps(100)
tr.synchronize()


def rep(n):
    tr.rt.replay_n(tr.stream.cuda_stream, n) if n != 10 else tr.rt.replay_multi(tr.stream.cuda_stream)
    tr.host_step += n


def one(n):
    tr.step(B, use_graph=True)


VARIANTS = {
    "A 10+10": [rep, 10, rep, 10],
    "B 1+10+9": [one, 1, rep, 10, rep, 9],
    "C 5+5+5+5": [rep, 5, rep, 5, rep, 5, rep, 5],
    "D 1+19": [one, 1, rep, 19],
}
res = {k: [] for k in VARIANTS}
first_call = {k: [] for k in VARIANTS}
longs = []
for r in range(15):
    for k, seq in VARIANTS.items():
        tr.set_epoch_indices(idx)
        tr.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(0, len(seq), 2):
            seq[i](seq[i + 1])
            if i == 0:
                first_call[k].append(time.perf_counter() - t0)
        tr.synchronize()
        res[k].append(time.perf_counter() - t0)
    tr.set_epoch_indices(idx)
    tr.synchronize()
    t0 = time.perf_counter()
    tr.run_steps(LONG)
    tr.synchronize()
    longs.append((time.perf_counter() - t0) / LONG)
per = st.median(longs)
print(f"long run ({LONG} steps): {per * 1e3:.4f} ms/step")
for k in VARIANTS:
    m = st.median(res[k])
    print(f"{k:12s} 20 steps {m * 1e3:.3f} ms = {m / 20 * 1e3:.4f} ms/step; overhead vs long {(m - 20 * per) * 1e6:6.1f} us; "
          f"first launch call {st.median(first_call[k]) * 1e6:6.1f} us (host)", flush=True)
