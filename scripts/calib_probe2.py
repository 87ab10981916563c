"""Bisect the calibration slowdown of the serial LeNet schedule at B=128 (see scripts/calib_probe.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
x, y = make_split(60000, seed=1)
dev = torch.device("cuda", 0)
tr = NativeTrainer("lenet5", "bf16", B, torch.from_numpy(x.reshape(-1, 784)).to(dev), torch.from_numpy(y).to(dev),
                   device=dev, lr=0.05, momentum=0.9, dropout=0.0, init=build_model("lenet5"))
order = torch.randperm(60000, dtype=torch.int32)[: (60000 // B) * B]
tr.set_epoch_indices(order)
ser, con = {"concurrent": False}, {"concurrent": True}
st = tr.stream
for c in (con, ser):
    tr.apply_plan(c)
    tr.prepare_graphs()


def seg(cfg, tag, n=6, blk=4, events=True):
    tr.apply_plan(cfg)
    with torch.cuda.stream(st):
        tr.step_ctr[0].zero_()
    ts = []
    a0, b0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a0.record(st)
    for j in range(n):
        if events:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
        for _ in range(blk):
            tr.rt.replay_multi(st.cuda_stream)
        if events:
            b.record(st)
            ts.append((a, b))
    b0.record(st)
    tr.synchronize()
    per = [x.elapsed_time(y) / (8 * blk) * 1000 for x, y in ts]
    print(f"{tag}: whole {a0.elapsed_time(b0) / (8 * blk * n) * 1000:.2f} us/step; samples "
          + " ".join(f"{v:.1f}" for v in per), flush=True)


seg(ser, "serial (events)")
seg(ser, "serial (no events)", events=False)
seg(con, "concurrent (events)")
seg(ser, "serial after concurrent (events)")
seg(ser, "serial again (events)")
seg(ser, "serial again (no events)", events=False)
seg(con, "concurrent (no events)", events=False)
seg(ser, "serial after concurrent (no events)", events=False)
