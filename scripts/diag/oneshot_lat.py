"""World-1 latency of the one-shot all-reduce kernel (graph-replayed, median) by block count and size, and where a
call's time goes: per-block wall-clock stamps (entry -> pushes drained -> own flags seen -> slots summed), medians
over blocks and calls (MNIST_AMD verdict r4 item 4: break the ~14.6 us world-1 floor down)."""
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.ops.native import load_c  # noqa: E402
from pytorch_ddp_mnist_amd.parallel.oneshot import time_oneshot  # noqa: E402

C = load_c()
dev = torch.device("cuda", 0)
for nblk in (8, 16, 64):
    o = C.OneShotAllReduce(0, 1, 0, 118272, nblk)
    for n in (2572, 59134, 118272):
        ms1 = time_oneshot(o, n, dev, iters=100, warmup=10)  # one call per graph: the host's launch rate
        ms = time_oneshot(o, n, dev, iters=100, warmup=10, per_graph=8)
        # phase breakdown (direct launches, stamps on)
        o.enable_stamps(True)
        buf = torch.zeros(n, device=dev)
        s = torch.cuda.current_stream()
        ph = {"push": [], "flag": [], "sum": [], "span": []}
        for _ in range(20):
            o.all_reduce_sum_f32(buf.data_ptr(), n, s.cuda_stream)
            s.synchronize()
            t = o.stamps()
            rows = [t[4 * b:4 * b + 4] for b in range(nblk)]
            t0 = min(r[0] for r in rows)
            ph["push"].append(st.median(r[1] - r[0] for r in rows))
            ph["flag"].append(st.median(r[2] - r[1] for r in rows))
            ph["sum"].append(st.median(r[3] - r[2] for r in rows))
            ph["span"].append(max(r[3] for r in rows) - t0)
        o.enable_stamps(False)
        med = {k: st.median(v) / 100.0 for k, v in ph.items()}  # 100 MHz ticks -> us
        print(f"nblk {nblk:3d}  count {n:6d}  per call {ms * 1000:6.2f} us (1/graph {ms1 * 1000:6.2f}) | in-kernel span {med['span']:6.2f}  "
              f"push {med['push']:5.2f}  flag {med['flag']:5.2f}  sum {med['sum']:5.2f} us", flush=True)
    assert o.check() == ""

# RCCL at world 1 for comparison (its collective is a local copy there), same per-call method
comm = C.RcclComm(C.RcclComm.make_unique_id(), 0, 1, 0)
s = torch.cuda.Stream()
for n in (2572, 59134, 118272):
    buf = torch.zeros(n, device=dev)
    s.wait_stream(torch.cuda.current_stream())
    one = st.median(comm.time_all_reduce(buf.data_ptr(), n, 10, 100, s.cuda_stream, 60.0, per_graph=1))
    per = st.median(comm.time_all_reduce(buf.data_ptr(), n, 10, 100, s.cuda_stream, 60.0, per_graph=8))
    print(f"rccl world 1  count {n:6d}  per call {per * 1000:6.2f} us (1/graph {one * 1000:6.2f})", flush=True)
assert comm.destroy(60.0) == ""
