"""One rank of the one-shot fault-injection job (tests/test_oneshot_gpu.py::test_oneshot_missing_peer_call_latches).

Two rank processes share one GPU (gloo control plane, one-shot data plane over IPC).  Both train three eager
MLP steps whose gradient all-reduce is the one-shot kernel; then rank 1 does NOT issue its fourth call
(``MNIST_AMD_ONESHOT_SKIP_CALL=1:3``, csrc/runtime/oneshot.cpp).  Rank 0's fourth call must time out in the
kernel (bound ``MNIST_AMD_ONESHOT_TIMEOUT``), latch the error, skip the parameter update behind it, and raise
CollectiveError at the next host wait.  Each rank prints one JSON line on stdout.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import torch

    from pytorch_ddp_mnist_amd.data.synthetic import make_split
    from pytorch_ddp_mnist_amd.engine.native import CollectiveError, NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    from pytorch_ddp_mnist_amd.parallel.comm import init_distributed
    from pytorch_ddp_mnist_amd.parallel.oneshot import make_oneshot

    ctx = init_distributed(None, parallel=True, device="cuda", comm="gloo", share_device=True)
    x, y = make_split(2048, seed=3)
    torch.manual_seed(0)
    tr = NativeTrainer("mlp", "fp32", 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                       device=ctx.device, lr=0.05, momentum=0.9, dropout=0.0, init=build_model("mlp"))
    tr.set_epoch_indices(torch.arange(2048, dtype=torch.int32))
    o = make_oneshot(ctx, tr.nparam)
    tr.attach_oneshot(o, ctx.world)
    tr.broadcast_params(0)
    for _ in range(3):  # one-shot calls 0, 1, 2 on both ranks
        tr.step(use_graph=False)
    tr.synchronize()
    before = tr.params.detach().cpu().clone()
    ctx.barrier()
    t0 = time.perf_counter()
    tr.step(use_graph=False)  # call 3: rank 1 skips it
    raised, msg = False, ""
    try:
        tr.synchronize()
    except CollectiveError as e:
        raised, msg = True, str(e)
    dt = time.perf_counter() - t0
    after = tr.params.detach().cpu()
    out = {"rank": ctx.rank, "raised": raised, "seconds": round(dt, 3), "msg": msg,
           "params_unchanged": bool(torch.equal(before, after)), "calls": o.calls}
    ctx.barrier()
    print(json.dumps(out), flush=True)
    ctx.finalize(tr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
