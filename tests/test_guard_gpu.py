"""Out-of-bounds store audit of every launch the trainer makes (verdict r4, next-round item 1: "a host-side check
that every launch's address ranges stay inside their allocations").

With MNIST_AMD_GUARD=1 every buffer NativeTrainer hands the kernels sits between two 4 KiB guard regions of a known
byte pattern (engine/native.py _alloc); after whole epochs -- full batches through the captured step graphs or the
eager phase API, a partial last batch, evaluation -- no guard byte may have changed.  The eager phase path at MLP fp32
B=128 is the one the two-ranks-on-one-GPU test (tests/test_shared_gpu_ranks.py) runs, whose round-4 driver run lost
its box.  Reference step: /root/reference/ddp_tutorial_multi_gpu.py:86-98 (B=128 at :126).
"""
import pytest
import torch

from pytorch_ddp_mnist_amd.models import build_model

pytestmark = pytest.mark.gpu

CASES = [
    # (model, dtype, batch, data plane)
    ("mlp", "fp32", 128, "eager"),     # the shared-GPU test's path: phase API, host all-reduce
    ("mlp", "fp32", 128, "graph"),
    ("mlp", "bf16", 128, "graph"),
    ("mlp", "bf16", 4096, "graph"),    # 8 FC batch splits
    ("mlp", "fp32", 8192, "graph"),
    ("lenet5", "bf16", 128, "graph"),  # conv_bwd + FC wgrad/SGD in one kernel
    ("lenet5", "fp32", 128, "eager"),
    ("lenet5", "bf16", 1000, "graph"),
    ("lenet5", "bf16", 8192, "graph"),  # fused forward + head
]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,dtype,batch,plane", CASES, ids=lambda v: str(v))
def test_no_store_outside_buffers(native, monkeypatch, model, dtype, batch, plane):
    from pytorch_ddp_mnist_amd.data.synthetic import make_split
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer

    monkeypatch.setenv("MNIST_AMD_GUARD", "1")
    n = 3 * batch + batch // 3 + 1  # three full batches and a partial one
    x, y = make_split(max(n, 1024), seed=3)
    xt, yt = make_split(1000, seed=4)
    tr = NativeTrainer(model, dtype, batch, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                       dropout=0.2 if model == "mlp" else 0.0, momentum=0.9, init=build_model(model))
    assert tr._guards, "MNIST_AMD_GUARD=1 did not guard the buffers"
    if plane == "eager":
        tr.attach_external_allreduce(lambda t: None, 1, host=True)  # world 1: the phase API, no exchange
    for epoch in range(2):
        g = torch.Generator().manual_seed(epoch)
        tr.train_epoch(torch.randperm(x.shape[0], generator=g)[:n].to(torch.int32), use_graph=plane == "graph")
    tr.evaluate(torch.from_numpy(xt.reshape(-1, 784)), torch.from_numpy(yt), torch.arange(1000, dtype=torch.int32))
    assert tr.check_guards() == []
    assert torch.isfinite(tr.params).all()
    tr.close()
    tr.close()  # idempotent
    assert tr.rt is None
