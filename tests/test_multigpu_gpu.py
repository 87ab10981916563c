"""Multi-rank arithmetic, plan autotuning and the collective watchdog of the native trainer, on ONE GPU.

RCCL refuses two ranks on one device, so a 2-rank job is emulated with the phase API: two
NativeTrainers train on the two DistributedSampler shards (disjoint halves of every global batch),
their reduced gradients are summed as the all-reduce would, and each applies ``optimizer_step(1/2)``.
That must equal ONE trainer stepping on the concatenated global batches (DDP semantics, reference
ddp_tutorial_multi_gpu.py:72 / survey CS5), partial last batch included.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _shards(n, world, batch):
    """Per-rank index orders (DistributedSampler) and the single-trainer order whose global batch j is
    the concatenation of every rank's batch j."""
    from pytorch_ddp_mnist_amd.data.sampler import epoch_indices
    per = [epoch_indices(n, world, r, 0, seed=42).to(torch.int32) for r in range(world)]
    glob = []
    for s in range(0, per[0].numel(), batch):
        glob += [p[s:s + batch] for p in per]
    return per, torch.cat(glob)


@pytest.mark.parametrize("model_name", ["mlp", "lenet5"])
def test_two_rank_emulation_equals_global_batch(native, small_mnist, model_name):
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    x, y, _, _ = small_mnist
    n, W, B = 1000, 2, 128                      # 500 per rank: 3 full batches + a partial one of 116
    per, glob = _shards(n, W, B)
    xs, ys = torch.from_numpy(x[:n].reshape(-1, 784)), torch.from_numpy(y[:n])
    torch.manual_seed(0)
    init = build_model(model_name)
    kw = dict(lr=0.05, momentum=0.9, dropout=0.0, init=init)
    ranks = [NativeTrainer(model_name, "fp32", B, xs, ys, **kw) for _ in range(W)]
    big = NativeTrainer(model_name, "fp32", W * B, xs, ys, **kw)
    for tr, idx in zip(ranks, per):
        tr.set_epoch_indices(idx)
    big.set_epoch_indices(glob)
    for s in range(0, per[0].numel(), B):
        b = min(B, per[0].numel() - s)
        for tr in ranks:
            tr.forward_backward(b)
        g = sum(tr.grads() for tr in ranks)        # the SUM all-reduce
        for tr in ranks:
            tr.grad.copy_(g.to(tr.grad.device))
            torch.cuda.current_stream().synchronize()
            tr.optimizer_step(1.0 / W)             # 1/W averaging folded into the SGD kernel
        big.forward_backward(W * b)
        big.optimizer_step(1.0)
    for tr in ranks + [big]:
        tr.synchronize()
    p = [tr.params.cpu() for tr in ranks] + [big.params.cpu()]
    assert torch.equal(p[0], p[1])                  # replicas stay identical
    rel = ((p[0] - p[2]).norm() / p[2].norm()).item()
    assert rel <= 1e-6, rel
    moved = ((p[2] - torch.cat([t.detach().reshape(-1) for t in init.parameters()])).norm() / p[2].norm()).item()
    assert moved > 1e-3                             # the comparison is not vacuous


def test_watchdog_times_out_and_aborts(native, small_mnist):
    """A stream that never drains (here: a bounded 3 s device spin) hits the collective deadline: the
    communicator is aborted and CollectiveError is raised promptly instead of a silent hang."""
    from pytorch_ddp_mnist_amd.engine.native import CollectiveError, NativeTrainer
    x, y, _, _ = small_mnist
    tr = NativeTrainer("lenet5", "bf16", 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y), dropout=0.0)
    comm = native.RcclComm(native.RcclComm.make_unique_id(), 0, 1, 0)
    tr.attach_comm(comm, 1)
    tr.broadcast_params(0)
    tr.check_comm()
    tr.rt.spin(3.0, tr.stream.cuda_stream)
    with pytest.raises(CollectiveError, match="timeout") as ei:
        tr.synchronize(timeout=0.3)
    assert 0.3 <= ei.value.detected_after < 1.0, ei.value.detected_after
    assert comm.aborted
    tr.stream.synchronize()                         # the spin ends on its own; the device is healthy
    z = torch.ones(4, device="cuda") * 2
    assert z.sum().item() == 8.0


def test_autotune_plan_restores_state(native, small_mnist):
    """Autotuning replays candidate step graphs on the real communicator, then restores the parameters,
    momentum, counters and metrics bitwise and leaves the chosen plan installed."""
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    x, y, _, _ = small_mnist
    torch.manual_seed(0)
    tr = NativeTrainer("lenet5", "bf16", 512, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                       lr=0.05, momentum=0.9, dropout=0.0, init=build_model("lenet5"))
    tr.attach_comm(native.RcclComm(native.RcclComm.make_unique_id(), 0, 1, 0), 1)
    tr.broadcast_params(0)
    tr.set_epoch_indices(torch.arange(4096, dtype=torch.int32))
    tr.step(512)                                    # non-trivial momentum / counters before tuning
    tr.synchronize()
    before = [t.clone() for t in (tr.params, tr.mom, tr.step_ctr, tr.metrics, tr.pack_buf)]
    out = tr.autotune_plan(iters=4, warmup=1)
    tr.synchronize()
    after = (tr.params, tr.mom, tr.step_ctr, tr.metrics, tr.pack_buf)
    for a, b in zip(before, after):
        assert torch.equal(a, b)
    assert out["chosen"] in out["timings_ms"] and all(v > 0 for v in out["timings_ms"].values())
    assert set(out["timings_ms"]) >= {"join", "split"}
    info = tr.plan_info()
    assert info["plan"] == out["candidates"][out["chosen"]]["plan"]
    assert tr.rt.bwd_grid == tr.C.conv_bwd_blocks(512, out["candidates"][out["chosen"]]["bwd_blocks"])
    assert sum(c["bytes"] for c in info["collectives"]) == 4 * tr.nparam
    tr.step(512)                                    # the installed plan trains
    tr.synchronize()
    assert torch.isfinite(tr.params).all()


def test_rccl_cross_stream_capture_pattern(native):
    """The capture pattern the SPLIT plan was written to avoid (ROCm 7.0: hipStreamEndCapture segfaulted on a
    related form): a stream waiting on an event recorded behind a captured RCCL all-reduce, joined back into the
    capturing stream.  On the box's runtime it captures, instantiates and replays (world 1), and the all-reduce
    it carries is the identity there."""
    comm = native.RcclComm(native.RcclComm.make_unique_id(), 0, 1, 0)
    x = torch.randn(61706, device="cuda")
    ref = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    err = comm.probe_cross_stream_capture(x.data_ptr(), x.numel(), s.cuda_stream, replays=3, timeout=60.0)
    assert err == "", err
    s.synchronize()
    assert torch.equal(x, ref)
    assert comm.destroy(60.0) == ""
