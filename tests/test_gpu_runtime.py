"""T5: native RCCL communicator and the GPU paths of the entry scripts on one MI355X.

RCCL refuses two ranks on one GPU, so multi-rank collectives are covered by the CPU gloo tests
(test_ddp_cpu.py) and by the driver's 8-GPU bench; here the communicator runs at world size 1
(a real ncclAllReduce / ncclBroadcast, also captured inside the step hipGraph).
"""
import os
import re
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_world1_collectives(native):
    C = native
    comm = C.RcclComm(C.RcclComm.make_unique_id(), 0, 1, 0)
    x = torch.arange(1000, dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    comm.all_reduce_sum_f32(x.data_ptr(), x.numel(), s.cuda_stream)
    comm.broadcast_f32(x.data_ptr(), x.numel(), 0, s.cuda_stream)
    assert comm.wait_stream(s.cuda_stream, 60.0) == ""
    assert torch.equal(x.cpu(), torch.arange(1000, dtype=torch.float32))
    assert comm.async_error() == ""
    assert (comm.rank, comm.world) == (0, 1)


@pytest.mark.parametrize("plan", ["join", "split"])
@pytest.mark.parametrize("model_name", ["mlp", "lenet5"])
def test_rccl_inside_captured_step(native, small_mnist, model_name, plan):
    """The step graph with the RCCL bucket all-reduces captured (main or comm stream) == eager without comm."""
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    x, y, _, _ = small_mnist
    torch.manual_seed(0)
    m = build_model(model_name)
    idx = torch.randperm(len(y), generator=torch.Generator().manual_seed(1))[:128 * 3].to(torch.int32)
    out = []
    for with_comm in (False, True):
        tr = NativeTrainer(model_name, "bf16", 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                           dropout=0.0, init=m)
        if with_comm:
            tr.attach_comm(native.RcclComm(native.RcclComm.make_unique_id(), 0, 1, 0), 1, plan=plan)
            tr.broadcast_params(0)
        tr.set_epoch_indices(idx)
        for _ in range(3):
            tr.step(128, use_graph=with_comm)
        tr.synchronize()
        out.append(tr.params.cpu())
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("model_name", ["mlp", "lenet5"])
def test_module_ddp_rccl_on_gpu(native, model_name):
    """Bring-your-own-model DDP wrapper on cuda:0 with the native RCCL comm (bucket all-reduces on its
    side stream, world 1) == the same torch model trained without the wrapper."""
    import torch.nn.functional as F
    from pytorch_ddp_mnist_amd.models import build_model
    from pytorch_ddp_mnist_amd.parallel.module_ddp import DistributedDataParallel
    comm = native.RcclComm(native.RcclComm.make_unique_id(), 0, 1, 0)
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(64, 784, generator=g) for _ in range(3)]
    ys = [torch.randint(0, 10, (64,), generator=g) for _ in range(3)]
    out = []
    for wrap in (False, True):
        torch.manual_seed(1)
        m = build_model(model_name).cuda()
        if model_name == "mlp":
            m[2].p = 0.0
        dm = DistributedDataParallel(m, rccl=comm, bucket_cap_mb=0.1, first_bucket_mb=0.05) if wrap else m
        opt = torch.optim.SGD(dm.parameters(), lr=0.05, momentum=0.9)
        for x, y in zip(xs, ys):
            x = x.cuda().view(-1, 1, 28, 28) if model_name == "lenet5" else x.cuda()
            opt.zero_grad()
            o = dm(x)
            (F.nll_loss(o, y.cuda()) if model_name == "lenet5" else F.cross_entropy(o, y.cuda())).backward()
            opt.step()
        torch.cuda.synchronize()
        out.append(torch.cat([p.detach().reshape(-1).cpu() for p in m.parameters()]))
        if wrap:
            assert len(dm.buckets) > 1
    if model_name == "mlp":
        assert torch.equal(out[0], out[1])
    else:  # MIOpen's conv weight-gradient kernels are not run-to-run deterministic
        assert torch.allclose(out[0], out[1], rtol=1e-5, atol=1e-6), (out[0] - out[1]).abs().max()
    assert comm.async_error() == ""


def _run(args, cwd, timeout=600):
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=dict(os.environ, PYTHONPATH=ROOT),
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:]
    return r.stdout


@pytest.mark.timeout(600)  # spawns fresh interpreters (torch import + GPU init)
def test_multi_gpu_tutorial_single_rank(tmp_path):
    out = _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
                "--master-port", "29617", os.path.join(ROOT, "ddp_tutorial_multi_gpu.py"), "--epochs", "2",
                "--model", "lenet5", "--dtype", "bf16", "--synthetic", "--init_seed", "0"], tmp_path)
    lines = re.findall(r"^Epoch=(\d), train_loss=\d+\.\d{4}, val_loss=\d+\.\d{4}$", out, re.M)
    assert lines == ["0", "1"], out
    assert "native-hip" in out
    sd = torch.load(tmp_path / "model.pt", weights_only=True)
    assert list(sd)[0] == "0.weight" and sd["7.weight"].shape == (120, 400)
    # learning, not a tuned accuracy: the reference seeds nothing, and two epochs of B=128 from different random
    # inits ended at val_acc 0.41 .. 0.95 on one box (profiles/r6_final/tutorial_runs.txt) -- so the init is
    # pinned (--init_seed) and the bar is well above chance with the validation loss falling
    acc = [float(a) for a in re.findall(r"val_acc=([0-9.]+)", out)]
    vl = [float(v) for v in re.findall(r"global_train_loss=[0-9.]+ train_acc=[0-9.]+ val_loss=([0-9.]+)", out)]
    assert acc[-1] > 0.3 and len(vl) == 2 and vl[1] < vl[0], out


@pytest.mark.timeout(600)  # spawns fresh interpreters (torch import + GPU init)
def test_reference_mlp_on_gpu_matches_cpu_engine(tmp_path):
    """Same script, same seed, fp32, dropout 0: native GPU and torch-CPU epochs agree closely."""
    args = [os.path.join(ROOT, "mnist_cpu_mp.py"), "--data_limit", "4096", "--synthetic", "--dropout", "0",
            "--init_seed", "3", "--no_save"]
    out_gpu = _run(args + ["--device", "cuda"], tmp_path)
    out_cpu = _run(args + ["--device", "cpu"], tmp_path)
    lg = re.search(r"global_train_loss=([0-9.]+).*val_loss=([0-9.]+) val_acc=([0-9.]+)", out_gpu).groups()
    lc = re.search(r"global_train_loss=([0-9.]+).*val_loss=([0-9.]+) val_acc=([0-9.]+)", out_cpu).groups()
    for a, b in zip(lg, lc):
        assert abs(float(a) - float(b)) < 2e-3, (out_gpu, out_cpu)

@pytest.mark.parametrize("with_comm", [False, True])
@pytest.mark.parametrize("model_name", ["mlp", "lenet5"])
def test_multi_step_graph_matches_single_steps(native, small_mnist, model_name, with_comm):
    """run_steps: k steps in one hipGraph (plus single-step remainder) == the same steps one graph each,
    bitwise (same kernels, same order); the loaded order bounds the k-step windows."""
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    x, y, _, _ = small_mnist
    torch.manual_seed(0)
    m = build_model(model_name)
    idx = torch.randperm(len(y), generator=torch.Generator().manual_seed(2))[:128 * 11].to(torch.int32)
    out = []
    for k in (1, 4):
        tr = NativeTrainer(model_name, "bf16", 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                           dropout=0.0, init=m)
        if with_comm:
            tr.attach_comm(native.RcclComm(native.RcclComm.make_unique_id(), 0, 1, 0), 1)
            tr.broadcast_params(0)
        tr.set_epoch_indices(idx)
        tr.run_steps(11, use_graph=True, k=k)   # k=4: two 4-step graphs + 3 single steps
        tr.synchronize()
        assert tr.host_step == 11
        out.append((tr.params.cpu(), tr.read_metrics().loss_sum))
        if k == 4:
            assert tr.rt.multi_steps == 4
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1] == pytest.approx(out[1][1], rel=1e-6)   # loss sum: float atomics, order-dependent


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_mlp_fused_wgrad_sgd_matches_separate_update(native, small_mnist, dtype, momentum):
    """MLP one-GPU step with the SGD update as the wgrad epilogue == wgrad + reduce_sgd kernels, bitwise
    (params, momentum, step counters), over full and partial batches, eager and captured."""
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    x, y, _, _ = small_mnist
    torch.manual_seed(0)
    m = build_model("mlp")
    idx = torch.randperm(len(y), generator=torch.Generator().manual_seed(3))[:128 * 4 + 40].to(torch.int32)
    out = []
    for fuse in (False, True):
        tr = NativeTrainer("mlp", dtype, 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                           dropout=0.2, init=m, fc_splits=1, momentum=momentum)
        tr.rt.fuse_wgrad_sgd = fuse
        tr.set_epoch_indices(idx)
        tr.run_steps(3, use_graph=True)
        tr.step(128, use_graph=False)
        tr.step(40, use_graph=False)
        tr.synchronize()
        out.append((tr.params.cpu(), tr.mom.cpu(), tr.step_ctr.cpu()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][2], out[1][2]) and out[1][2].tolist()[:2] == [5, 5]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_mlp_lookahead_gather_matches_direct_gather(native, small_mnist, dtype, monkeypatch):
    """Small-batch MLP: the rows gathered one step ahead (by the previous head kernel / the prime after
    set_epoch_indices) give bitwise the same training as gathering through the index order in place --
    over graph and eager steps, a partial last batch and a second epoch with a new order."""
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    x, y, _, _ = small_mnist
    torch.manual_seed(0)
    m = build_model("mlp")
    g = torch.Generator().manual_seed(7)
    orders = [torch.randperm(len(y), generator=g)[:128 * 5 + 40].to(torch.int32) for _ in range(2)]
    out = []
    for look in (False, True):
        if look:
            monkeypatch.delenv("MNIST_AMD_NO_LOOKAHEAD", raising=False)
        else:
            monkeypatch.setenv("MNIST_AMD_NO_LOOKAHEAD", "1")
        tr = NativeTrainer("mlp", dtype, 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                           dropout=0.2, init=m, momentum=0.9)
        assert (tr.xnext is not None) == look
        for order in orders:
            tr.set_epoch_indices(order)
            tr.reset_metrics()
            tr.run_steps(3, use_graph=True)
            tr.step(128, use_graph=False)
            tr.step(128, use_graph=True)
            tr.step(40, use_graph=False)
        tr.synchronize()
        out.append((tr.params.cpu(), tr.read_metrics().correct))
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]
