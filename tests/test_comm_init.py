"""Bounded RCCL bring-up and ordered teardown (survey §5.3; reference: init_process_group(NCCL, env://)'s
c10d timeout, ddp_tutorial_multi_gpu.py:133-134).

CPU: the constructor's deadline logic (RcclComm.poll_ready + init_outcome) against a FAKE communicator that
never finishes its init, one that fails, and one that comes up; and the Python bring-up path
(make_rccl) with a rank whose unique id never arrives.  GPU: a real non-blocking RCCL init of a world of 2
whose second rank never arrives fails within the deadline, naming the rank, and the communicator of a
world of 1 is created non-blocking, used, and torn down in order.
"""
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _C():
    from pytorch_ddp_mnist_amd.ops.native import load_c
    return load_c()


def test_fake_init_never_ready_is_bounded():
    C = _C()
    t0 = time.perf_counter()
    err, waited, aborted = C.RcclComm._fake_init(3, 8, 0.3)
    el = time.perf_counter() - t0
    assert "rank 3 of 8" in err and "did not complete within" in err and "aborted" in err
    assert aborted
    assert 0.3 <= waited < 2.0 and el < 3.0


def test_fake_init_error_aborts():
    C = _C()
    err, waited, aborted = C.RcclComm._fake_init(1, 2, 5.0, fail=True)
    assert "rank 1 of 2" in err and "failed" in err
    assert aborted and waited < 1.0


def test_fake_init_ready():
    C = _C()
    err, waited, aborted = C.RcclComm._fake_init(0, 4, 5.0, ready_after=20)
    assert err == "" and not aborted and waited < 1.0


def test_make_rccl_uid_wait_is_bounded(tmp_path):
    """A non-zero rank whose unique id never appears in the TCPStore raises CommInitError within the deadline
    (in a subprocess: it initialises a gloo process group)."""
    code = textwrap.dedent(f"""
        import os, sys, time
        sys.path.insert(0, {ROOT!r})
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ["PORT"], WORLD_SIZE="1", RANK="0")
        import torch, torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://", world_size=1, rank=0)
        from pytorch_ddp_mnist_amd.parallel.comm import DistContext, make_rccl, CommInitError
        ctx = DistContext(rank=1, world=2, local_rank=0)
        t0 = time.perf_counter()
        try:
            make_rccl(ctx, timeout_s=0.5)
        except CommInitError as e:
            print("BOUNDED", round(time.perf_counter() - t0, 2), str(e)[:80])
        dist.destroy_process_group()
    """)
    from pytorch_ddp_mnist_amd.parallel.launch import free_port
    env = dict(os.environ, PORT=str(free_port()))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert "BOUNDED" in r.stdout, r.stdout + r.stderr
    secs = float(r.stdout.split("BOUNDED")[1].split()[0])
    assert secs < 10.0
    assert "rank 1 of 2" in r.stdout


@pytest.mark.gpu
def test_rccl_init_missing_peer_is_bounded(native):
    """World of 2, rank 1 never arrives: the non-blocking init is polled against the deadline, aborted, and
    the constructor raises naming the rank -- instead of hanging in ncclCommInitRank (own process: the
    aborted half-built communicator is left behind)."""
    code = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import torch
        from pytorch_ddp_mnist_amd.ops.native import require_gpu
        C = require_gpu()
        t0 = time.perf_counter()
        try:
            C.RcclComm(C.RcclComm.make_unique_id(), 0, 2, 0, init_timeout=5.0)
            print("NO-ERROR")
        except RuntimeError as e:
            print("BOUNDED", round(time.perf_counter() - t0, 2), str(e))
        sys.stdout.flush()
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=150)
    assert "BOUNDED" in r.stdout, r.stdout + r.stderr[-3000:]
    secs = float(r.stdout.split("BOUNDED")[1].split()[0])
    assert 5.0 <= secs < 60.0
    assert "rank 0 of 2" in r.stdout and "did not complete" in r.stdout


@pytest.mark.gpu
def test_rccl_nonblocking_world1_and_ordered_teardown(native, small_mnist):
    import torch

    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    C = native
    comm = C.RcclComm(C.RcclComm.make_unique_id(), 0, 1, 0)
    assert comm.nonblocking and comm.init_seconds >= 0.0
    x, y, _, _ = small_mnist
    torch.manual_seed(0)
    tr = NativeTrainer("lenet5", "bf16", 256, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                       init=build_model("lenet5"))
    tr.attach_comm(comm, 1)
    tr.set_epoch_indices(torch.arange(4096, dtype=torch.int32))
    tr.run_steps(12)
    tr.synchronize()
    # teardown order: graphs (captured collectives) dropped, then the communicator destroyed
    tr.release()
    assert tr.comm is None and not tr.rt.has_comm
    assert comm.destroy(60.0) == "" and comm.destroyed
    assert comm.destroy(60.0) == ""  # idempotent
    tr.run_steps(2, use_graph=False)  # the trainer still runs local steps
    tr.synchronize()
