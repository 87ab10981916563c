"""Teardown order at interpreter exit (verdict r5 item 7, the round-4 rank exit 139).

What the round-5 change prevents: the native trainer's streams, events and device counters used to be released by
the pybind11 destructor of ``Trainer``, which for a trainer still referenced at exit runs during interpreter
finalisation -- possibly after torch's exit handlers and the C++ static destructors have torn the HIP runtime down,
so hipStreamSynchronize / hipStreamDestroy / hipEventDestroy / hipFree then run against a dead runtime (a host
SIGSEGV, exit 139).  Now ``DistContext.finalize`` closes trainers explicitly, and an atexit hook
(engine/native.py ``_close_live_trainers``, registered after ``import torch``, so it runs first) closes every
trainer without collectives that a script left open.  The original crash was never reproduced (PARITY.md §5.3), so
the GPU test below pins the order rather than the crash: a script that exits holding a live trainer must exit 0 with
its native teardown done by the hook."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Fake:
    def __init__(self, comm=None):
        self.comm, self.oneshot, self.closed = comm, None, 0

    def close(self):
        self.closed += 1


def test_exit_hook_closes_local_trainers_only():
    from pytorch_ddp_mnist_amd.engine import native
    a, b = _Fake(), _Fake(comm=object())
    native._LIVE_TRAINERS.add(a)
    native._LIVE_TRAINERS.add(b)
    try:
        native._close_live_trainers()
    finally:
        native._LIVE_TRAINERS.discard(a)
        native._LIVE_TRAINERS.discard(b)
    assert a.closed == 1 and b.closed == 0  # a comm-attached trainer belongs to DistContext.finalize


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_live_trainer_at_exit_is_closed_by_the_hook():
    code = (
        "import torch, sys\n"
        "from pytorch_ddp_mnist_amd.data.synthetic import make_split\n"
        "from pytorch_ddp_mnist_amd.engine import native\n"
        "from pytorch_ddp_mnist_amd.models import build_model\n"
        "x, y = make_split(512, seed=1)\n"
        "tr = native.NativeTrainer('lenet5', 'bf16', 128, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),\n"
        "                          init=build_model('lenet5'))\n"
        "tr.set_epoch_indices(torch.arange(512, dtype=torch.int32))\n"
        "tr.run_steps(3)\n"
        "tr.synchronize()\n"
        "orig = native.NativeTrainer.close\n"
        "def close(self):\n"
        "    print('hook-close', file=sys.stderr, flush=True)\n"
        "    orig(self)\n"
        "native.NativeTrainer.close = close\n"
        "GLOBAL = tr  # still referenced when the interpreter exits\n"
    )
    env = dict(os.environ, PYTHONPATH=ROOT, MNIST_AMD_SEGV_TRACE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "hook-close" in r.stdout and "teardown at exit" not in r.stdout


def test_oneshot_epoch_barrier_and_end_agreement_selection():
    """The runner's one-shot guards (advisor r5): a barrier before each epoch's steps and an end-of-run latch
    agreement run exactly when a one-shot plane (data plane or OVERLAP instances) is attached."""
    from types import SimpleNamespace

    from pytorch_ddp_mnist_amd.engine.runner import _uses_oneshot
    assert not _uses_oneshot(SimpleNamespace(tr=SimpleNamespace(oneshot=None, overlap=None)))
    assert _uses_oneshot(SimpleNamespace(tr=SimpleNamespace(oneshot=object(), overlap=None)))
    assert _uses_oneshot(SimpleNamespace(tr=SimpleNamespace(oneshot=None, overlap=(object(), object()))))
    assert not _uses_oneshot(SimpleNamespace())  # the torch-CPU engine has no native trainer


def test_agree_oneshot_raises_on_every_rank():
    """NativeTrainer.agree_oneshot: a latch on ANY rank (reduce_max > 0) raises CollectiveError on this rank too,
    also when this rank's own instances report no error."""
    import pytest as _pt

    from pytorch_ddp_mnist_amd.engine.native import CollectiveError, NativeTrainer

    class _Inst:
        def __init__(self, err):
            self.err = err

        def check(self):
            return self.err

    class _Stream:
        def synchronize(self):
            pass

    fake = type("FakeTrainer", (), {})()
    fake.stream = _Stream()
    fake.oneshot, fake.overlap = _Inst(""), None
    fake._oneshot_instances = lambda: [fake.oneshot]
    NativeTrainer.agree_oneshot(fake, lambda v: v)           # nobody failed: no error
    with _pt.raises(CollectiveError, match="peer rank"):
        NativeTrainer.agree_oneshot(fake, lambda v: 1.0)     # a peer latched a failure
    fake.oneshot = _Inst("flag wait timed out")
    with _pt.raises(CollectiveError, match="timed out"):
        NativeTrainer.agree_oneshot(fake, lambda v: v)
