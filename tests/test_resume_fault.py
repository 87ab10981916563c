"""Resume (params + momentum + epoch), fault injection and the NaN/Inf guard (survey §5.2-5.4)."""
import os
import subprocess
import sys

import pytest
import torch

from pytorch_ddp_mnist_amd.config import TrainConfig
from pytorch_ddp_mnist_amd.engine.runner import run
from pytorch_ddp_mnist_amd.utils.fault import FaultInjector, InjectedFault, check_finite

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(tmp_path, **kw):
    c = TrainConfig(model="mlp", dropout=0.0, momentum=0.9, lr=0.05, device="cpu", data_format="synthetic",
                    data_limit=1024, batch_size=128, save_path=None, init_seed=0)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@pytest.mark.parametrize("model", ["mlp", "lenet5"])
def test_resume_equals_uninterrupted(tmp_path, model):
    full = run(_cfg(tmp_path, model=model, n_epochs=3))["state_dict"]
    path = str(tmp_path / "resume.pt")
    run(_cfg(tmp_path, model=model, n_epochs=1, resume=path))
    assert os.path.exists(path)
    part2 = run(_cfg(tmp_path, model=model, n_epochs=3, resume=path))
    assert [h["epoch"] for h in part2["history"]] == [1, 2]
    for k in full:
        assert torch.allclose(full[k], part2["state_dict"][k], rtol=1e-6, atol=1e-7), k
    # the resume file holds only tensors and plain values (weights_only loading)
    blob = torch.load(path, weights_only=True)
    assert blob["epoch"] == 2 and blob["model"] == model and "momentum" in blob


def test_fault_injector_semantics():
    f = FaultInjector(rank=1, env={"MNIST_AMD_FAIL_AT_STEP": "2", "MNIST_AMD_FAIL_RANK": "1"})
    f.tick()
    f.tick()
    with pytest.raises(InjectedFault):
        f.tick()
    other = FaultInjector(rank=0, env={"MNIST_AMD_FAIL_AT_STEP": "0", "MNIST_AMD_FAIL_RANK": "1"})
    for _ in range(5):
        other.tick()
    with pytest.raises(FloatingPointError):
        check_finite("loss", 1.0, float("nan"))


def test_injected_rank_failure_takes_job_down(tmp_path):
    """Rank 1 dies at step 3; rank 0 would block in its next gradient all-reduce: the launcher must
    end the whole job promptly with a non-zero code and the injected message."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", MNIST_AMD_FAIL_AT_STEP="3", MNIST_AMD_FAIL_RANK="1")
    r = subprocess.run([sys.executable, "-m", "pytorch_ddp_mnist_amd.parallel.launch", "-n", "2", "--style", "ompi",
                        "--timeout", "120", "--", sys.executable, os.path.join(ROOT, "mnist_cpu_mp.py"), "--parallel",
                        "--wireup_method", "gloo", "--data_limit", "4096", "--device", "cpu", "--synthetic"],
                       cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=150)
    assert r.returncode != 0
    assert "injected failure at step 3 on rank 1" in r.stdout
