"""Interleaved per-sample netCDF reads on the native GPU engine (reference mnist_pnetcdf_cpu_mp.py:39-49: each
batch read through MNISTNetCDF.__getitem__ inside the training loop).  The batch rows go through a pinned ring
one batch ahead of their step (the small-batch MLP head gathers the NEXT step's rows), so the training must be
bitwise that of the read-the-epoch-first mode."""
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = re.compile(r"^Epoch=0, train_loss=\d+\.\d{4}, val_loss=\d+\.\d{4}$", re.M)


def _run(args, cwd):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    return r.stdout


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model", ["mlp", "lenet5"])
def test_interleaved_equals_per_sample_on_gpu(native, tmp_path, model):
    _run([os.path.join(ROOT, "mnist_to_netcdf.py"), "--synthetic", "--output_dir", str(tmp_path)], tmp_path)
    args = [os.path.join(ROOT, "mnist_pnetcdf_cpu.py"), "--data_limit", "1000", "--init_seed", "1", "--model", model,
            "--device", "cuda"]
    per = _run(args + ["--io_mode", "per_sample"], tmp_path)
    inter = _run(args + ["--io_mode", "interleaved"], tmp_path)
    assert "native-hip" in inter, inter[-2000:]
    m = re.search(r"per-sample netCDF train: (\d+) samples", inter)
    assert m and int(m.group(1)) == 1000, inter
    assert LINE.search(inter).group(0) == LINE.search(per).group(0)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model", ["mlp", "lenet5"])
def test_bulk_netcdf_equals_idx_on_gpu(native, tmp_path, model):
    """The bulk netCDF path (CDF-5 file -> threaded pread -> pinned host memory -> hipMemcpyAsync -> HBM,
    data/device_loader.py upload_netcdf) trains bitwise like the idx-ubyte path on the same split: the same
    synthetic split is written both ways, one epoch each, and the two model.pt checkpoints are identical."""
    import torch
    _run([os.path.join(ROOT, "mnist_to_netcdf.py"), "--synthetic", "--output_dir", str(tmp_path)], tmp_path)
    common = ["--data_limit", "3000", "--init_seed", "1", "--model", model, "--device", "cuda"]
    nc = _run([os.path.join(ROOT, "mnist_pnetcdf_cpu.py"), "--io_mode", "bulk", "--save_path", "nc.pt"] + common,
              tmp_path)
    assert "native-hip" in nc and "Reading NetCDF" in nc, nc[-2000:]
    idx = _run([os.path.join(ROOT, "ddp_tutorial_cpu.py"), "--data_path", str(tmp_path / "mnist_data"),
                "--save_path", "idx.pt"] + common, tmp_path)
    assert "native-hip" in idx, idx[-2000:]
    a = torch.load(tmp_path / "nc.pt", weights_only=True)
    b = torch.load(tmp_path / "idx.pt", weights_only=True)
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert LINE.search(nc).group(0) == LINE.search(idx).group(0)
