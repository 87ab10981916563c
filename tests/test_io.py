"""idx-ubyte and CDF-5 (PnetCDF '64BIT_DATA') readers/writers: native vs pure Python (survey App. A/B)."""
import os
import struct

import numpy as np
import pytest
import torch

from pytorch_ddp_mnist_amd.data import cdf5, idx
from pytorch_ddp_mnist_amd.data.datasets import MNISTIdx, MNISTNetCDF, find_idx, load_arrays, mnist_transform
from pytorch_ddp_mnist_amd.data.synthetic import make_split
from pytorch_ddp_mnist_amd.ops.native import load_io

HAVE_IO = load_io() is not None


@pytest.fixture(scope="module")
def data():
    return make_split(300, seed=3)


@pytest.mark.parametrize("native", [False, True] if HAVE_IO else [False])
def test_idx_roundtrip(tmp_path, data, native):
    x, y = data
    pi, pl = str(tmp_path / "img"), str(tmp_path / "lab")
    idx.write_idx(pi, x, native=native)
    idx.write_idx(pl, y, native=native)
    with open(pi, "rb") as f:
        assert struct.unpack(">IIII", f.read(16)) == (2051, 300, 28, 28)
    with open(pl, "rb") as f:
        assert struct.unpack(">II", f.read(8)) == (2049, 300)
    for nat in ([False, True] if HAVE_IO else [False]):
        assert np.array_equal(idx.read_idx(pi, native=nat), x)
        assert np.array_equal(idx.read_idx(pl, native=nat), y)
        assert np.array_equal(idx.read_idx(pi, limit=7, native=nat), x[:7])
    xi, yi = idx.read_images_labels(pi, pl)
    assert np.array_equal(xi, x) and np.array_equal(yi, y)
    with pytest.raises(ValueError):
        idx.read_images_labels(pl, pi)


@pytest.mark.parametrize("writer_native", [False, True] if HAVE_IO else [False])
def test_cdf5_roundtrip_and_header(tmp_path, data, writer_native):
    x, y = data
    p = str(tmp_path / "mnist_train_images.nc")
    cdf5.write_mnist_nc(p, x, y, native=writer_native)
    raw = open(p, "rb").read()
    assert raw[:4] == b"CDF\x05"
    for reader_native in ([False, True] if HAVE_IO else [False]):
        f = cdf5.open_nc(p, native=reader_native)
        assert [tuple(d) for d in f.dims()] == [("Y", 28), ("X", 28), ("idx", 300)]
        assert list(f.variables()) == ["images", "labels"]
        info = f.var_info("images")
        assert info["type"] == 7 and list(info["shape"]) == [300, 28, 28] and info["begin"] % 512 == 0
        assert list(info["dims"]) == ["idx", "Y", "X"]
        assert np.array_equal(f.read_rows("images"), x)
        assert np.array_equal(f.read_rows("labels"), y)
        assert np.array_equal(f.read_rows("images", 17, 5), x[17:22])
        assert np.array_equal(f.read_row("images", 299)[0], x[299])
        # data bytes sit exactly at the header's begin offsets
        b = f.begin("labels")
        assert raw[b:b + 300] == y.tobytes()


def test_cdf5_general_types(tmp_path):
    p = str(tmp_path / "t.nc")
    a = np.arange(12, dtype=np.float32).reshape(3, 4) * 0.5
    b = np.arange(3, dtype=np.int16) - 1
    for native in ([False, True] if HAVE_IO else [False]):
        cdf5.write_cdf5(p, [("r", 3), ("c", 4)], [("a", [0, 1], a), ("b", [0], b)], native=native)
        for rn in ([False, True] if HAVE_IO else [False]):
            f = cdf5.open_nc(p, native=rn)
            assert np.array_equal(f.read_rows("a"), a) and np.array_equal(f.read_rows("b"), b)


@pytest.mark.skipif(not HAVE_IO, reason="native _io not built")
def test_read_rows_into_pinned_like_buffer(tmp_path, data):
    x, y = data
    p = str(tmp_path / "m.nc")
    cdf5.write_mnist_nc(p, x, y)
    f = cdf5.open_nc(p)
    buf = torch.zeros(50 * 784, dtype=torch.uint8)
    n = f.read_rows_into("images", 100, 50, buf.data_ptr(), buf.numel(), 4)
    assert n == 50 * 784 and torch.equal(buf.view(50, 28, 28), torch.from_numpy(x[100:150]))
    with pytest.raises(Exception):
        f.read_rows_into("images", 0, 51, buf.data_ptr(), buf.numel(), 1)


def test_sharded_read(tmp_path, data):
    x, y = data
    p = str(tmp_path / "m.nc")
    cdf5.write_mnist_nc(p, x, y)
    parts = [cdf5.read_mnist_nc(p, rank=r, world=3) for r in range(3)]
    assert np.array_equal(np.concatenate([a for a, _ in parts]), x)
    assert np.array_equal(np.concatenate([b for _, b in parts]), y)


def test_datasets_api(tmp_path, data, capsys):
    x, y = data
    cdf5.write_mnist_nc(str(tmp_path / "mnist_train_images.nc"), x, y)
    ds = MNISTNetCDF(str(tmp_path), is_train=True, transforms=mnist_transform)
    out = capsys.readouterr().out
    assert "=> Reading NetCDF File..." in out and "=> Dataset created, image nc file is : " in out
    assert len(ds) == 300
    img, lab = ds[5]
    assert img.shape == (1, 28, 28) and lab.dtype == np.uint8 and lab.shape == () and int(lab) == int(y[5])
    ref = (torch.from_numpy(x[5]).float() / 255 - 0.1307) / 0.3081
    assert torch.allclose(img[0], ref)
    idx.write_mnist_idx(str(tmp_path / "d"), (x, y), (x[:10], y[:10]), layout="kaggle")
    assert find_idx(str(tmp_path / "d")) is not None
    m = MNISTIdx(str(tmp_path / "d"), train=False)
    assert len(m) == 10 and m[3][1] == int(y[3])
    xt, yt, xe, ye, src = load_arrays("idx", str(tmp_path / "d"), limit=100)
    assert xt.shape == (100, 28, 28) and xe.shape == (10, 28, 28) and "idx" in src


def test_synthetic_is_deterministic_and_learnable():
    a, la = make_split(2000, seed=1)
    b, lb = make_split(2000, seed=1)
    assert np.array_equal(a, b) and np.array_equal(la, lb)
    # nearest-class-mean on raw pixels already separates the classes well
    means = np.stack([a[la == c].reshape(-1, 784).mean(0) for c in range(10)])
    t, lt = make_split(500, seed=2)
    pred = np.argmin(((t.reshape(-1, 1, 784) - means[None]) ** 2).sum(-1), axis=1)
    assert (pred == lt).mean() > 0.7
