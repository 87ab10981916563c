"""idx-ubyte -> CDF-5 converter (reference: mnist_to_netcdf.ipynb).

Reads the four MNIST idx files (the notebook's Kaggle layout ``<dir>/<name>/<name>``, the
torchvision layout ``<dir>/MNIST/raw/<name>`` or flat files) with magic-number checks, and writes
``mnist_train_images.nc`` / ``mnist_test_images.nc``: CDF-5 ("64BIT_DATA"), dims Y=28, X=28,
idx=N, variables images(idx,Y,X) and labels(idx) as NC_UBYTE — the notebook's ``to_nc`` layout —
with one bulk write per variable from one process (survey Q17: upstream issued one collective
write per image from every rank).  ``--synthetic`` converts the deterministic synthetic set.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_ddp_mnist_amd.data import cdf5, idx  # noqa: E402
from pytorch_ddp_mnist_amd.data.datasets import IDX_NAMES, find_idx  # noqa: E402
from pytorch_ddp_mnist_amd.data.synthetic import make_mnist  # noqa: E402


def to_nc(samples, labels, out="mnist_train_images.nc"):
    cdf5.write_mnist_nc(out, samples, labels)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--input_dir", default=".")
    ap.add_argument("--output_dir", default=".")
    ap.add_argument("--synthetic", action="store_true")
    a = ap.parse_args(argv)
    if a.synthetic:
        (xtr, ytr), (xte, yte) = make_mnist(0)
    else:
        paths = find_idx(a.input_dir)
        if paths is None:
            print(f"no MNIST idx files under {a.input_dir} (expected {sorted(set(IDX_NAMES.values()))}); "
                  "use --synthetic", file=sys.stderr)
            return 1
        xtr, ytr = idx.read_images_labels(paths[("train", "images")], paths[("train", "labels")])
        xte, yte = idx.read_images_labels(paths[("test", "images")], paths[("test", "labels")])
    os.makedirs(a.output_dir, exist_ok=True)
    print("=> ========= Converting Train Images ========= <=")
    p1 = to_nc(xtr, ytr, os.path.join(a.output_dir, "mnist_train_images.nc"))
    print("=> ========= Converting Test Images ========= <=")
    p2 = to_nc(xte, yte, os.path.join(a.output_dir, "mnist_test_images.nc"))
    print(p1, p2)
    return 0


if __name__ == "__main__":
    sys.exit(main())
