"""Single-process training from PnetCDF-format files (reference: mnist_pnetcdf_cpu.py).

Reads ``./mnist_train_images.nc`` / ``./mnist_test_images.nc`` (CDF-5, written by
``mnist_to_netcdf.py``; synthesised when absent) with the native CDF-5 reader instead of
pncpy/MPI-IO, batch_size=128, epochs=1, and — like upstream — saves no checkpoint unless
``--save_path`` is given (survey Q13).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_ddp_mnist_amd.config import TrainConfig, configure_simple  # noqa: E402
from pytorch_ddp_mnist_amd.data.datasets import MNISTNetCDF  # noqa: E402,F401  (reference API)
from pytorch_ddp_mnist_amd.engine.runner import run  # noqa: E402

DISABLE_TQDM = True

if __name__ == "__main__":
    cfg = configure_simple(base=TrainConfig(batch_size=128, n_epochs=1, device="cpu", data_format="netcdf",
                                            save_path=None), description="MNIST from netCDF, single process")
    run(cfg, entry="mnist_pnetcdf_cpu")
