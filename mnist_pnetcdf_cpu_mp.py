"""Multi-process training from PnetCDF-format files (reference: mnist_pnetcdf_cpu_mp.py).

CLI of ``mnist_cpu_mp.py`` plus the ``mpich`` wire-up (PMI_RANK/PMI_SIZE; upstream's c10d "mpi"
backend does not exist in stock PyTorch, survey Q6, so it maps to the same RCCL / gloo data plane).
Every rank reads the CDF-5 files with the native reader (header parsed once, bulk pread into
pinned memory, one async copy into HBM on a GPU).  Launch without MPI via
``python -m pytorch_ddp_mnist_amd.parallel.launch -n 4 -- python3 mnist_pnetcdf_cpu_mp.py --parallel --wireup_method mpich``.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_ddp_mnist_amd.config import configure  # noqa: E402
from pytorch_ddp_mnist_amd.data.datasets import MNISTNetCDF  # noqa: E402,F401  (reference API)
from pytorch_ddp_mnist_amd.engine.runner import run  # noqa: E402

if __name__ == "__main__":
    config = configure(pnetcdf=True)
    if config.data_format == "auto":
        config.data_format = "netcdf"
    run(config, entry="mnist_pnetcdf_cpu_mp", show_banner=True)
