"""Config-driven multi-process training (reference: mnist_cpu_mp.py).

Same CLI as upstream ``configure()``: --wireup_method {nccl-slurm,nccl-openmpi,nccl-mpich,gloo},
--data_path, --data_limit, --batch_size, --n_epochs, --num_workers, --parallel, --hdf5; same
rank-0 banner layout and per-epoch line; rank-0 ``model.pt``.  Fixed upstream quirks: the device
chosen by the wire-up is honoured (Q3: GPUs run the native MI355X trainer with RCCL, CPUs the
torch loop over gloo), no DDP without --parallel (Q4), SLURM/OpenMPI env parsing (Q1/Q2), and
--data_path/--data_limit take effect (Q9).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_ddp_mnist_amd.config import configure  # noqa: E402
from pytorch_ddp_mnist_amd.engine.runner import run  # noqa: E402

if __name__ == "__main__":
    config = configure()
    if config.data_format == "auto":
        config.data_format = "idx"
    run(config, entry="mnist_cpu_mp", show_banner=True)
