"""Single-process training (reference: ddp_tutorial_cpu.py; launcher train_cpu.sh).

Same defaults as upstream — MLP, batch_size=128, epochs=1, SGD(lr=0.01), CPU, writes model.pt —
and the same per-epoch line.  Data: ./mnist_data idx files (synthesised in the same layout when
absent: no network).  Additive flags (``--model lenet5 --device cuda --dtype bf16`` ...) route the
same loop through the native MI355X trainer.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_ddp_mnist_amd.config import TrainConfig, configure_simple  # noqa: E402
from pytorch_ddp_mnist_amd.engine.runner import run  # noqa: E402
from pytorch_ddp_mnist_amd.models import create_model  # noqa: E402,F401  (reference API)

DISABLE_TQDM = True

if __name__ == "__main__":
    batch_size = 128
    epochs = 1
    cfg = configure_simple(base=TrainConfig(batch_size=batch_size, n_epochs=epochs, device="cpu", data_format="idx"),
                           description="MNIST MLP, single process")
    run(cfg, entry="ddp_tutorial_cpu")
