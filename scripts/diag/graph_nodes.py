"""The captured single-step graph of the LeNet step (schedules concurrent and serial): node types and edges as the
runtime holds them (hipGraphNodeType: 0 kernel, 1 memcpy, 2 memset, 3 host, 4 graph, 5 empty, 6 wait event,
7 event record).  Usage: python scripts/diag/graph_nodes.py [--batch 8192] [--dtype bf16]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8192)
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--model", default="lenet5")
a = ap.parse_args()
x, y = make_split(a.batch * 3, seed=1)
tr = NativeTrainer(a.model, a.dtype, a.batch, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y),
                   init=build_model(a.model))
tr.set_epoch_indices(torch.arange(a.batch * 3, dtype=torch.int32))
for conc in (True, False):
    tr.apply_plan(dict(concurrent=conc))
    tr.prepare_graphs(k=1)
    print(f"concurrent={conc}:", flush=True)
    for line in tr.rt.graph_nodes():
        print("   " + line, flush=True)
tr.close()
