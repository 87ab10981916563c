"""Model zoo: the reference MLP and the LeNet-5 north-star ConvNet.

Each model exists in two forms that share ONE parameter layout:
  * a plain ``torch.nn.Sequential`` (CPU plumbing path, test oracle, and the module whose
    ``state_dict`` is written to ``model.pt``), and
  * the native MI355X trainer, whose flat fp32 master slab holds the same tensors in the same
    order (``csrc/kernels/models.h``), so ``model.pt`` keys/shapes/dtypes are identical
    (survey §0.1: ``0.weight[128,784] 0.bias[128] 3.weight[128,128] 3.bias[128] 5.weight[10,128]``).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
from torch import nn

from .mlp import create_model
from .lenet import create_lenet5

MODEL_IDS = {"mlp": 0, "lenet5": 1}
FACTORIES = {"mlp": create_model, "lenet5": create_lenet5}
NPARAM = {"mlp": 118272, "lenet5": 61706}
CONV_PARAMS = {"mlp": 0, "lenet5": 2572}
# first parameter of backward phase 0 = the late layers, whose gradients backward produces first
# (LeNet: the FC head after the convs; MLP: layers 3.* and 5.* after 0.*) -- csrc model_phase_split
PHASE_SPLIT = {"mlp": 100480, "lenet5": 2572}
# Gradient-producing units in backward-READY order, (name, p0, p1) in the flat slab: the FC layers last to first
# (each one weight-gradient job of the native kernels, csrc model_job_begin), then LeNet's convolutions (conv_bwd).
# Reference gradient-ready order: survey §2.7.  Bucket plans (parallel/ddp.py) group contiguous runs of them.
UNITS = {
    "mlp": [("5.*", 116992, 118272), ("3.*", 100480, 116992), ("0.*", 0, 100480)],
    "lenet5": [("11.*", 60856, 61706), ("9.*", 50692, 60856), ("7.*", 2572, 50692), ("conv", 0, 2572)],
}


def build_model(name: str) -> nn.Module:
    if name not in FACTORIES:
        raise ValueError(f"unknown model {name!r} (choices: {sorted(FACTORIES)})")
    return FACTORIES[name]()


def param_layout(module: nn.Module) -> List[Tuple[str, Tuple[int, ...], int]]:
    """[(state_dict key, shape, flat offset)] in state_dict order."""
    out, off = [], 0
    for k, v in module.state_dict().items():
        out.append((k, tuple(v.shape), off))
        off += v.numel()
    return out


def flatten_state(module: nn.Module) -> torch.Tensor:
    return torch.cat([v.detach().reshape(-1).float().cpu() for v in module.state_dict().values()])


def unflatten_state(module: nn.Module, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
    sd = {}
    flat = flat.detach().float().cpu()
    for k, shape, off in param_layout(module):
        n = 1
        for s in shape:
            n *= s
        sd[k] = flat[off:off + n].view(shape).clone()
    return sd


def flatten_grads(module: nn.Module) -> torch.Tensor:
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).detach().reshape(-1).float()
                      for p in module.parameters()])


__all__ = ["create_model", "create_lenet5", "build_model", "param_layout", "flatten_state",
           "unflatten_state", "flatten_grads", "MODEL_IDS", "NPARAM", "CONV_PARAMS",
           "PHASE_SPLIT", "UNITS"]
