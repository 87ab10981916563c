"""``model.pt`` checkpoints.

Reference: ``torch.save(model.state_dict(), 'model.pt')`` on rank 0 after training, module
unwrapped (ddp_tutorial_multi_gpu.py:118,143-144; ddp_tutorial_cpu.py:110).  Same file, keys,
shapes and fp32 dtype here, written from the native trainer's flat master slab.  Additive:
``save_resume`` / ``load_resume`` keep params + momentum + epoch for ``--resume`` without changing
the default ``model.pt`` layout (survey §5.4).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch


def save_model(state_dict: Dict[str, torch.Tensor], path: str = "model.pt") -> str:
    sd = {k: v.detach().to("cpu", torch.float32).contiguous() for k, v in state_dict.items()}
    tmp = path + ".tmp"
    torch.save(sd, tmp)
    os.replace(tmp, path)
    return path


def load_model(path: str = "model.pt") -> Dict[str, torch.Tensor]:
    """Loads only tensors (``weights_only=True``: nothing in the file is executed)."""
    return torch.load(path, map_location="cpu", weights_only=True)


def save_resume(path: str, params: torch.Tensor, momentum: Optional[torch.Tensor], epoch: int,
                model: str, dtype: str, global_step: int = 0) -> str:
    """``global_step`` seeds the native dropout stream: restoring it keeps the masks of a resumed run
    from replaying those of the first epochs."""
    blob = {"params": params.detach().cpu(), "epoch": int(epoch), "model": model, "dtype": dtype,
            "global_step": int(global_step)}
    if momentum is not None:
        blob["momentum"] = momentum.detach().cpu()
    tmp = path + ".tmp"
    torch.save(blob, tmp)
    os.replace(tmp, path)
    return path


def load_resume(path: str) -> dict:
    return torch.load(path, map_location="cpu", weights_only=True)
