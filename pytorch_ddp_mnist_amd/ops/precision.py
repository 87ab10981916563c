"""What an fp32 training step actually computes its products with (bench JSON ``config.fp32_products``).

The fp32 path is not uniformly ``v_mfma_f32_16x16x4_f32``: where it measured faster, a product runs as the EXACT
3-part bf16 split of csrc/kernels/common.h ``Mma<float>`` (each fp32 operand cut into hi + mid + lo bf16 parts, the
six partial products of weight >= 2^-16 on three ``v_mfma_f32_16x16x32_bf16``; ~2^-24 relative error, fp32-like,
every fp32 tolerance test passes).  This mirrors the launchers' choices so a result line says which is which:

* LeNet-5 conv1 / conv2 forward: split (lenet.hip conv_fwd_images, ``MNIST_AMD_F32_C2SPLIT`` on by default);
* the FC head's layer products: split on >= 32-row tiles, i.e. batches above ``L1_SPLIT_MAX_B`` (head.hip
  ``head_mma<T, true>``); at smaller batches the layer-1 split-K kernel + 16-row head run exact fp32;
* the FC weight gradient: split for LeNet and, from B = 4096, for the MLP (head.hip ``wg_mma`` / ``wgrad_launch``),
  exact where it is the SGD-fused one-split kernel of small batches (``wgrad_sgd_tile``);
* LeNet conv_bwd (conv dgrad + conv weight gradients): exact fp32 MFMA.

Reference precision: fp32 everywhere, no autocast (/root/reference/ddp_tutorial_multi_gpu.py:75; survey §0.1).
"""
from __future__ import annotations

from typing import Dict, List

L1_SPLIT_MAX_B = 1024      # csrc/kernels/launch.h
SPLIT_ERROR = "exact 3-part bf16 split: six partial products of weight >= 2^-16, ~2^-24 relative (common.h Mma<float>)"


def fc_splits(batch: int, kc: int = 16) -> int:
    """FC weight-gradient batch splits of the native trainer (engine/native.py default, fp32 K-chunk 16)."""
    bp = -(-batch // kc) * kc
    return max(1, min(16, bp // 512))


def fp32_products(model: str, batch: int, split_build: int = 0) -> Dict[str, List[str]]:
    """{"bf16x3_split": [...], "exact_fp32_mfma": [...], "split_error": str} for an fp32 step of ``batch`` rows."""
    if split_build:  # opt-in -DMNIST_AMD_F32_SPLIT build: every fp32 product
        return {"bf16x3_split": ["every fp32 product (opt-in MNIST_AMD_F32_SPLIT build)"], "exact_fp32_mfma": [],
                "split_error": SPLIT_ERROR}
    split, exact = [], []
    if model == "lenet5":
        split += ["conv1 forward", "conv2 forward"]
        exact += ["conv_bwd (conv dgrad + conv weight gradients)"]
    head = "FC head layer products (forward + dgrad)"
    (split if batch > L1_SPLIT_MAX_B else exact).append(head + (" (>= 32-row tiles)" if batch > L1_SPLIT_MAX_B else
                                                                 " (layer-1 split-K kernel + 16-row tiles)"))
    fused = fc_splits(batch) == 1
    wg_split = (model == "lenet5" or batch >= 4096) and not fused
    (split if wg_split else exact).append("FC weight gradient" + (" (SGD-fused one-split kernel)" if fused else ""))
    return {"bf16x3_split": split, "exact_fp32_mfma": exact, "split_error": SPLIT_ERROR}


def dtype_label(dtype: str, model: str, batch: int, split_build: int = 0) -> str:
    """The bench JSON ``dtype``: the compute dtype, plus, for fp32, which products are bf16 splits."""
    if dtype != "fp32":
        return dtype
    p = fp32_products(model, batch, split_build)
    if not p["bf16x3_split"]:
        return "fp32"
    return "fp32 (" + ", ".join(p["bf16x3_split"]) + " as exact 3-part bf16 splits)"
