"""The fp32 precision statement of the bench JSON (ops/precision.py): which products of an fp32 step run as exact
3-part bf16 splits (verdict r5 item 6).  The rules mirror the launchers: lenet.hip conv_fwd_images (conv1 / conv2
forward split), head.hip head_launch_t (split head products at >= 32-row tiles, above L1_SPLIT_MAX_B), wgrad_launch
(split weight gradients: LeNet always, MLP from B = 4096; the SGD-fused one-split kernel exact)."""
from pytorch_ddp_mnist_amd.ops.precision import dtype_label, fc_splits, fp32_products


def test_lenet_headline_fp32():
    p = fp32_products("lenet5", 8192)
    assert "conv1 forward" in p["bf16x3_split"] and "conv2 forward" in p["bf16x3_split"]
    assert any("FC head" in s for s in p["bf16x3_split"]) and any("weight gradient" in s for s in p["bf16x3_split"])
    assert any("conv_bwd" in s for s in p["exact_fp32_mfma"])
    lab = dtype_label("fp32", "lenet5", 8192)
    assert lab.startswith("fp32 (") and "3-part bf16" in lab and "conv1 forward" in lab
    assert "2^-24" in p["split_error"]


def test_small_batches_are_exact_where_the_kernels_are():
    p = fp32_products("lenet5", 128)  # 16-row head + l1 split kernel, SGD-fused one-split FC wgrad
    assert fc_splits(128) == 1
    assert not any("FC" in s for s in p["bf16x3_split"])
    assert any("FC head" in s for s in p["exact_fp32_mfma"]) and any("weight gradient" in s for s in p["exact_fp32_mfma"])
    m = fp32_products("mlp", 128)
    assert m["bf16x3_split"] == [] and dtype_label("fp32", "mlp", 128) == "fp32"
    m = fp32_products("mlp", 2048)  # split head tiles, exact MLP weight gradient below 4096
    assert any("FC head" in s for s in m["bf16x3_split"]) and any("weight gradient" in s for s in m["exact_fp32_mfma"])
    m = fp32_products("mlp", 8192)
    assert any("weight gradient" in s for s in m["bf16x3_split"])


def test_bf16_and_split_build_labels():
    assert dtype_label("bf16", "lenet5", 8192) == "bf16"
    p = fp32_products("mlp", 128, split_build=3)
    assert p["exact_fp32_mfma"] == [] and "every fp32 product" in p["bf16x3_split"][0]
