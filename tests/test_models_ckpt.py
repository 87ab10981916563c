"""Model specs, parameter-slab layout (shared with csrc/kernels/models.h) and model.pt layout (§0.1)."""
import torch

from pytorch_ddp_mnist_amd.models import (CONV_PARAMS, NPARAM, build_model, flatten_state, param_layout,
                                          unflatten_state)
from pytorch_ddp_mnist_amd.ops.native import load_c
from pytorch_ddp_mnist_amd.utils.checkpoint import load_model, save_model

MLP_KEYS = [("0.weight", (128, 784)), ("0.bias", (128,)), ("3.weight", (128, 128)), ("3.bias", (128,)),
            ("5.weight", (10, 128))]
LENET_KEYS = [("0.weight", (6, 1, 5, 5)), ("0.bias", (6,)), ("3.weight", (16, 6, 5, 5)), ("3.bias", (16,)),
              ("7.weight", (120, 400)), ("7.bias", (120,)), ("9.weight", (84, 120)), ("9.bias", (84,)),
              ("11.weight", (10, 84)), ("11.bias", (10,))]


def test_reference_mlp_layout():
    m = build_model("mlp")
    assert [(k, s) for k, s, _ in param_layout(m)] == MLP_KEYS
    assert sum(p.numel() for p in m.parameters()) == NPARAM["mlp"] == 118272
    assert list(m.named_buffers()) == []


def test_lenet_layout():
    m = build_model("lenet5")
    assert [(k, s) for k, s, _ in param_layout(m)] == LENET_KEYS
    assert sum(p.numel() for p in m.parameters()) == NPARAM["lenet5"] == 61706
    assert dict((k, o) for k, _, o in param_layout(m))["7.weight"] == CONV_PARAMS["lenet5"]


def test_native_geometry_matches_python():
    try:
        C = load_c()
    except ImportError:
        import pytest
        pytest.skip("_C not built")
    assert C.model_nparam(0) == NPARAM["mlp"] and C.model_nparam(1) == NPARAM["lenet5"]
    assert C.model_conv_params(1) == CONV_PARAMS["lenet5"] and C.model_conv_params(0) == 0


def test_flatten_roundtrip_and_checkpoint(tmp_path):
    for name in ("mlp", "lenet5"):
        m = build_model(name)
        flat = flatten_state(m)
        sd = unflatten_state(m, flat)
        m2 = build_model(name)
        m2.load_state_dict(sd)
        p = save_model(m2.state_dict(), str(tmp_path / f"{name}.pt"))
        loaded = load_model(p)
        assert list(loaded) == list(m.state_dict())
        for k, v in m.state_dict().items():
            assert loaded[k].dtype == torch.float32 and torch.equal(loaded[k], v)
        ref = build_model(name)
        ref.load_state_dict(torch.load(p, weights_only=True))  # a plain nn.Sequential loads it
