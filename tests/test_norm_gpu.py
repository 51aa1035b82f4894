"""Residual add + LayerNorm kernel (csrc/norm.hip) against an fp64 torch reference of
``LayerNorm(a + b)`` (msdeformattn.py:92-131 post-norm)."""
import pytest
import torch
from torch import nn

from bm2f_amd import _native
from bm2f_amd.norm_ops import AddLayerNorm, add_layernorm

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("rows,C", [(1, 256), (7, 256), (3000, 256), (513, 4), (100, 12), (64, 1024), (65, 260),
                                    (33, 768)])
@pytest.mark.parametrize("with_b", [True, False])
def test_add_layernorm_vs_fp64(device, rows, C, with_b):
    g = torch.Generator(device="cpu").manual_seed(rows * 7 + C)
    a = (torch.randn(rows, C, generator=g) * 3 + 1).to(device).requires_grad_(True)
    b = torch.randn(rows, C, generator=g).to(device).requires_grad_(True) if with_b else None
    norm = nn.LayerNorm(C).to(device)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(C, generator=g))
        norm.bias.copy_(torch.randn(C, generator=g))
    dy = torch.randn(rows, C, generator=g).to(device)

    y = add_layernorm(a, b, norm)
    y.backward(dy)

    ad = a.detach().double().requires_grad_(True)
    bd = b.detach().double().requires_grad_(True) if with_b else None
    wd = norm.weight.detach().double().requires_grad_(True)
    bsd = norm.bias.detach().double().requires_grad_(True)
    yd = torch.nn.functional.layer_norm(ad + bd if with_b else ad, (C,), wd, bsd, norm.eps)
    yd.backward(dy.double())

    assert _rel(y, yd) < 1e-6
    assert _rel(a.grad, ad.grad) < 1e-5
    if with_b:
        assert torch.equal(a.grad, b.grad)
    assert _rel(norm.weight.grad, wd.grad) < 1e-5
    assert _rel(norm.bias.grad, bsd.grad) < 1e-5


def test_add_layernorm_encoder_size_deterministic(device):
    # one encoder layer's rows at config 2 (16 images x 21504 tokens, C = 256); the parameter gradients
    # are reduced in a fixed order, so two runs agree bit for bit
    rows, C = 16 * 21504, 256
    a = torch.randn(rows, C, device=device, requires_grad=True)
    b = torch.randn(rows, C, device=device, requires_grad=True)
    norm = nn.LayerNorm(C).to(device)
    dy = torch.randn(rows, C, device=device)
    outs = []
    for _ in range(2):
        a.grad = b.grad = norm.weight.grad = norm.bias.grad = None
        y = add_layernorm(a, b, norm)
        y.backward(dy)
        outs.append((y.detach().clone(), a.grad.clone(), norm.weight.grad.clone(), norm.bias.grad.clone()))
    for x, z in zip(*outs):
        assert torch.equal(x, z)
    ref = torch.nn.functional.layer_norm(a.detach() + b.detach(), (C,), norm.weight, norm.bias, norm.eps)
    assert _rel(outs[0][0], ref) < 1e-6
    # sum of dgamma-ish check against torch fp32
    a2 = a.detach().clone().requires_grad_(True)
    y2 = torch.nn.functional.layer_norm(a2 + b.detach(), (C,), norm.weight.detach().requires_grad_(True),
                                        norm.bias.detach().requires_grad_(True), norm.eps)
    y2.backward(dy)
    assert _rel(outs[0][1], a2.grad) < 1e-5


def test_add_layernorm_rejects(device):
    x = torch.randn(4, 6, device=device)
    with pytest.raises(RuntimeError, match="C 6"):
        AddLayerNorm.apply(x, None, torch.ones(6, device=device), torch.zeros(6, device=device), 1e-5)
    x = torch.randn(2, 2048, device=device)
    with pytest.raises(RuntimeError, match="C 2048"):
        AddLayerNorm.apply(x, None, torch.ones(2048, device=device), torch.zeros(2048, device=device), 1e-5)


def test_add_layernorm_non_eligible_uses_module(device):
    # fp64 / odd widths stay on the module's own math (same results as the reference's nn.LayerNorm)
    norm = nn.LayerNorm(6).to(device).double()
    a = torch.randn(5, 6, device=device, dtype=torch.float64)
    torch.testing.assert_close(add_layernorm(a, a, norm), norm(a + a))
