"""GroupNorm (+ ReLU) on csrc/gnorm.hip (norm_ops.group_norm_act) against fp64 torch GroupNorm + ReLU:
the pixel decoder's GN layers (msdeformattn.py:216-219, :269-281)."""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

from bm2f_amd.norm_ops import group_norm_act

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("shape,groups", [((2, 256, 16, 16), 32), ((3, 64, 5, 8), 8), ((1, 32, 2, 2), 32),
                                          ((2, 256, 64, 64), 32)])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("affine", [True, False])
def test_group_norm_act_vs_fp64(device, shape, groups, relu, affine):
    torch.manual_seed(shape[1] + groups)
    norm = nn.GroupNorm(groups, shape[1], affine=affine).to(device)
    if affine:
        with torch.no_grad():
            norm.weight.normal_()
            norm.bias.normal_()
    x = (torch.randn(*shape, device=device) * 3 + 1).requires_grad_()
    y = group_norm_act(x, norm, relu)
    g = torch.randn_like(y)
    y.backward(g)
    xd = x.detach().double().requires_grad_()
    wd = norm.weight.detach().double().requires_grad_() if affine else None
    bd = norm.bias.detach().double().requires_grad_() if affine else None
    yd = F.group_norm(xd, groups, wd, bd, norm.eps)
    if relu:
        yd = yd.relu()
    yd.backward(g.double())
    assert _rel(y, yd) < 1e-6
    assert _rel(x.grad, xd.grad) < 1e-5
    if affine:
        assert _rel(norm.weight.grad, wd.grad) < 1e-5
        assert _rel(norm.bias.grad, bd.grad) < 1e-5
    # deterministic: a second run gives the same bits
    x2 = x.detach().clone().requires_grad_()
    y2 = group_norm_act(x2, norm, relu)
    y2.backward(g)
    assert torch.equal(y, y2) and torch.equal(x.grad, x2.grad)


@pytest.mark.parametrize("offset", [100.0, 1000.0])
def test_group_norm_large_mean(device, offset):
    """|mean| >> std: the statistics are fp64 sums of fp64 squares, so the variance does not
    cancel; what is left is the fp32 rounding of x itself and of y = x a + b', which torch's fp32 GroupNorm
    shares -- the bar is "no worse than torch fp32 (+50%)" next to an absolute 1e-4 / 1e-3 vs fp64."""
    torch.manual_seed(7)
    norm = nn.GroupNorm(32, 256).to(device)
    x = (torch.randn(2, 256, 32, 32, device=device) + offset).requires_grad_()
    y = group_norm_act(x, norm, False)
    g = torch.randn_like(y)
    y.backward(g)
    xd = x.detach().double().requires_grad_()
    yd = F.group_norm(xd, 32, norm.weight.double(), norm.bias.double(), norm.eps)
    yd.backward(g.double())
    xt = x.detach().clone().requires_grad_()
    yt = F.group_norm(xt, 32, norm.weight, norm.bias, norm.eps)
    yt.backward(g)
    assert _rel(y, yd) < max(1.5 * _rel(yt, yd), 1e-6) and _rel(y, yd) < 1e-4 * offset / 100
    assert _rel(x.grad, xd.grad) < max(1.5 * _rel(xt.grad, xd.grad), 1e-5) and _rel(x.grad, xd.grad) < 1e-3
