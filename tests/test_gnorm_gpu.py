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
