"""The benchmark backbone's fused bias(+shortcut)+ReLU (csrc/eltwise.hip) against the unfused torch ops."""
import pytest
import torch
import torch.nn.functional as F

from bm2f_amd.bench_model import bias_act

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("residual", [False, True])
def test_bias_act_matches_unfused(device, dtype, residual):
    torch.manual_seed(0)
    x = torch.randn(2, 64, 16, 24, device=device, dtype=dtype)
    r = torch.randn_like(x) if residual else None
    b = torch.randn(64, device=device)
    want = x.float() + b.view(1, -1, 1, 1) + (r.float() if residual else 0)
    want = F.relu(want).to(dtype)
    xa = x.clone().requires_grad_()
    ra = r.clone().requires_grad_() if residual else None
    got = bias_act(xa.clone(), b, ra)
    torch.testing.assert_close(got, want, rtol=0, atol=0)
    g = torch.randn_like(got)
    got.backward(g)
    mask = want > 0
    torch.testing.assert_close(xa.grad, torch.where(mask, g, torch.zeros_like(g)))
    if residual:
        torch.testing.assert_close(ra.grad, torch.where(mask, g, torch.zeros_like(g)))
