"""The benchmark backbone's fused bias(+shortcut)+ReLU (csrc/eltwise.hip) against the unfused torch ops."""
import pytest
import torch
import torch.nn.functional as F

from bm2f_amd.bench_model import bias_act

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
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


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("nout,unused", [(2, None), (3, None), (3, 1)])
def test_bias_act_fork_sums_consumer_grads(device, dtype, nout, unused):
    """bias_act(..., nout): one handle per consumer; the backward (m2f_relu_bwd_sum) gives sum_k g_k * (y > 0)
    with the sum formed in fp32 in consumer order and rounded once (bit-exact against that torch sum), to x
    and the residual; an unused handle contributes nothing."""
    torch.manual_seed(nout)
    x = torch.randn(2, 64, 16, 24, device=device, dtype=dtype)
    r = torch.randn_like(x)
    b = torch.randn(64, device=device)
    xa, ra = x.clone().requires_grad_(), r.clone().requires_grad_()
    hs = bias_act(xa.clone(), b, ra, nout)
    assert len(hs) == nout and all(h.data_ptr() == hs[0].data_ptr() for h in hs)
    gs = [torch.randn_like(hs[0]) for _ in range(nout)]
    loss = sum((h.float() * g.float()).sum() for k, (h, g) in enumerate(zip(hs, gs)) if k != unused)
    loss.backward()
    y = hs[0].detach()
    tot = None
    for k, g in enumerate(gs):
        if k != unused:
            tot = g.float() if tot is None else tot + g.float()
    want = torch.where(y > 0, tot, torch.zeros_like(tot)).to(dtype)
    torch.testing.assert_close(xa.grad, want, rtol=0, atol=0)
    torch.testing.assert_close(ra.grad, want, rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("H,W", [(16, 24), (7, 9), (1, 1), (2, 3), (5, 16), (1, 8)])
def test_stem_maxpool_matches_torch(device, dtype, H, W):
    """The stem max pool (csrc/eltwise.hip, 1-byte winners) against F.max_pool2d(3, 2, 1): forward and
    gradient bit-exact, with ties (integer-valued inputs), -inf and NaN."""
    from bm2f_amd.bench_model import max_pool_stem
    torch.manual_seed(H * 31 + W)
    x = torch.randint(-3, 4, (2, 5, H, W), device=device).to(dtype)     # many ties
    x.view(-1)[::7] = float("-inf")
    if H * W > 4:
        x.view(-1)[5] = float("nan")
    xa = x.clone().requires_grad_()
    xb = x.clone().requires_grad_()
    ya = max_pool_stem(xa)
    yb = F.max_pool2d(xb, kernel_size=3, stride=2, padding=1)
    assert torch.equal(ya.isnan(), yb.isnan())
    assert torch.equal(ya.nan_to_num(), yb.nan_to_num())
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    assert torch.equal(xa.grad, xb.grad)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,W,C", [(16, 24, 64), (7, 9, 8), (1, 1, 16), (5, 16, 24)])
def test_stem_maxpool_nhwc_matches_torch(device, dtype, H, W, C):
    """The channels-last stem max pool (m2f_maxpool3s2_nhwc) against F.max_pool2d(3, 2, 1) on the same
    channels-last tensor: forward and gradient bit-exact (ties, -inf, NaN), output and gradient channels-last."""
    from bm2f_amd.bench_model import max_pool_stem
    torch.manual_seed(H * 31 + W + C)
    x = torch.randint(-3, 4, (2, C, H, W), device=device).to(dtype)
    x.view(-1)[::7] = float("-inf")
    if H * W > 4:
        x.view(-1)[5] = float("nan")
    x = x.contiguous(memory_format=torch.channels_last)
    xa = x.clone(memory_format=torch.channels_last).requires_grad_()
    xb = x.clone(memory_format=torch.channels_last).requires_grad_()
    ya = max_pool_stem(xa)
    yb = F.max_pool2d(xb, kernel_size=3, stride=2, padding=1)
    assert ya.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(ya.isnan(), yb.isnan())
    assert torch.equal(ya.nan_to_num(), yb.nan_to_num())
    g = torch.randn_like(yb)
    ya.backward(g)
    yb.backward(g)
    assert xa.grad.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(xa.grad, xb.grad)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_bias_act_nan_follows_torch(device, dtype):
    """NaN activations: the forward propagates them as torch's relu does, and the multi-consumer backward
    (m2f_relu_bwd_sum) passes the gradient where y is NaN, as torch's threshold_backward (y <= 0 -> 0)."""
    torch.manual_seed(1)
    x = torch.randn(2, 64, 16, 24, device=device, dtype=dtype)
    x.view(-1)[::97] = float("nan")
    b = torch.randn(64, device=device)
    xa = x.clone().requires_grad_()
    hs = bias_act(xa.clone(), b, None, 2)
    want_y = F.relu(x.float() + b.view(1, -1, 1, 1)).to(dtype)
    assert torch.equal(hs[0].isnan(), want_y.isnan())
    torch.testing.assert_close(hs[0].nan_to_num(), want_y.nan_to_num(), rtol=0, atol=0)
    gs = [torch.randn_like(hs[0]) for _ in range(2)]
    sum((h.float() * g.float()).sum() for h, g in zip(hs, gs)).backward()
    tot = gs[0].float() + gs[1].float()
    want = torch.ops.aten.threshold_backward(tot, want_y.float(), 0).to(dtype)
    torch.testing.assert_close(xa.grad, want, rtol=0, atol=0)
