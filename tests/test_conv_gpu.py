"""x3 fp32 convolutions (csrc/conv_x3.hip, conv_ops.py) against fp64 F.conv2d: forward, input, weight and
bias gradients, for the pixel decoder's conv shapes (msdeformattn.py:213-292) at reduced batch/size."""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

from bm2f_amd import conv_ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("N,Ci,Co,H,W,k,bias", [(2, 256, 256, 32, 32, 3, False), (1, 256, 256, 16, 24, 3, True),
                                                (2, 512, 256, 16, 16, 1, True), (1, 2048, 256, 8, 16, 1, True),
                                                (3, 256, 256, 8, 16, 1, False), (1, 32, 48, 8, 16, 3, True),
                                                (2, 16, 32, 16, 8, 3, True), (1, 48, 16, 128, 8, 3, False)])
@pytest.mark.parametrize("wgrad3", ["x3", "miopen", "tn"])
def test_conv_x3_vs_fp64(device, N, Ci, Co, H, W, k, bias, wgrad3, monkeypatch):
    if k == 1 and wgrad3 == "miopen":
        pytest.skip("the switch only selects the 3x3 weight-gradient engine")
    monkeypatch.setattr(conv_ops, "WGRAD3", wgrad3)
    torch.manual_seed(Ci + Co + H)
    conv = nn.Conv2d(Ci, Co, k, padding=k // 2, bias=bias).to(device)
    x = torch.randn(N, Ci, H, W, device=device, requires_grad=True)
    assert conv_ops.eligible(x, conv)
    y = conv_ops.conv2d(x, conv)
    g = torch.randn_like(y)
    y.backward(g)
    xd = x.detach().double().requires_grad_()
    wd = conv.weight.detach().double().requires_grad_()
    bd = conv.bias.detach().double().requires_grad_() if bias else None
    yd = F.conv2d(xd, wd, bd, padding=k // 2)
    yd.backward(g.double())
    assert _rel(y, yd) < 2e-6
    assert _rel(x.grad, xd.grad) < 2e-6
    assert _rel(conv.weight.grad, wd.grad) < 2e-6
    if bias:
        assert _rel(conv.bias.grad, bd.grad) < 2e-6


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("layout", ["nchw", "channels_last"])
@pytest.mark.parametrize("N,Ci,Co,H,W,bias", [(2, 512, 256, 16, 16, True), (1, 64, 48, 8, 16, False),
                                              (3, 256, 256, 16, 8, True)])
def test_conv_x3_16bit_input_bitwise(device, dtype, layout, N, Ci, Co, H, W, bias):
    """A 16-bit backbone feature into a 1x1 conv (m2f_conv_x3_io / _wgrad_io: read as it is, NCHW or channels-last)
    gives bit for bit what the fp32 kernels give on the reference's ``x.float()``: output, weight and bias gradients
    equal, and the input gradient equals the fp32 one rounded to the feature dtype (the cast's backward), returned
    in the feature's layout."""
    torch.manual_seed(Ci + Co + H + (layout == "nchw"))
    conv = nn.Conv2d(Ci, Co, 1, bias=bias).to(device)
    x16 = torch.randn(N, Ci, H, W, device=device).to(dtype)
    if layout == "channels_last":
        x16 = x16.contiguous(memory_format=torch.channels_last)
    x16.requires_grad_()
    assert conv_ops.eligible(x16, conv)
    y = conv_ops.conv2d(x16, conv)
    g = torch.randn_like(y)
    y.backward(g)
    dw, db = conv.weight.grad.clone(), conv.bias.grad.clone() if bias else None
    conv.zero_grad()
    x32 = x16.detach().float().contiguous().requires_grad_()
    y32 = conv_ops.conv2d(x32, conv)
    y32.backward(g)
    assert y.dtype == torch.float32 and torch.equal(y, y32)
    assert x16.grad.dtype == dtype and torch.equal(x16.grad, x32.grad.to(dtype))
    if layout == "channels_last":
        assert x16.grad.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(dw, conv.weight.grad)
    if bias:
        assert torch.equal(db, conv.bias.grad)


def test_conv_x3_fallback_shapes(device):
    conv = nn.Conv2d(256, 256, 3, padding=1, stride=2).to(device)
    x = torch.randn(1, 256, 16, 16, device=device)
    assert not conv_ops.eligible(x, conv)
    torch.testing.assert_close(conv_ops.conv2d(x, conv), conv(x))


@pytest.mark.parametrize("N,C,h,w,transposed", [(2, 256, 16, 16, True), (1, 8, 5, 6, False), (3, 4, 1, 2, True),
                                                (2, 16, 7, 10, False), (2, 128, 13, 6, True), (1, 64, 3, 256, True),
                                                (1, 64, 2, 7, True)])
def test_upsample2x_add_vs_fp64(device, N, C, h, w, transposed):
    """conv_ops.upsample_add (csrc/upsample.hip) = lateral + F.interpolate(bilinear, align_corners=False) at
    2x, forward and both gradients, against fp64 torch; the coarse map as the encoder's transposed view (C % 64 == 0
    and even w <= 256: the channels-last LDS-tiled kernels, gradient returned channels-last)."""
    torch.manual_seed(N * 100 + h)
    if transposed:   # the last level of the encoder's (N, S, C) output, as forward_features slices it
        z = torch.randn(N, h * w + 5 * 4, C, device=device, requires_grad=True)
        src = z[:, 20:].transpose(1, 2).view(N, C, h, w)
    else:
        z = torch.randn(N, C, h, w, device=device, requires_grad=True)
        src = z
    lat = torch.randn(N, C, 2 * h, 2 * w, device=device, requires_grad=True)
    y = conv_ops.upsample_add(src, lat)
    g = torch.randn_like(y)
    y.backward(g)
    zd = z.detach().double().requires_grad_()
    srcd = zd[:, 20:].transpose(1, 2).reshape(N, C, h, w) if transposed else zd
    latd = lat.detach().double().requires_grad_()
    yd = latd + F.interpolate(srcd, size=(2 * h, 2 * w), mode="bilinear", align_corners=False)
    yd.backward(g.double())
    assert y.is_contiguous()
    assert _rel(y, yd) < 1e-6
    assert _rel(z.grad, zd.grad) < 1e-6
    assert torch.equal(lat.grad, g)
    if transposed and C % 64 == 0 and w % 2 == 0 and w <= 256:   # the channels-last pair: its own layout both ways
        assert conv_ops._nhwc_view(src)
        y2 = conv_ops.upsample_add(src.detach().contiguous(), lat.detach())   # NCHW kernels on the same values
        torch.testing.assert_close(y, y2, rtol=1e-6, atol=1e-6)
    # the library's fp32 result for the same inputs (its NHWC path for the transposed view)
    torch.testing.assert_close(y, lat + F.interpolate(src, size=(2 * h, 2 * w), mode="bilinear",
                                                      align_corners=False), rtol=1e-6, atol=1e-6)


def test_flatten_levels_matches_cat(device):
    """conv_ops.flatten_levels (LDS-tiled transposes) = cat of the transposed levels, values and gradients
    exact (pure data movement), ragged level sizes included."""
    torch.manual_seed(0)
    xs = [torch.randn(3, 40, h, w, device=device, requires_grad=True) for h, w in ((4, 4), (9, 7), (16, 33))]
    ys = [x.detach().clone().requires_grad_() for x in xs]
    a = conv_ops.flatten_levels(xs)
    b = torch.cat([y.flatten(2).transpose(1, 2) for y in ys], 1)
    assert torch.equal(a, b)
    g = torch.randn_like(a)
    a.backward(g)
    b.backward(g)
    for x, y in zip(xs, ys):
        assert torch.equal(x.grad, y.grad)


def test_upsample2x_strided_and_row_kernels_agree(device):
    """m2f_upsample2x_add_fwd_f32 on a transposed view (generic strided kernel) and on its contiguous copy
    (row-window kernel): the same taps and products (the compiler may contract them into FMAs differently,
    so equal to fp32 rounding)."""
    import ctypes
    from bm2f_amd import _native
    torch.manual_seed(1)
    N, C, h, w = 2, 24, 6, 10
    z = torch.randn(N, h * w, C, device=device)
    view = z.transpose(1, 2).view(N, C, h, w)
    cont = view.contiguous()
    lat = torch.randn(N, C, 2 * h, 2 * w, device=device)
    outs = []
    for src in (view, cont):
        out = torch.empty_like(lat)
        _native.call("m2f_upsample2x_add_fwd_f32", src.data_ptr(), *(ctypes.c_int64(s) for s in src.stride()),
                     lat.data_ptr(), out.data_ptr(), N, C, h, w, torch.cuda.current_stream().cuda_stream)
        outs.append(out)
    torch.cuda.synchronize()
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-6, atol=1e-6)
