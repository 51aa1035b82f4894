"""MaskFeatureFold: every head's mask einsum against one feature map, with the features' gradient summed
over the heads by one GEMM (decoder_ops.py).  Checked against an fp64 sum of per-head einsums
(mask2former_transformer_decoder.py:442 / video :449 semantics)."""
import pytest
import torch

from bm2f_amd import decoder_ops


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _run(device, dtype, video, heads=4, B=2, C=48, T=3, H=12, W=10, Q=30, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    fshape = (B, T, C, H, W) if video else (B, C, H, W)
    f = torch.randn(fshape, generator=g).to(device).requires_grad_(True)
    es = [torch.randn(B, Q, C, generator=g).to(device).requires_grad_(True) for _ in range(heads)]
    oshape = (B, Q, T, H, W) if video else (B, Q, H, W)
    gs = [torch.randn(oshape, generator=g).to(device=device, dtype=dtype) for _ in range(heads)]
    f_lp = f.detach().to(dtype)
    if video:
        lp = f_lp.transpose(1, 2).reshape(B, C, T * H * W)
        fold = decoder_ops.MaskFeatureFold(
            f, lp, (T, H, W), lambda df, s: df.view(s[0], s[2], s[1], s[3], s[4]).transpose(1, 2))
    else:
        fold = decoder_ops.image_mask_fold(f, f_lp)
    outs = [fold(e) for e in es]
    torch.autograd.backward(outs, gs)

    # fp64 reference on the same rounded operands
    fr = f_lp.double()
    eq = "bqc,btchw->bqthw" if video else "bqc,bchw->bqhw"
    geq_f = "bqc,bqthw->btchw" if video else "bqc,bqhw->bchw"
    geq_e = "bqthw,btchw->bqc" if video else "bqhw,bchw->bqc"
    want_out = [torch.einsum(eq, e.detach().to(dtype).double(), fr) for e in es]
    want_df = sum(torch.einsum(geq_f, e.detach().to(dtype).double(), gg.double()) for e, gg in zip(es, gs))
    want_de = [torch.einsum(geq_e, gg.double(), fr) for gg in gs]
    return outs, f.grad, [e.grad for e in es], want_out, want_df, want_de


@pytest.mark.parametrize("video", [False, True])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
def test_fold_cpu(video, dtype, tol):
    outs, df, des, wo, wdf, wde = _run("cpu", dtype, video)
    assert df.dtype == torch.float32 and df.shape == wdf.shape
    assert _rel(df, wdf) < tol
    for o, w in zip(outs, wo):
        assert o.dtype == dtype and _rel(o, w) < tol
    for d, w in zip(des, wde):
        assert d.dtype == torch.float32 and _rel(d, w) < tol


def test_fold_no_grad_features():
    f = torch.randn(1, 8, 4, 4)                     # no requires_grad: no gate, einsums still work
    e = torch.randn(1, 5, 8, requires_grad=True)
    fold = decoder_ops.image_mask_fold(f)
    assert fold.token is None
    out = fold(e)
    out.sum().backward()
    torch.testing.assert_close(out, torch.einsum("bqc,bchw->bqhw", e, f))
    assert e.grad is not None


def test_fold_unused_heads():
    # a head whose output does not reach the loss contributes nothing; the rest still sum correctly
    f = torch.randn(2, 8, 5, 6, requires_grad=True)
    es = [torch.randn(2, 3, 8, requires_grad=True) for _ in range(3)]
    fold = decoder_ops.image_mask_fold(f)
    outs = [fold(e) for e in es]
    (outs[0].sum() + 2 * outs[2].sum()).backward()
    ones = torch.ones(2, 3, 5, 6)
    want = torch.einsum("bqc,bqhw->bchw", es[0].detach(), ones) + torch.einsum("bqc,bqhw->bchw", es[2].detach(), 2 * ones)
    torch.testing.assert_close(f.grad, want)
    assert es[1].grad is None


@pytest.mark.gpu
@pytest.mark.parametrize("video", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_fold_gpu_lowp(device, video, dtype):
    # fp32-output GEMM over the stacked heads: one rounding, so tighter than the per-head bf16 sum
    outs, df, des, wo, wdf, wde = _run(device, dtype, video, heads=10, Q=100, C=64, H=32, W=24)
    assert df.dtype == torch.float32
    assert _rel(df.cpu(), wdf) < 1e-5
    for o, w in zip(outs, wo):
        assert _rel(o.cpu(), w) < 1e-2
    for d, w in zip(des, wde):
        assert _rel(d.cpu(), w) < 1e-2
