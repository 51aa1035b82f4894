"""Decoder HIP kernels on the GPU: attention-mask bits (bit-exact vs torch's own GPU interpolate +
sigmoid + threshold in the same dtype, i.e. the reference's ops on the same device) and masked
attention fwd/bwd vs an fp32 restatement of nn.MultiheadAttention's math (oracle/decoder_ref.py)."""
import math

import numpy as np
import pytest
import torch

from oracle.decoder_ref import pack_bits, ref_attn_bool, ref_masked_attention, unpack_bits

pytestmark = pytest.mark.gpu

DT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}


@pytest.mark.parametrize("dt", ["f32", "f16", "bf16"])
@pytest.mark.parametrize("src,dst", [((64, 64), (8, 8)), ((64, 64), (16, 16)), ((64, 64), (32, 32)),
                                     ((96, 160), (12, 20)), ((50, 70), (13, 17)), ((16, 16), (16, 16))])
def test_attn_mask_bits_exact(device, dt, src, dst):
    from bm2f_amd import decoder_ops
    g = torch.Generator(device=device).manual_seed(1)
    B, Q = 2, 37
    x = torch.randn(B, Q, *src, device=device, generator=g) * 3.0
    # values straddling the threshold in every dtype: +-2^-k and exact zeros
    tiny = torch.tensor([0.0, -0.0, 1e-7, -1e-7, -2e-7, 3e-4, -3e-4, -1e-3, 1e-3, -5e-3], device=device)
    x[0, :5] = tiny[torch.randint(0, len(tiny), (5, *src), device=device, generator=g)]
    x[1, 3] = -5.0          # a fully blocked row -> cleared by the row fix
    x[1, 4] = 5.0
    x = x.to(DT[dt])
    bits = decoder_ops.attn_mask_bits(x, dst)
    want = ref_attn_bool(x, dst)
    got = unpack_bits(bits, dst[0] * dst[1])
    assert torch.equal(got, want), f"{(got != want).sum().item()} mask bits differ"
    assert not got[1, 3].any()
    nofix = unpack_bits(decoder_ops.attn_mask_bits(x, dst, row_fix=False), dst[0] * dst[1])
    assert nofix[1, 3].all()


def test_attn_mask_bits_video_frames(device):
    from bm2f_amd import decoder_ops
    g = torch.Generator(device=device).manual_seed(2)
    x = torch.randn(1, 20, 3, 16, 18, device=device, generator=g)
    for size in [(2, 3), (4, 5), (8, 9)]:
        got = unpack_bits(decoder_ops.attn_mask_bits(x, size), 3 * size[0] * size[1])
        assert torch.equal(got, ref_attn_bool(x, size))


def _attn_case(device, B, Lq, Lk, H, dtype, density, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    C = 32 * H
    q = torch.randn(B, Lq, C, device=device, generator=g).to(dtype)
    k = torch.randn(B, Lk, C, device=device, generator=g).to(dtype)
    v = torch.randn(B, Lk, C, device=device, generator=g).to(dtype)
    blocked = torch.rand(B, Lq, Lk, device=device, generator=g) < density
    blocked[:, 0] = True          # only the first key open
    blocked[:, 0, 0] = False
    blocked[:, 1] = True          # only the last key open
    blocked[:, 1, -1] = False
    blocked[:, 2] = False
    return q, k, v, blocked


@pytest.mark.parametrize("dt,tol", [("f32", 2e-5), ("bf16", 2e-2), ("f16", 4e-3)])
@pytest.mark.parametrize("B,Lq,Lk", [(2, 100, 1024), (2, 100, 64), (1, 37, 4096 + 17), (3, 200, 300),
                                     (1, 128, 700), (1, 129, 700)])
def test_masked_attention(device, dt, tol, B, Lq, Lk):
    from bm2f_amd import decoder_ops
    H = 8
    q, k, v, blocked = _attn_case(device, B, Lq, Lk, H, DT[dt], 0.6, Lq + Lk)
    bits = pack_bits(blocked)
    qa, ka, va = (t.clone().requires_grad_() for t in (q, k, v))
    out = decoder_ops.masked_attention(qa, ka, va, bits, H)
    qr, kr, vr = (t.float().clone().requires_grad_() for t in (q, k, v))
    ref = ref_masked_attention(qr, kr, vr, blocked, H)
    scale = ref.abs().max().item()
    err = (out.float() - ref).abs().max().item() / scale
    assert err < tol, err
    gout = torch.randn_like(ref)
    out.backward(gout.to(out.dtype))
    ref.backward(gout)
    for a, r, name in ((qa, qr, "dq"), (ka, kr, "dk"), (va, vr, "dv")):
        e = (a.grad.float() - r.grad).abs().max().item() / max(r.grad.abs().max().item(), 1e-12)
        assert e < tol * 3, (name, e)


def test_masked_attention_strided_inputs(device):
    """k and v as column slices of one packed projection (row stride 3C), as a fused in-proj yields."""
    from bm2f_amd import decoder_ops
    B, Lq, Lk, H = 2, 100, 512, 8
    C = 32 * H
    g = torch.Generator(device=device).manual_seed(5)
    kv = torch.randn(B, Lk, 3 * C, device=device, generator=g, dtype=torch.bfloat16)
    k, v = kv[..., C:2 * C], kv[..., 2 * C:]
    q = torch.randn(B, Lq, C, device=device, generator=g, dtype=torch.bfloat16)
    blocked = torch.rand(B, Lq, Lk, device=device, generator=g) < 0.5
    out = decoder_ops.masked_attention(q, k, v, pack_bits(blocked), H)
    ref = ref_masked_attention(q, k, v, blocked, H)
    assert (out.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


def test_masked_attention_fully_blocked_row_is_zero(device):
    """Kernel contract: a row with every key blocked yields 0 output and 0 gradient (the reference
    never produces one: its row fix, mask2former_transformer_decoder.py:400)."""
    from bm2f_amd import decoder_ops
    q, k, v, blocked = _attn_case(device, 1, 20, 200, 8, torch.float32, 0.5, 3)
    blocked[:, 5] = True
    qa = q.clone().requires_grad_()
    out = decoder_ops.masked_attention(qa, k, v, pack_bits(blocked), 8)
    assert out[:, 5].abs().max().item() == 0.0
    out.sum().backward()
    assert qa.grad[:, 5].abs().max().item() == 0.0
    assert torch.isfinite(qa.grad).all()


@pytest.mark.parametrize("rows", [262144, 6000])
def test_token_linear_split_k_wgrad(device, rows):
    """The K/V projection over memory tokens: forward == F.linear, weight gradient by split-K bmm within
    bf16 rounding of the fp64 product (one rounding of an fp32 sum, like the library GEMM)."""
    from bm2f_amd import decoder_ops
    torch.manual_seed(rows)
    x = torch.randn(rows, 256, device=device, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(256, 256, device=device) * 0.05).bfloat16().requires_grad_()
    b = torch.randn(256, device=device, dtype=torch.bfloat16, requires_grad=True)
    y = decoder_ops._TokenLinear.apply(x, w, b)
    torch.testing.assert_close(y, torch.nn.functional.linear(x, w, b), rtol=0, atol=0)
    g = torch.randn_like(y)
    y.backward(g)
    ref_w = g.double().t() @ x.double()
    err = ((w.grad.double() - ref_w).abs().max() / ref_w.abs().max()).item()
    assert err < 8e-3, err   # bf16 output rounding (2^-8 relative)
    ref_b = g.double().sum(0)
    assert ((b.grad.double() - ref_b).abs().max() / ref_b.abs().max()).item() < 8e-3
    torch.testing.assert_close(x.grad, g @ w)
