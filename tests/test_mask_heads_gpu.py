"""Mask-heads kernel (csrc/mask_heads.hip) on the GPU: the einsum ``bqc,bchw->bqhw`` / ``bqc,btchw->bqthw``
(reference mask2former_transformer_decoder.py:442, video_..._decoder.py:449) within one dtype ulp of the exact
product of the same operands rounded once, and the fused attention bitmask bit-exact against the reference's
resize + sigmoid + threshold + row fix (:446-449, :400 via oracle/decoder_ref.ref_attn_bool) applied to the
kernel's own logits, and against the standalone m2f_attn_mask_bits kernel."""
import pytest
import torch

from oracle.decoder_ref import ref_attn_bool, unpack_bits

pytestmark = pytest.mark.gpu

DT = {"f16": torch.float16, "bf16": torch.bfloat16}
ULP = {"f16": 2.0 ** -10, "bf16": 2.0 ** -7}


def _case(device, B, Q, C, T, H, W, dt, seed=0):
    g = torch.Generator(device=device).manual_seed(seed)
    e = torch.randn(B, Q, C, device=device, generator=g)
    f = torch.randn(B, C, T, H, W, device=device, generator=g) / C ** 0.5
    if Q > 6:
        f[:, 0] = 1.0 / C ** 0.5          # a constant channel: rows that are blocked everywhere
        e[-1, 3] = 0.0
        e[-1, 3, 0] = -40.0               # logits -2.5 everywhere -> a fully blocked row, cleared by the fix
        e[0, 4] = 0.0                     # logits exactly 0: sigmoid 0.5, not blocked
        e[0, 5] *= 1e-3                   # logits straddling 0
        e[0, 6] *= 3e-2
    return e.to(DT[dt]), f.to(DT[dt])


def _fold(f, T):
    from bm2f_amd import decoder_ops
    B, C = f.shape[:2]
    tail = f.shape[3:] if T == 1 else f.shape[2:]
    return decoder_ops.MaskFeatureFold(f, f.reshape(B, C, -1), tuple(tail), lambda df, shape: df.view(shape))


def _check_logits(out, e, f, dt):
    """Within one dtype ulp of the exact (fp64) product of the same operands rounded once.  (An fp32 GEMM
    rounded to the dtype is itself up to 1 ulp off that, so it is not the yardstick: the two may sit 2 ulp
    apart near a binade edge, as measured in round 2.)"""
    B, C = f.shape[:2]
    ref = torch.bmm(e.double(), f.double().reshape(B, C, -1)).to(out.dtype).view(out.shape)
    d = (out.float() - ref.float()).abs()
    bound = ref.float().abs() * ULP[dt] + 1e-6
    assert bool((d <= bound).all()), f"logits beyond 1 ulp: max {d.max().item():.3g}"
    assert (d > 0).float().mean().item() < 0.01


CASES = [  # B, Q, C, T, H, W, target
    (2, 100, 256, 1, 64, 64, (32, 32)),
    (2, 100, 256, 1, 64, 64, (16, 16)),
    (2, 100, 256, 1, 64, 64, (8, 8)),
    (1, 200, 256, 1, 64, 96, (16, 24)),     # 7 query tiles, ragged column chunk
    (2, 37, 64, 1, 40, 48, (5, 6)),         # odd row count with the offset pairing, partial tiles
    (1, 20, 256, 3, 24, 40, (12, 20)),      # video: 3 frames, frame-major keys
    (1, 20, 256, 3, 24, 40, (6, 10)),
    (1, 20, 256, 3, 24, 48, (3, 6)),
    (2, 7, 32, 1, 16, 16, None),            # einsum only
]


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:6])) + f"-{c[6]}")
def test_mask_heads_exact(device, dt, case):
    from bm2f_amd import decoder_ops
    B, Q, C, T, H, W, size = case
    e, f = _case(device, B, Q, C, T, H, W, dt)
    fold = _fold(f, T)
    assert fold.fused_ok(Q, size)
    out, bits = decoder_ops.mask_heads(fold, e, size)
    torch.cuda.synchronize()
    want_shape = (B, Q, H, W) if T == 1 else (B, Q, T, H, W)
    assert out.shape == want_shape and out.dtype == DT[dt]
    _check_logits(out, e, f, dt)
    if size is None:
        assert bits is None
        return
    keys = T * size[0] * size[1]
    got = unpack_bits(bits, keys)
    want = ref_attn_bool(out, size)
    assert torch.equal(got, want), f"{(got != want).sum().item()} mask bits differ"
    assert torch.equal(bits, decoder_ops.attn_mask_bits(out, size))   # tail bits included
    if Q > 6:
        assert not got[-1, 3].any()                # the fully blocked row was cleared
        nofix = ref_attn_bool(out, size, row_fix=False)
        assert nofix[-1, 3].all()


def test_mask_heads_full_size(device):
    """1024^2 input: 256^2 mask features, Q = 100, the three pyramid targets, bf16."""
    from bm2f_amd import decoder_ops
    e, f = _case(device, 2, 100, 256, 1, 256, 256, "bf16", seed=3)
    fold = _fold(f, 1)
    for size in [(32, 32), (64, 64), (128, 128)]:
        out, bits = decoder_ops.mask_heads(fold, e, size)
        _check_logits(out, e, f, "bf16")
        assert torch.equal(unpack_bits(bits, size[0] * size[1]), ref_attn_bool(out, size))


def test_mask_heads_fallback_shapes(device):
    """Shapes the kernel does not take (non-integer ratio, fp32) go through bmm + m2f_attn_mask_bits."""
    from bm2f_amd import decoder_ops
    e, f = _case(device, 1, 10, 32, 1, 50, 70, "bf16")
    fold = _fold(f, 1)
    assert not fold.fused_ok(10, (13, 17))
    out, bits = decoder_ops.mask_heads(fold, e, (13, 17))
    assert torch.equal(unpack_bits(bits, 13 * 17), ref_attn_bool(out, (13, 17)))
    f32 = _fold(f.float(), 1)
    assert not f32.fused_ok(10, (25, 35))


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("B,Q,N", [(2, 100, 4096), (1, 7, 1040), (2, 37, 65536), (1, 128, 2064), (3, 65, 512),
                                   (2, 200, 16384), (1, 129, 1040), (2, 256, 4096), (1, 161, 528), (2, 224, 2064)])
def test_mask_heads_bwd_embed(device, dt, B, Q, N):
    """d embed = G F^T (split over N, fp32 partials summed in a fixed order): within one dtype ulp of the
    exact product rounded once, plus the fp32 accumulation error sqrt(N) 2^-24 sum|g f| that any fp32 GEMM
    has on results that cancel (measured: torch's fp32 bmm is off by more there, tools/dbg_mask_bwd.py)."""
    from bm2f_amd import decoder_ops
    gen = torch.Generator(device=device).manual_seed(Q + N)
    g = torch.randn(B, Q, N, device=device, generator=gen).to(DT[dt])
    f = (torch.randn(B, 256, N, device=device, generator=gen) / 16).to(DT[dt])
    de = decoder_ops.mask_heads_bwd_embed(g, f)
    ref = torch.bmm(g.double(), f.double().transpose(1, 2)).to(DT[dt])
    mag = torch.bmm(g.float().abs(), f.float().abs().transpose(1, 2))
    d = (de.float() - ref.float()).abs()
    bound = ref.float().abs() * ULP[dt] + mag * (N ** 0.5 * 2.0 ** -24) + 1e-6
    assert bool((d <= bound).all()), f"max {d.max().item():.3g}"
    assert decoder_ops._bwd_fusable(f, g)
    assert not decoder_ops._bwd_fusable(f, torch.empty(B, 257, N, device=device, dtype=DT[dt]))  # -> torch.bmm


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("H,B,Q,N,out", [(10, 2, 100, 4096, "f32"), (10, 2, 100, 4096, "same"), (1, 1, 7, 200, "f32"),
                                         (3, 2, 37, 1000, "same"), (16, 1, 20, 520, "f32"), (10, 1, 200, 1040, "f32"),
                                         (2, 1, 256, 264, "same")])
@pytest.mark.parametrize("stage", [4, 1])
def test_mask_heads_bwd_feats(device, dt, H, B, Q, N, out, stage):
    """d feats = sum_h E_h^T G_h over the heads' gradient buffers in place: fp32 output within fp32
    accumulation error of the fp64 sum, dtype output within one ulp of it rounded once; 64 (the default) or 16 G
    rows per LDS stage (stages spanning head boundaries, partial last stages)."""
    from bm2f_amd import _native
    with _native.options(mask_df_stage=stage):
        _bwd_feats_case(device, dt, H, B, Q, N, out)


def _bwd_feats_case(device, dt, H, B, Q, N, out):
    from bm2f_amd import decoder_ops
    gen = torch.Generator(device=device).manual_seed(H * 1000 + N)
    es = [torch.randn(B, Q, 256, device=device, generator=gen).to(DT[dt]) for _ in range(H)]
    gs = [torch.randn(B, Q, N, device=device, generator=gen).to(DT[dt]) for _ in range(H)]
    odt = torch.float32 if out == "f32" else DT[dt]
    assert decoder_ops._fold_fusable(es, gs, odt)
    df = decoder_ops.mask_heads_bwd_feats(es, gs, odt)
    ref = sum(torch.bmm(e.double().transpose(1, 2), g.double()) for e, g in zip(es, gs))
    mag = sum(torch.bmm(e.float().abs().transpose(1, 2), g.float().abs()) for e, g in zip(es, gs))
    acc_err = mag * ((H * Q) ** 0.5 * 2.0 ** -24)
    if out == "f32":
        assert bool(((df.double() - ref).abs() <= acc_err + ref.abs() * 2.0 ** -23 + 1e-6).all())
    else:
        r = ref.to(odt)
        d = (df.float() - r.float()).abs()
        assert bool((d <= r.float().abs() * ULP[dt] + acc_err + 1e-6).all()), f"max {d.max().item():.3g}"


def test_mask_heads_backward_vs_fp64(device):
    """Three heads through the fold (fused forward + the backward kernels) against fp64 autograd of the
    einsums: embed and (fp32) feature gradients."""
    from bm2f_amd import decoder_ops
    e0, f0 = _case(device, 2, 100, 256, 1, 32, 32, "bf16", seed=7)
    e = e0.float().clone().requires_grad_()
    f = f0.float().clone().requires_grad_()
    fold = decoder_ops.MaskFeatureFold(f, f.detach().to(torch.bfloat16).reshape(2, 256, -1), (32, 32),
                                       lambda df, shape: df.view(shape))
    # scales 1, 2, 4: exact in bf16, so the kernels see exactly ed * 2^i
    outs = [decoder_ops.mask_heads(fold, e * 2 ** i, size)[0] for i, size in enumerate([(16, 16), (8, 8), None])]
    gl = [torch.randn_like(o.float()) for o in outs]
    sum((o.float() * gg).sum() for o, gg in zip(outs, gl)).backward()
    ed = e0.double().requires_grad_()
    fd = f0.double().requires_grad_()
    od = [torch.einsum("bqc,bchw->bqhw", ed * 2 ** i, fd[:, :, 0]) for i in range(3)]
    # the kernels see the bf16-rounded incoming gradients, as the reference's autocast GEMMs would
    sum((o * gg.to(torch.bfloat16).double()).sum() for o, gg in zip(od, gl)).backward()
    assert ((e.grad.double() - ed.grad).abs().max() / ed.grad.abs().max()).item() < 1e-2   # bf16 rounding of d embed
    assert ((f.grad.double() - fd.grad).abs().max() / fd.grad.abs().max()).item() < 1e-4


def test_mask_heads_backward(device):
    """Gradients through the fused forward equal those of the bmm-forward fold (same backward)."""
    from bm2f_amd import decoder_ops
    e0, f0 = _case(device, 2, 100, 256, 1, 32, 32, "bf16", seed=5)
    grads = []
    for fused in (True, False):
        e = e0.float().clone().requires_grad_()
        f = f0.float().clone().requires_grad_()
        fold = decoder_ops.MaskFeatureFold(f, f.detach().to(torch.bfloat16).reshape(2, 256, -1), (32, 32),
                                           lambda df, shape: df.view(shape))
        outs = []
        for size in [(16, 16), (8, 8), None]:
            if fused:
                o, _ = decoder_ops.mask_heads(fold, e * (1 + len(outs)), size)
            else:
                o = fold(e * (1 + len(outs)))
            outs.append(o)
        sum((o.float() * (i + 1)).sum() for i, o in enumerate(outs)).backward()
        grads.append((e.grad, f.grad, [o.detach() for o in outs]))
    (ge1, gf1, o1), (ge2, gf2, o2) = grads
    for a, b in zip(o1, o2):
        assert ((a.float() - b.float()).abs() <= b.float().abs() * 2 * ULP["bf16"] + 1e-6).all()   # 1 ulp each
    assert torch.equal(ge1, ge2)
    assert torch.equal(gf1, gf2)
