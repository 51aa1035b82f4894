"""MSDA HIP kernels vs the oracle and the reference's golden vectors (runs on the GPU box).

Mirrors the reference's own checks (ops/test.py): fp64 equality with allclose defaults (:34-47),
fp32 within tolerance (:50-63; we hold rtol 1e-3 per the north star) and gradcheck over the channel
widths {30,32,64,71,1025,2048,3096} (:66-89) that exercised every reference backward branch.
"""
import numpy as np
import pytest
import torch

from conftest import check_crossing_entries, golden, loc_crossing_mask
from oracle import msda_ref

pytestmark = pytest.mark.gpu


def _t(a, device, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(device)
    return t.to(dtype) if dtype is not None else t


def _close(got, want, rtol=1e-3, atol_frac=1e-5):
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    scale = max(np.abs(want).max(), 1e-30)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol_frac * scale)


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_testpy_fixture(device, tag):
    from bm2f_amd.msda import MSDeformAttnFunction
    g = golden("msda_testpy.npz")
    shapes, lsi = _t(g["shapes"], device), _t(g["level_start_index"], device)
    v, loc, a = (_t(g[f"{tag}_{k}"], device).requires_grad_() for k in ("value", "loc", "attn"))
    out = MSDeformAttnFunction.apply(v, shapes, lsi, loc, a, 2)
    if tag == "f64":
        assert torch.allclose(out.cpu(), torch.from_numpy(g["f64_out"]))  # test.py:44
    else:
        assert torch.allclose(out.cpu(), torch.from_numpy(g["f32_out"]), rtol=1e-3, atol=1e-6)
    out.backward(_t(g[f"{tag}_grad_out"], device))
    rtol = 1e-9 if tag == "f64" else 1e-3
    _close(v.grad.cpu(), g[f"{tag}_grad_value"], rtol)
    _close(loc.grad.cpu(), g[f"{tag}_grad_loc"], rtol)
    _close(a.grad.cpu(), g[f"{tag}_grad_attn"], rtol)


@pytest.mark.parametrize("variant", ["uniform", "local"])
@pytest.mark.parametrize("host_shapes", [False, True])
def test_slice_fixture(device, variant, host_shapes):
    from bm2f_amd.msda import MSDeformAttnFunction, attach_host_shapes
    g = golden("msda_slice.npz")
    shapes, lsi = _t(g["shapes"], device), _t(g["level_start_index"], device)
    if host_shapes:
        attach_host_shapes(shapes, g["shapes"].tolist())
    v, loc, a = (_t(g[f"{variant}_{k}"], device).requires_grad_() for k in ("value", "loc", "attn"))
    out = MSDeformAttnFunction.apply(v, shapes, lsi, loc, a, 64)
    _close(out.detach().cpu(), g[f"{variant}_out"])
    out.backward(_t(g[f"{variant}_grad_out"], device))
    _close(v.grad.cpu(), g[f"{variant}_grad_value"])
    _close(a.grad.cpu(), g[f"{variant}_grad_attn"])
    _close(loc.grad.cpu(), g[f"{variant}_grad_loc"], atol_frac=1e-4)


def _random_case(N, Lq, M, D, shapes, P, dtype, device, seed, spread=1.2):
    gen = torch.Generator().manual_seed(seed)
    shapes_t = torch.tensor(shapes, dtype=torch.int64)
    lsi = torch.cat((shapes_t.new_zeros(1), shapes_t.prod(1).cumsum(0)[:-1]))
    S = int(shapes_t.prod(1).sum())
    L = len(shapes)
    value = torch.randn(N, S, M, D, generator=gen, dtype=torch.float64)
    loc = torch.rand(N, Lq, M, L, P, 2, generator=gen, dtype=torch.float64) * spread - (spread - 1) / 2
    attn = torch.rand(N, Lq, M, L, P, generator=gen, dtype=torch.float64)
    gout = torch.randn(N, Lq, M * D, generator=gen, dtype=torch.float64)
    cast = lambda t: t.to(dtype).contiguous()  # noqa: E731
    return [cast(x) for x in (value, loc, attn, gout)], shapes_t, lsi


@pytest.mark.parametrize("D", [16, 32, 64, 8, 30])
@pytest.mark.parametrize("P", [4, 3])
def test_fp32_vs_oracle(device, D, P):
    from bm2f_amd import msda
    (v, loc, a, gout), shapes, lsi = _random_case(2, 37, 3, D, [(7, 5), (4, 3), (2, 2)], P, torch.float32, device, D * 10 + P)
    out = msda.ms_deform_attn_forward(v.to(device), shapes.to(device), lsi.to(device), loc.to(device), a.to(device), 64)
    want = msda_ref.msda_forward(v.double(), shapes, lsi, loc.double(), a.double())
    _close(out.cpu(), want)
    gv, gl, ga = msda.ms_deform_attn_backward(v.to(device), shapes.to(device), lsi.to(device), loc.to(device),
                                             a.to(device), gout.to(device), 64)
    wv, wl, wa = msda_ref.msda_backward(v.double(), shapes, lsi, loc.double(), a.double(), gout.double())
    _close(gv.cpu(), wv)
    _close(ga.cpu(), wa)
    _close(gl.cpu(), wl, atol_frac=1e-4)


@pytest.mark.parametrize("channels", [30, 32, 64, 71, 1025, 2048, 3096])
def test_gradcheck_channels(device, channels):
    """ops/test.py:66-89 — gradcheck in fp64 at the reference's toy shape for every width."""
    from bm2f_amd.msda import MSDeformAttnFunction
    N, M, Lq, L, P = 1, 2, 2, 2, 2
    shapes = torch.as_tensor([(6, 4), (3, 2)], dtype=torch.long, device=device)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = 30
    torch.manual_seed(3)
    value = (torch.rand(N, S, M, channels) * 0.01).double().to(device).requires_grad_()
    loc = torch.rand(N, Lq, M, L, P, 2).double().to(device).requires_grad_()
    attn = torch.rand(N, Lq, M, L, P) + 1e-5
    attn = (attn / attn.sum(-1, keepdim=True).sum(-2, keepdim=True)).double().to(device).requires_grad_()
    assert torch.autograd.gradcheck(MSDeformAttnFunction.apply, (value, shapes, lsi, loc, attn, 2))
    # and the analytic gradients agree with the oracle
    out = MSDeformAttnFunction.apply(value, shapes, lsi, loc, attn, 2)
    gout = torch.rand_like(out)
    out.backward(gout)
    wv, wl, wa = msda_ref.msda_backward(value.detach().cpu(), shapes.cpu(), lsi.cpu(), loc.detach().cpu(),
                                        attn.detach().cpu(), gout.cpu())
    _close(value.grad.cpu(), wv, rtol=1e-9)
    _close(loc.grad.cpu(), wl, rtol=1e-9)
    _close(attn.grad.cpu(), wa, rtol=1e-9)


def test_errors_like_reference(device):
    from bm2f_amd import msda
    (v, loc, a, gout), shapes, lsi = _random_case(3, 5, 2, 32, [(4, 4), (2, 2)], 4, torch.float32, device, 1)
    dv, ds, dl, dloc, da = (t.to(device) for t in (v, shapes, lsi, loc, a))
    with pytest.raises(RuntimeError, match="contiguous"):
        msda.ms_deform_attn_forward(dv.transpose(1, 2), ds, dl, dloc, da, 64)
    with pytest.raises(RuntimeError, match="CUDA tensor"):
        msda.ms_deform_attn_forward(v, ds, dl, dloc, da, 64)
    with pytest.raises(RuntimeError, match="im2col_step"):
        msda.ms_deform_attn_forward(dv, ds, dl, dloc, da, 2)  # batch 3 % min(3,2) != 0
    with pytest.raises(RuntimeError, match="not implemented"):
        msda.ms_deform_attn_forward(dv.half(), ds, dl, dloc.half(), da.half(), 64)


def test_full_size_properties(device):
    """Config-2 sized layer (N=16, 1024^2 pyramid): linearity in value and attn, and a sum check."""
    from bm2f_amd import msda
    shapes = [(32, 32), (64, 64), (128, 128)]
    N, M, D, L, P = 4, 8, 32, 3, 4
    st = torch.tensor(shapes, dtype=torch.int64, device=device)
    lsi = torch.cat((st.new_zeros(1), st.prod(1).cumsum(0)[:-1]))
    msda.attach_host_shapes(st, shapes)
    S = int(st.prod(1).sum())
    g = torch.Generator(device=device).manual_seed(0)
    v1 = torch.randn(N, S, M, D, device=device, generator=g)
    v2 = torch.randn(N, S, M, D, device=device, generator=g)
    loc = torch.rand(N, S, M, L, P, 2, device=device, generator=g)
    a = torch.rand(N, S, M, L, P, device=device, generator=g)
    o1 = msda.ms_deform_attn_forward(v1, st, lsi, loc, a, 64)
    o2 = msda.ms_deform_attn_forward(v2, st, lsi, loc, a, 64)
    o12 = msda.ms_deform_attn_forward(v1 + v2, st, lsi, loc, a, 64)
    torch.testing.assert_close(o12, o1 + o2, rtol=1e-4, atol=1e-4)
    # <grad_out, fwd(v)> == <bwd_value(grad_out), v>  (the backward is the adjoint of the forward in v)
    gout = torch.randn_like(o1)
    gv, gl, ga = msda.ms_deform_attn_backward(v1, st, lsi, loc, a, gout, 64)
    lhs = (gout.double() * o1.double()).sum()
    rhs = (gv.double() * v1.double()).sum()
    assert abs((lhs - rhs) / lhs).item() < 1e-4
    # <grad_attn, a> == <grad_out, out> (the forward is linear in attn too)
    rhs_a = (ga.double() * a.double()).sum()
    assert abs((lhs - rhs_a) / lhs).item() < 1e-4


def _pyramid_case(shapes, N, M, far_frac, seed):
    """Encoder-like inputs: query i = pyramid position i, samples near the reference point plus a
    fraction far away (exercising the out-of-window path of the tiled backward)."""
    gen = torch.Generator().manual_seed(seed)
    st = torch.tensor(shapes, dtype=torch.int64)
    lsi = torch.cat((st.new_zeros(1), st.prod(1).cumsum(0)[:-1]))
    S = int(st.prod(1).sum())
    L, P, D = len(shapes), 4, 32
    refs = []
    for h, w in shapes:
        ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h), torch.linspace(0.5, w - 0.5, w), indexing="ij")
        refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
    ref = torch.cat(refs, 0)
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)
    off = torch.randn(N, S, M, L, P, 2, generator=gen) * 2.0
    loc = ref[None, :, None, None, None, :] + off / norm[None, None, None, :, None, :]
    far = torch.rand(N, S, M, L, P, 1, generator=gen) < far_frac
    loc = torch.where(far, torch.rand(N, S, M, L, P, 2, generator=gen) * 1.2 - 0.1, loc)
    value = torch.randn(N, S, M, D, generator=gen)
    attn = torch.rand(N, S, M, L, P, generator=gen)
    gout = torch.randn(N, S, M * D, generator=gen)
    return value, st, lsi, loc.contiguous(), attn, gout


@pytest.mark.parametrize("tile,rows,halo", [(16, 2304, 8), (12, 2304, 8), (8, 480, 8), (4, 64, 2), (8, 200, 0),
                                           (6, 2304, 12), (16, 700, 8)])
@pytest.mark.parametrize("overlap,ratio", [(1, 1), (1, 3), (0, 1)])
@pytest.mark.parametrize("threads", [1024, 512])
def test_tiled_backward_vs_oracle(device, monkeypatch, tile, rows, halo, overlap, ratio, threads):
    """The tiled backward over tile / cell-budget / halo geometries (m2f_set_option msda_*: geometry only), on a
    non-square pyramid whose tiles do not divide every level evenly, 5 % of the samples thrown far (the
    direct-atomic path), against the C oracle and the untiled kernel; phases 2 and 3 as one interleaved work queue
    (msda_bwd_overlap 1, the default) and one after the other."""
    from bm2f_amd import _native, msda
    with _native.options(msda_tile=tile, msda_win_rows=rows, msda_halo=halo, msda_bwd_overlap=overlap,
                         msda_bwd_ratio=ratio, msda_threads=threads):
        _tiled_backward_case(device, tile, rows)


@pytest.mark.parametrize("shapes,tile,tile_w", [([(48, 48)], 24, 24), ([(24, 24), (48, 48)], 24, 24),
                                                ([(64, 64)], 16, 32), ([(32, 64)], 16, 32)])
def test_tiled_backward_large_tiles_vs_oracle(device, shapes, tile, tile_w):
    """Tiles of 512 or more queries (phase 3's slots hold a g-row byte offset below 2^16, the zero row's included)
    take the untiled kernel.  1- and 2-level pyramids, against the C oracle."""
    from bm2f_amd import _native
    with _native.options(msda_tile=tile, msda_tile_w=tile_w, msda_threads=1024):
        _tiled_backward_case(device, tile, 0, shapes)


def _tiled_backward_case(device, tile, rows, shapes=((6, 10), (12, 20), (24, 40))):
    from bm2f_amd import _native, msda
    shapes = [tuple(s) for s in shapes]   # default: non-square, tiles not dividing every level evenly
    value, st, lsi, loc, attn, gout = _pyramid_case(shapes, 2, 8, 0.05, tile + rows)
    dst = msda.attach_host_shapes(st.to(device), shapes)
    gv, gl, ga = msda.ms_deform_attn_backward(value.to(device), dst, lsi.to(device), loc.to(device),
                                             attn.to(device), gout.to(device), 64)
    wv, wl, wa = msda_ref.msda_backward(value.double(), st, lsi, loc.double(), attn.double(), gout.double())
    _close(gv.cpu(), wv)
    _close(ga.cpu(), wa)
    amb = loc_crossing_mask(loc, shapes)
    assert amb.mean() < 2e-3
    _close(np.where(amb, 0.0, gl.cpu().numpy()), np.where(amb, 0.0, wl), atol_frac=1e-4)
    check_crossing_entries(gl.cpu().numpy(), value.double(), shapes, lsi, loc.numpy(), attn.numpy(), gout.numpy(), amb,
                           scale=np.abs(wl).max())
    # identical to the untiled kernel up to summation order
    with _native.options(msda_bwd_tiled=0):
        gv2, gl2, ga2 = msda.ms_deform_attn_backward(value.to(device), dst, lsi.to(device), loc.to(device),
                                                    attn.to(device), gout.to(device), 64)
    torch.testing.assert_close(gv, gv2, rtol=1e-5, atol=1e-5)
    # channel sums in another order (DPP tree vs shuffle tree)
    torch.testing.assert_close(ga, ga2, rtol=1e-4, atol=1e-6 * ga2.abs().max().item())
    torch.testing.assert_close(gl, gl2, rtol=1e-4, atol=1e-6 * gl2.abs().max().item())


@pytest.mark.parametrize("overlap", [1, 0])
def test_tiled_backward_nonfinite_and_zero_grads(device, overlap):
    """NaN in grad_output propagates into grad_value exactly where the reference's atomics put it, and zero
    grad_output rows give zeros, with phases 2 and 3 overlapped or not."""
    from bm2f_amd import _native, msda
    shapes = [(4, 4), (8, 8), (16, 16)]
    value, st, lsi, loc, attn, gout = _pyramid_case(shapes, 1, 8, 0.0, 7)
    gout[:, :16] = 0.0
    gout[0, 100, 5] = float("nan")
    dst = msda.attach_host_shapes(st.to(device), shapes)
    with _native.options(msda_bwd_overlap=overlap):
        gv, gl, ga = msda.ms_deform_attn_backward(value.to(device), dst, lsi.to(device), loc.to(device),
                                                 attn.to(device), gout.to(device), 64)
    wv, wl, wa = msda_ref.msda_backward(value.double(), st, lsi, loc.double(), attn.double(), gout.double())
    got, want = gv.cpu().double().numpy(), wv
    assert np.array_equal(np.isnan(got), np.isnan(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], rtol=1e-3, atol=1e-5 * np.abs(want[fin]).max())


@pytest.mark.parametrize("quad", [0, 1])
def test_forward_nonfinite_values_like_oracle(device, quad):
    """Both forwards (the reference-API op and the fused front end) read a corner outside the level from a
    clamped row and drop it by a zero weight, and drop a sample outside (-1, H) x (-1, W) by a select on its
    sum.  With non-finite values on every level's first pixel (where out-of-range samples are clamped) and
    one interior NaN, the outputs must be non-finite in exactly the oracle's elements and equal elsewhere."""
    from bm2f_amd import msda
    shapes = [(4, 4), (8, 8), (16, 16)]
    value, st, lsi, loc, attn, _ = _pyramid_case(shapes, 2, 8, 0.25, 11)
    for l0 in lsi.tolist():
        value[:, l0, :, :3] = float("inf")
    value[1, 40, 2, 7] = float("nan")
    dst = msda.attach_host_shapes(st.to(device), shapes)
    want = msda_ref.msda_forward(value.double(), st, lsi, loc.double(), attn.double())
    from bm2f_amd import _native
    with _native.options(msda_fwd_quad=quad):
        got = msda.ms_deform_attn_forward(value.to(device), dst, lsi.to(device), loc.to(device), attn.to(device),
                                          64).cpu().double().numpy().reshape(want.shape)
    assert np.array_equal(np.isfinite(got), np.isfinite(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], rtol=1e-4, atol=1e-5 * np.abs(want[fin]).max())
    # the fused front end on the same samples: proj = [offsets in pixels from the reference points | logits
    # whose softmax is attn]
    N, S, M, L, P = loc.shape[0], loc.shape[1], loc.shape[2], loc.shape[3], loc.shape[4]
    refs = []
    for h, w in shapes:
        ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h), torch.linspace(0.5, w - 0.5, w), indexing="ij")
        refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
    ref = torch.cat(refs, 0)[None, :, None, :].expand(N, S, L, 2).contiguous()
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)
    off = (loc - ref[:, :, None, :, None, :]) * norm[None, None, None, :, None, :]
    logits = attn.reshape(N, S, M, L * P).log()
    proj = torch.cat([off.reshape(N, S, -1), logits.reshape(N, S, -1)], -1).contiguous()
    with _native.options(msda_fwd_quad=quad):  # the quad form skips an out-of-range point by the exec mask
        out = msda.MSDeformAttnFusedFunction.apply(value.to(device), proj.to(device), ref.to(device), shapes, P)
    # the fused path recomputes loc and attn (softmax of log attn, ref + off / (W, H)) in fp32: same
    # finite pattern as the oracle on the materialised tensors, values within the rounding of that round trip
    sm = torch.softmax(logits, -1).reshape(attn.shape)
    loc2 = ref[:, :, None, :, None, :] + off / norm[None, None, None, :, None, :]
    want2 = msda_ref.msda_forward(value.double(), st, lsi, loc2.double(), sm.double())
    got2 = out.cpu().double().numpy().reshape(want2.shape)
    assert np.array_equal(np.isfinite(got2), np.isfinite(want2))
    fin2 = np.isfinite(want2)
    np.testing.assert_allclose(got2[fin2], want2[fin2], rtol=1e-3, atol=1e-4 * np.abs(want2[fin2]).max())


@pytest.mark.parametrize("shapes", [[(4, 4), (8, 8), (16, 16)], [(6, 10), (12, 20), (24, 40)], [(5, 7), (10, 13)]])
def test_fused_front_end_matches_unfused(device, monkeypatch, shapes):
    """MSDeformAttn with the fused front end == the reference-structured path (Linear -> softmax -> loc ->
    MSDA), outputs and every gradient, on an encoder-shaped call."""
    from bm2f_amd import msda
    from bm2f_amd.msda import MSDeformAttn, attach_host_shapes
    torch.manual_seed(0)
    L = len(shapes)
    m = MSDeformAttn(256, L, 8, 4).to(device)
    with torch.no_grad():  # make the offsets/logits non-trivial
        m.sampling_offsets.weight.normal_(0, 0.02)
        m.attention_weights.weight.normal_(0, 0.05)
    st = torch.tensor(shapes, dtype=torch.int64, device=device)
    attach_host_shapes(st, shapes)
    lsi = torch.cat((st.new_zeros(1), st.prod(1).cumsum(0)[:-1]))
    S = int(st.prod(1).sum())
    N = 2
    refs = []
    for h, w in shapes:
        ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h), torch.linspace(0.5, w - 0.5, w), indexing="ij")
        refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
    ref = torch.cat(refs, 0).to(device)[None, :, None, :].expand(N, S, L, 2)
    src = torch.randn(N, S, 256, device=device)
    pos = torch.randn(N, S, 256, device=device)
    outs, grads = [], []
    for fused in (True, False):
        monkeypatch.setattr(msda, "FUSED", fused)
        m.zero_grad()
        x = src.clone().requires_grad_()
        out = m(x + pos, ref, x, st, lsi)
        out.backward(torch.ones_like(out) * 0.01 + out.detach() * 0.1)
        outs.append(out.detach())
        grads.append([x.grad] + [p.grad.clone() for p in m.parameters()])
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-5)
    for a, b in zip(grads[0], grads[1]):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4 * max(b.abs().max().item(), 1e-6))


@pytest.mark.parametrize("shapes", [[(32, 32), (64, 64), (128, 128)], [(5, 7), (10, 13), (20, 26)],
                                    [(9, 17)], [(4, 4), (8, 8), (16, 16), (32, 32)], [(6, 10), (12, 20)]])
@pytest.mark.parametrize("quad,pb,lds,pair", [(0, 2, 0, 0), (1, 1, 0, 0), (1, 2, 0, 0), (1, 4, 0, 0), (1, 2, 1, 0),
                                              (1, 2, 1, 1)])
def test_fused_forward_variants_vs_oracle(device, shapes, quad, pb, lds, pair):
    """The fused forward (m2f_msda_fused_fwd_f32) in its LDS-window forms (value windows staged in LDS per tile and
    level; two lanes per query, the default, or a lane quad per query), its quad form (a lane quad per (query, head), point geometry by DPP broadcast,
    out-of-range points skipped by the exec mask; 1, 2 or 4 points per load batch) and its 8-lane form, against
    the C oracle on the loc / attn the reference front end derives from the same projection: power-of-two and odd
    level shapes (tile edges), 1-4 levels, 5 % of the samples thrown far (out of the level and out of range)."""
    from bm2f_amd import _native
    from bm2f_amd.msda import MSDeformAttnFusedFunction
    from test_scale_gpu import _fused_case, _loc_attn
    N, P = 2, 4
    L = len(shapes)
    value, proj, ref = _fused_case(shapes, N, 0.05, seed=21 + L)
    S = value.shape[1]
    rf = ref.float()[None, :, None, :].expand(N, S, L, 2).to(device)
    with _native.options(msda_fwd_quad=quad, msda_fwd_pb=pb, msda_fwd_lds=lds, msda_fwd_pair=pair):
        out = MSDeformAttnFusedFunction.apply(value.to(device), proj.to(device), rf, tuple(shapes), P)
    torch.cuda.synchronize()
    loc, attn = _loc_attn(proj, ref, shapes)
    st = torch.tensor(shapes, dtype=torch.int64)
    lsi = torch.cat((st.new_zeros(1), st.prod(1).cumsum(0)[:-1]))
    want = msda_ref.msda_forward(value.double(), st, lsi, loc, attn)
    _close(out.cpu(), want)


@pytest.mark.parametrize("shapes", [[(32, 32), (64, 64), (128, 128)], [(5, 7), (10, 13), (20, 26)], [(9, 17)],
                                    [(4, 4), (8, 8), (16, 16), (32, 32)], [(6, 10), (12, 20)]])
@pytest.mark.parametrize("tile,tile_w,cap,halo", [(4, 8, 64, 2), (16, 16, 1024, 8), (8, 16, 96, 0), (3, 5, 48, 1),
                                               (8, 16, 312, 4), (8, 12, 304, 3), (4, 12, 40, 1)])
@pytest.mark.parametrize("pair,xcd", [(1, 0), (0, 0), (1, 1)])
def test_fused_forward_lds_geometries_bitwise(device, shapes, tile, tile_w, cap, halo, pair, xcd):
    """The LDS-window forwards (two lanes per query, or a lane quad; a tile of more than 128 queries runs the quad
    form) compute each output element with the quad kernel's arithmetic in the same order, so every window
    geometry (tile, window rows, halo; small budgets force the halo to shrink and send samples to the HBM path)
    returns the quad kernel's output bit for bit, 5 % of the samples thrown far; under both block -> (tile, head)
    mappings (msda_fwd_xcd: a tile range per XCD, or the head fastest)."""
    from bm2f_amd import _native
    from bm2f_amd.msda import MSDeformAttnFusedFunction
    from test_scale_gpu import _fused_case
    N, P = 2, 4
    L = len(shapes)
    value, proj, ref = _fused_case(shapes, N, 0.05, seed=41 + L)
    S = value.shape[1]
    args = (value.to(device), proj.to(device), ref.float()[None, :, None, :].expand(N, S, L, 2).to(device),
            tuple(shapes), P)
    with _native.options(msda_fwd_lds=0):
        want = MSDeformAttnFusedFunction.apply(*args)
    with _native.options(msda_fwd_lds=1, msda_fwd_tile=tile, msda_fwd_tile_w=tile_w, msda_fwd_cap=cap,
                         msda_fwd_halo=halo, msda_fwd_xcd=xcd, msda_fwd_pair=pair):
        got = MSDeformAttnFusedFunction.apply(*args)
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@pytest.mark.parametrize("shapes", [[(5, 7), (10, 13), (20, 26)], [(9, 17)], [(4, 4), (8, 8), (16, 16), (32, 32)],
                                    [(6, 10), (12, 20)]])
@pytest.mark.parametrize("quad", [1, 0])
def test_fused_backward_variants_vs_oracle(device, shapes, quad):
    """The fused forward (quad or 8-lane form) and backward (phases 2 and 3 overlapped or not), 1-4 levels, odd
    level shapes, 5 % of the samples thrown far (the out-of-window atomics of every lane of a quad), against the
    C oracle: grad_value, d offsets (crossing entries one-sided) and d logits."""
    from bm2f_amd import _native
    from test_scale_gpu import fused_fwd_bwd_vs_oracle
    with _native.options(msda_bwd_overlap=quad, msda_fwd_quad=quad):
        fused_fwd_bwd_vs_oracle(device, shapes, N=2, far=0.05, seed=31 + len(shapes))


@pytest.mark.parametrize("lds,pair", [(1, 1), (1, 0), (0, 0)])
def test_fused_forward_nan_weights_on_skipped_points(device, lds, pair):
    """A (query, head) whose every point lies outside its level adds nothing, whatever its attention weights hold:
    the reference kernel tests the sample position before it touches the weight (ms_deform_im2col_cuda.cuh:257-262),
    so NaN logits on such a row give a zero output.  The LDS-window forwards, two lanes or a lane quad per query
    (whose LDS-only gathers run the FMAs of skipped points on a zero row: the weights must be zeroed, not multiplied
    by 0), and the quad kernel."""
    from bm2f_amd import _native
    from bm2f_amd.msda import MSDeformAttnFusedFunction
    from test_scale_gpu import _fused_case
    shapes = [(32, 32), (64, 64), (128, 128)]
    N, M, L, P = 2, 8, 3, 4
    value, proj, ref = _fused_case(shapes, N, 0.0, seed=5)
    S = value.shape[1]
    off = proj[..., :M * L * P * 2].view(N, S, M, L, P, 2)
    logit = proj[..., M * L * P * 2:].view(N, S, M, L * P)
    rows = [(0, 7, 3), (0, 1500, 0), (1, 20000, 5), (1, 21000, 7)]   # (image, query, head), all three levels
    for n, q, m in rows:
        off[n, q, m] = 1e5
        logit[n, q, m] = float("nan")
    args = (value.to(device), proj.to(device), ref.float()[None, :, None, :].expand(N, S, L, 2).to(device),
            tuple(shapes), P)
    with _native.options(msda_fwd_lds=lds, msda_fwd_pair=pair):
        out = MSDeformAttnFusedFunction.apply(*args)
    torch.cuda.synchronize()
    out = out.cpu().view(N, S, M, 32)
    assert torch.isfinite(out).all(), "a skipped point's NaN weight reached the output"
    for n, q, m in rows:
        assert (out[n, q, m] == 0).all()
    with _native.options(msda_fwd_lds=1 - lds, msda_fwd_pair=1 - pair):
        other = MSDeformAttnFusedFunction.apply(*args).cpu().view(N, S, M, 32)
    assert torch.equal(out, other)


@pytest.mark.parametrize("walk4,rowsort", [(1, 1), (0, 1), (1, 0), (0, 0)])
def test_fused_backward_phase3_forms_vs_oracle(device, walk4, rowsort):
    """Phase 3 of the tiled backward in its four forms -- records four per step decoded once per quad (msda_bwd_walk4
    1, the default) or two per step (0); rows dealt in order of their record count (msda_bwd_rowsort 1, the default) or
    window order (0) -- against the C oracle, odd level shapes and 5 % far samples."""
    from bm2f_amd import _native
    from test_scale_gpu import fused_fwd_bwd_vs_oracle
    with _native.options(msda_bwd_walk4=walk4, msda_bwd_rowsort=rowsort):
        fused_fwd_bwd_vs_oracle(device, [(5, 7), (10, 13), (20, 26)], N=2, far=0.05, seed=77)


@pytest.mark.parametrize("walk4", [1, 0])
def test_tiled_backward_nonfinite_grad_stays_local(device, walk4):
    """A non-finite grad_output row reaches only the value rows its own samples touch, as in the reference's scatter:
    phase 3's padding records (quad form) read a zero g row, not another query's.  The finite / non-finite pattern
    of grad_value equals the oracle's."""
    from bm2f_amd import _native, msda
    shapes = [(6, 10), (12, 20), (24, 40)]
    value, st, lsi, loc, attn, gout = _pyramid_case(shapes, 2, 8, 0.0, 11)
    gout = gout.clone()
    gout[0, 37, :5] = float("inf")
    gout[1, 500, 40] = float("nan")
    dst = msda.attach_host_shapes(st.to(device), shapes)
    with _native.options(msda_bwd_walk4=walk4, msda_threads=1024):
        gv, _, _ = msda.ms_deform_attn_backward(value.to(device), dst, lsi.to(device), loc.to(device),
                                                attn.to(device), gout.to(device), 64)
    wv, _, _ = msda_ref.msda_backward(value.double(), st, lsi, loc.double(), attn.double(), gout.double())
    fin = torch.isfinite(gv.cpu()).numpy()
    assert (~fin).any() and fin.any()
    assert (fin == np.isfinite(wv)).all(), f"{(fin != np.isfinite(wv)).sum()} elements differ in finiteness"


def _to_head_major(t, M, LP):
    """(N, S, M*3*LP) rows in the reference order [offsets (M, LP, 2) | logits (M, LP)] -> one record per head."""
    N, S, _ = t.shape
    return torch.cat([t[..., :2 * M * LP].reshape(N, S, M, 2 * LP), t[..., 2 * M * LP:].reshape(N, S, M, LP)],
                     -1).reshape(N, S, -1).contiguous()


@pytest.mark.parametrize("shapes", [[(32, 32), (64, 64), (128, 128)], [(5, 7), (10, 13), (20, 26)],
                                    [(4, 4), (8, 8), (16, 16), (32, 32)]])
@pytest.mark.parametrize("quad,lds,pair", [(1, 1, 0), (1, 0, 0), (0, 0, 0), (1, 1, 1)])
def test_fused_head_major_matches_reference_layout(device, shapes, quad, lds, pair):
    """The head-major entry points (m2f_msda_fused_{fwd,bwd}_hm_f32: one [offsets | logits] record per head in
    each projection row, the module's layout) return the reference-layout calls' output and gradients bit for
    bit -- grad_value in deterministic mode, d proj in the head-major layout -- for every forward form, 5 % of
    the samples thrown far."""
    from bm2f_amd import _native
    from bm2f_amd.msda import MSDeformAttnFusedFunction
    from test_scale_gpu import _fused_case
    N, M, P = 2, 8, 4
    L = len(shapes)
    value, proj, ref = _fused_case(shapes, N, 0.05, seed=61 + L)
    S = value.shape[1]
    rf = ref.float()[None, :, None, :].expand(N, S, L, 2).to(device)
    gout = torch.randn(N, S, M * 32, generator=torch.Generator().manual_seed(3)).to(device)
    res = []
    with _native.options(msda_fwd_quad=quad, msda_fwd_lds=lds, msda_fwd_pair=pair, msda_bwd_det=1):
        for hm in (False, True):
            v = value.to(device).requires_grad_()
            pj = (_to_head_major(proj, M, L * P) if hm else proj).to(device).requires_grad_()
            out = MSDeformAttnFusedFunction.apply(v, pj, rf, tuple(shapes), P, hm)
            out.backward(gout)
            res.append((out.detach(), v.grad, pj.grad))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    assert torch.equal(_to_head_major(res[0][2], M, L * P), res[1][2])
