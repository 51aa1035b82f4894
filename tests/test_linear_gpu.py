"""fp32 MFMA GEMMs (csrc/gemm.hip) and the encoder's linear / FFN autograd nodes (linear_ops.py) against
fp64 torch references of nn.Linear / linear2(relu(linear1(x))) (msdeformattn.py:101-106,
ms_deform_attn.py:59-62)."""
import pytest
import torch
from torch import nn

from bm2f_amd import linear_ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,N,K", [(1, 4, 4), (37, 256, 256), (1000, 288, 256), (129, 1024, 256), (300, 256, 1024),
                                   (5000, 96, 36), (77, 132, 260)])
@pytest.mark.parametrize("epi", ["none", "bias", "relu", "bias_relu", "mask", "bias_mask"])
@pytest.mark.parametrize("engine,b_kn", [("exact", False), ("x3", False), ("x3", True)])
def test_gemm_nt_vs_fp64(device, M, N, K, epi, engine, b_kn):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(device)
    b = torch.randn(N, K, generator=g).to(device)
    bias = torch.randn(N, generator=g).to(device) if "bias" in epi else None
    mask = torch.randn(M, N, generator=g).to(device) if "mask" in epi else None
    bb = b.t().contiguous() if b_kn else b
    out = linear_ops.gemm_nt(a, bb, bias, relu="relu" in epi, mask=mask, engine=engine, b_kn=b_kn)
    ref = a.double() @ b.double().t()
    if bias is not None:
        ref = ref + bias.double()
    if "relu" in epi:
        ref = ref.clamp_min(0)
    if mask is not None:
        ref = torch.where(mask.double() > 0, ref, torch.zeros_like(ref))
    assert _rel(out, ref) < 2e-6


@pytest.mark.parametrize("M,N1,N2", [(1, 4, 4), (31, 256, 256), (4097, 288, 256), (10000, 1024, 256),
                                     (777, 256, 1024), (33, 132, 8)])
@pytest.mark.parametrize("engine", ["exact", "x3"])
def test_gemm_tn_vs_fp64(device, M, N1, N2, engine):
    g = torch.Generator(device="cpu").manual_seed(M * 3 + N1)
    a = torch.randn(M, N1, generator=g).to(device)
    b = torch.randn(M, N2, generator=g).to(device)
    c, cs = linear_ops.gemm_tn(a, b, colsum=True, engine=engine)
    assert _rel(c, a.double().t() @ b.double()) < 2e-6
    assert _rel(cs, a.double().sum(0)) < 2e-6
    c2, cs2 = linear_ops.gemm_tn(a, b, colsum=True, engine=engine)     # fixed-order slab reduce: repeatable
    assert torch.equal(c, c2) and torch.equal(cs, cs2)


@pytest.mark.parametrize("engine", ["exact", "x3"])
def test_gemm_tn_zero_rows(device, engine):
    a = torch.empty(0, 8, device=device)
    b = torch.empty(0, 4, device=device)
    c, cs = linear_ops.gemm_tn(a, b, colsum=True, engine=engine)
    assert torch.equal(c, torch.zeros(8, 4, device=device)) and torch.equal(cs, torch.zeros(8, device=device))


@pytest.mark.parametrize("shape,cin,cout,relu", [((2, 333, 256), 256, 256, False), ((2, 333, 256), 256, 288, False),
                                                 ((700, 256), 256, 1024, True), ((3, 50, 1024), 1024, 256, False)])
def test_linear_autograd_vs_fp64(device, shape, cin, cout, relu):
    torch.manual_seed(cin + cout)
    lin = nn.Linear(cin, cout).to(device)
    x = torch.randn(*shape, device=device, requires_grad=True)
    y = linear_ops.linear(x, lin, relu=relu)
    gy = torch.randn_like(y)
    y.backward(gy)
    xd = x.detach().double().requires_grad_(True)
    wd = lin.weight.detach().double().requires_grad_(True)
    bd = lin.bias.detach().double().requires_grad_(True)
    yd = torch.nn.functional.linear(xd, wd, bd)
    if relu:
        yd = yd.clamp_min(0)
    yd.backward(gy.double())
    assert _rel(y, yd) < 2e-6
    assert _rel(x.grad, xd.grad) < 2e-6
    assert _rel(lin.weight.grad, wd.grad) < 2e-6
    assert _rel(lin.bias.grad, bd.grad) < 2e-6


def test_ffn_autograd_vs_fp64(device):
    # fp64 reference on the fp32 forward's ReLU pattern: a pre-activation within an ulp of 0 can take the
    # other branch in fp64, and one flipped unit moves a whole row of grad_h (~1e-3 of the norm here)
    torch.manual_seed(5)
    l1, l2 = nn.Linear(256, 1024).to(device), nn.Linear(1024, 256).to(device)
    x = torch.randn(3, 1111, 256, device=device, requires_grad=True)
    y = linear_ops.ffn(x, l1, l2)
    gy = torch.randn_like(y)
    y.backward(gy)
    x2 = x.detach().reshape(-1, 256)
    on = linear_ops.gemm_nt(x2, l1.weight.detach(), l1.bias.detach(), relu=True) > 0
    X, W1, B1, W2 = x2.double(), l1.weight.detach().double(), l1.bias.detach().double(), l2.weight.detach().double()
    G = gy.reshape(-1, 256).double()
    H = torch.where(on, X @ W1.t() + B1, torch.zeros((), dtype=torch.float64, device=device))
    GH = torch.where(on, G @ W2, torch.zeros((), dtype=torch.float64, device=device))
    assert _rel(y.reshape(-1, 256), H @ W2.t() + l2.bias.detach().double()) < 2e-6
    want = {"x": GH @ W1, "w1": GH.t() @ X, "b1": GH.sum(0), "w2": G.t() @ H, "b2": G.sum(0)}
    got = {"x": x.grad.reshape(-1, 256), "w1": l1.weight.grad, "b1": l1.bias.grad, "w2": l2.weight.grad,
           "b2": l2.bias.grad}
    errs = {k: _rel(got[k], want[k]) for k in want}
    assert max(errs.values()) < 2e-6, str(errs)


def test_gemm_rejects(device):
    a = torch.randn(4, 6, device=device)
    with pytest.raises(RuntimeError, match="multiples of 4"):
        linear_ops.gemm_nt(a, torch.randn(4, 6, device=device))
    with pytest.raises(RuntimeError, match="exclusive"):
        linear_ops.gemm_nt(torch.randn(4, 8, device=device), torch.randn(4, 8, device=device), relu=True,
                           mask=torch.ones(4, 4, device=device))


@pytest.mark.parametrize("M,N,K", [(4096, 256, 256), (2048, 1024, 256), (2048, 256, 1024)])
def test_x3_error_matches_exact_fp32(device, M, N, K):
    """The split-bf16 engine is an fp32 GEMM: its error vs fp64 stays at the exact-f32 MFMA's level,
    elementwise and in norm, on wide-dynamic-range data (values spanning 2^-20 .. 2^20)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    a = torch.randn(M, K, generator=g) * torch.exp2(torch.randint(-20, 21, (M, K), generator=g).float())
    b = torch.randn(N, K, generator=g)
    a, b = a.to(device), b.to(device)
    ref = a.double() @ b.double().t()
    scale = a.double().abs() @ b.double().abs().t()       # sum |a||b| per element: the fp32 error scale
    e_x3 = ((linear_ops.gemm_nt(a, b, engine="x3").double() - ref).abs() / scale).max().item()
    e_ex = ((linear_ops.gemm_nt(a, b, engine="exact").double() - ref).abs() / scale).max().item()
    assert e_x3 < 4 * 2.0 ** -24 * K ** 0.5 + 2 * e_ex, (e_x3, e_ex)


def test_x3_nonfinite_inputs_propagate(device):
    """A non-finite input gives non-finite outputs exactly where fp32 does.  (An inf can come out as a
    NaN: inf times the split planes of one finite operand can meet opposite signs.)"""
    a = torch.randn(64, 32, device=device)
    b = torch.randn(16, 32, device=device)
    a[3, 5] = float("inf")
    a[7, 1] = float("nan")
    for eng in ("x3", "exact"):
        c = linear_ops.gemm_nt(a, b, engine=eng)
        ref = a @ b.t()
        assert torch.equal(torch.isfinite(c), torch.isfinite(ref))


@pytest.mark.parametrize("M,N,K", [(1, 4, 4), (1000, 256, 288), (129, 256, 1024), (77, 132, 260)])
@pytest.mark.parametrize("n_add,bias,alias", [(1, False, False), (2, False, False), (1, True, False),
                                              (2, False, True)])
def test_gemm_nt_addends_vs_fp64(device, M, N, K, n_add, bias, alias):
    """m2f_gemm_f32x3_nt_add: C = A.B (+ bias) + D1 (+ D2), C may alias an addend."""
    g = torch.Generator(device="cpu").manual_seed(M + 7 * N + K + n_add)
    a = torch.randn(M, K, generator=g).to(device)
    w = torch.randn(K, N, generator=g).to(device)            # b_kn: the weight of an input gradient
    bv = torch.randn(N, generator=g).to(device) if bias else None
    adds = [torch.randn(M, N, generator=g).to(device) for _ in range(n_add)]
    ref = a.double() @ w.double() + (bv.double() if bias else 0) + sum(d.double() for d in adds)
    out = linear_ops.gemm_nt(a, w, bv, b_kn=True, add=adds, out=adds[0] if alias else None)
    assert _rel(out, ref) < 2e-6
    if alias:
        assert out.data_ptr() == adds[0].data_ptr()


@pytest.mark.parametrize("pos_batch", [2, 1])
def test_encoder_layer_residual_fused_matches_autograd_sums(device, pos_batch):
    """The encoder layer with residual gradients summed in GEMM epilogues (EncoderInProjF32 /
    FFNResidualF32) against the same layer with plain autograd sums: outputs equal, gradients to fp32
    rounding of the reordered sums.  A batch-shared embedding (pos_batch 1) is folded into the query projection by
    linearity (src Wq^T + (pos Wq^T + bq), m2f_gemm_f32x3_nt_rowadd), a different fp32 rounding of the same sum:
    outputs within 1e-5, gradients 1e-3 (measured 1.8e-4: a reordered rounding of a sampling coordinate moves
    its d loc term)."""
    from bm2f_amd import pixel_decoder
    from bm2f_amd.msda import attach_host_shapes

    torch.manual_seed(0)
    layer = pixel_decoder.MSDeformAttnTransformerEncoderLayer(256, 1024, 0.0, "relu", 3, 8, 4).to(device)
    for p in layer.parameters():                 # reference init zeros the sampling weights; perturb them
        p.data.add_(torch.randn_like(p) * 0.02)
    shapes = [(8, 8), (16, 16), (32, 32)]
    S = sum(h * w for h, w in shapes)
    st = attach_host_shapes(torch.tensor(shapes, device=device), shapes)
    lsi = torch.tensor([0, 64, 320], device=device)
    enc = pixel_decoder.MSDeformAttnTransformerEncoder
    ref_pts = enc.get_reference_points(shapes, torch.ones(2, 3, 2, device=device), device)
    src0 = torch.randn(2, S, 256, device=device)
    pos0 = torch.randn(pos_batch, S, 256, device=device)      # 1: a batch-shared embedding, broadcast
    gout = torch.randn(2, S, 256, device=device)
    res = {}
    for fused in (True, False):
        pixel_decoder.RESIDUAL_FUSED = fused
        try:
            layer.zero_grad()
            src = src0.clone().requires_grad_()
            pos = pos0.clone().requires_grad_()
            out = layer(src, pos, ref_pts, st, lsi)
            out.backward(gout)
            res[fused] = [out.detach(), src.grad, pos.grad] + [p.grad.clone() for p in layer.parameters()]
        finally:
            pixel_decoder.RESIDUAL_FUSED = True
    if pos_batch == 2:
        assert torch.equal(res[True][0], res[False][0])
    else:
        assert _rel(res[True][0], res[False][0]) < 1e-5
    for a, b in zip(res[True][1:], res[False][1:]):
        assert _rel(a, b) < (1e-6 if pos_batch == 2 else 1e-3)


@pytest.mark.parametrize("M,period,N,K", [(2 * 5376, 5376, 288, 256), (3 * 100, 100, 96, 64), (999, 1000, 128, 32)])
def test_gemm_nt_rowadd_vs_fp64(device, M, period, N, K):
    """m2f_gemm_f32x3_nt_rowadd: C = A B^T + R[m % period] against fp64."""
    torch.manual_seed(M)
    a = torch.randn(M, K, device=device)
    w = torch.randn(N, K, device=device) / K ** 0.5
    r = torch.randn(period, N, device=device)
    out = linear_ops.gemm_nt_rowadd(a, w, r, period)
    idx = torch.arange(M, device=device) % period
    ref = a.double() @ w.double().t() + r.double()[idx]
    assert _rel(out, ref) < 2e-6


@pytest.mark.parametrize("M,N,K,b_kn", [(1000, 1024, 256, False), (777, 64, 96, False), (513, 256, 1024, True)])
def test_gemm_nt_relu_bits(device, M, N, K, b_kn):
    """The FFN's 1-bit ReLU mask (m2f_gemm_f32x3_nt_bits): the forward writes bit (m, n) = relu(.)[m, n] > 0 and
    the same relu output as the float path; the masked input gradient from the bits equals the one masked by
    the fp32 activation, bit for bit."""
    torch.manual_seed(M + N)
    a = torch.randn(M, K, device=device)
    w = torch.randn(N, K, device=device) / K ** 0.5
    b = torch.randn(N, device=device)
    bits = torch.empty(M, N // 32, device=device, dtype=torch.int32)
    h = linear_ops.gemm_nt_bits(a, w, b, bits_out=bits)
    assert torch.equal(h, linear_ops.gemm_nt(a, w, b, relu=True))
    shifts = torch.arange(32, device=device, dtype=torch.int64)
    unpacked = ((bits.to(torch.int64).unsqueeze(-1) >> shifts) & 1).reshape(M, N).bool()
    assert torch.equal(unpacked, h > 0)
    g = torch.randn(M, K if not b_kn else K, device=device)
    w2 = torch.randn(N, K, device=device) / K ** 0.5 if not b_kn else torch.randn(K, N, device=device) / K ** 0.5
    if b_kn:   # grad_h = g . W2 with W2 (K, N) read in place, as the FFN's backward
        got = linear_ops.gemm_nt_bits(g, w2, bits_in=bits, b_kn=True)
        want = linear_ops.gemm_nt(g, w2, mask=h, b_kn=True)
    else:
        got = linear_ops.gemm_nt_bits(g, w2, bits_in=bits)
        want = linear_ops.gemm_nt(g, w2, mask=h)
    assert torch.equal(got, want)


def test_x3_tn_zero_rows_graph_capture_no_memset(device):
    """The x3 TN GEMM over M = 0 rows writes C = 0 (and colsum = 0) with the library's fill kernels: captured in a
    HIP graph it leaves no memset node (memsets replay wrongly under the runtime's graph packet capture), a strided C
    keeps its padding columns, and every replay re-zeroes C."""
    import ctypes
    from bm2f_amd import _native
    from bm2f_amd.bench_model import graph_node_counts
    N1, N2, ldc = 40, 48, 64
    dummy = torch.zeros(4, device=device)
    C = torch.full((N1, ldc), 7.0, device=device)
    cs = torch.full((N1,), 7.0, device=device)
    wsb = ctypes.c_int64(0)
    _native.call("m2f_gemm_f32x3_tn_workspace", 0, N1, N2, ctypes.byref(wsb))
    ws = torch.empty(max(wsb.value, 16), device=device, dtype=torch.uint8)

    def run():
        _native.call("m2f_gemm_f32x3_tn", dummy.data_ptr(), ctypes.c_int64(N1), dummy.data_ptr(), ctypes.c_int64(N2),
                     C.data_ptr(), ctypes.c_int64(ldc), cs.data_ptr(), 0, N1, N2, ws.data_ptr(),
                     ctypes.c_int64(ws.numel()), torch.cuda.current_stream().cuda_stream)
    run()
    torch.cuda.synchronize()
    assert (C[:, :N2] == 0).all() and (C[:, N2:] == 7).all() and (cs == 0).all()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            run()
    nodes = graph_node_counts(g)
    assert not nodes.get("memset"), nodes
    g.instantiate()
    for _ in range(2):
        C.fill_(7.0)
        cs.fill_(7.0)
        g.replay()
        torch.cuda.synchronize()
        assert (C[:, :N2] == 0).all() and (C[:, N2:] == 7).all() and (cs == 0).all()
