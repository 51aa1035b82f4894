"""m2f_colsum (column sums without a memset, graph-safe) and the bias-add autograd functions built on it, against
fp64 sums and torch autograd (the level-embedding adds of mask2former_transformer_decoder.py:376,
msdeformattn.py:75, video_mask2former_transformer_decoder.py:388, and the memory-token projection biases)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 7), (255, 256), (257, 256), (262144, 256), (70000, 65), (0, 8)])
def test_colsum_matches_fp64(device, dt, rows, cols):
    from bm2f_amd.decoder_ops import colsum_f32
    g = torch.Generator(device=device).manual_seed(rows * 31 + cols)
    x = torch.randn(rows, cols, device=device, generator=g).to(dt)
    got = colsum_f32(x)
    ref = x.double().sum(0)
    assert got.dtype == torch.float32 and got.shape == (cols,)
    tol = 1e-5 * max(1.0, rows ** 0.5) * 4
    torch.testing.assert_close(got.double(), ref, rtol=1e-5, atol=tol)
    assert torch.equal(got, colsum_f32(x))   # same order every call


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("k", [1, 2, 6, 8])
def test_sum_to_f32_bitwise_vs_sequential_adds(device, dt, k):
    """m2f_sum_to_f32 (the decoder's memory-gradient sink) equals terms[0].float() followed by k - 1 in-place
    mixed-dtype adds -- the arithmetic of autograd's cast-and-accumulate -- bit for bit."""
    from bm2f_amd.decoder_ops import sum_to_f32
    g = torch.Generator(device=device).manual_seed(k)
    terms = [(torch.randn(2048, 256, device=device, generator=g) * 10 ** (i % 3)).to(dt) for i in range(k)]
    want = terms[0].to(torch.float32, copy=True)         # (an fp32 term's .float() would alias it)
    for t in terms[1:]:
        torch.add(want, t, out=want)
    got = sum_to_f32(terms)
    assert got.dtype == torch.float32 and torch.equal(got, want)
    odd = [t.reshape(-1)[:1001] for t in terms]          # 1001 elements: the torch path
    want_odd = odd[0].to(torch.float32, copy=True)
    for t in odd[1:]:
        torch.add(want_odd, t, out=want_odd)
    assert torch.equal(sum_to_f32(odd), want_odd)


def test_colsum_non_contiguous_input(device):
    from bm2f_amd.decoder_ops import colsum_f32
    x = torch.randn(256, 4096, device=device).t()   # (4096, 256) view with stride (1, 4096)
    torch.testing.assert_close(colsum_f32(x).double(), x.double().sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("xdt", [torch.float32, torch.float16])
def test_row_bias_add_grads(device, xdt):
    from bm2f_amd.decoder_ops import row_bias_add
    g = torch.Generator(device=device).manual_seed(5)
    x = torch.randn(2, 4096, 256, device=device, generator=g).to(xdt).requires_grad_()
    b = torch.randn(256, device=device, generator=g).requires_grad_()
    y = row_bias_add(x.transpose(0, 1).contiguous().transpose(0, 1), b)   # a non-contiguous x as the decoder's
    gy = torch.randn(y.shape, device=device, generator=g, dtype=y.dtype)
    y.backward(gy)
    x2, b2 = x.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    y2 = x2 + b2
    y2.backward(gy)
    assert y.dtype == y2.dtype and torch.equal(y, y2)
    assert torch.equal(x.grad, x2.grad)
    torch.testing.assert_close(b.grad.double(), gy.double().sum((0, 1)), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("L", [3840, 4095])
def test_chan_bias_add_grads(device, L):
    """L = 4095 (odd): the gradient's L sum is zero-padded to a multiple of 64, so both stages stay short."""
    from bm2f_amd.decoder_ops import chan_bias_add
    g = torch.Generator(device=device).manual_seed(6)
    x = torch.randn(10, 256, L, device=device, generator=g).requires_grad_()
    b = torch.randn(256, device=device, generator=g).requires_grad_()
    y = chan_bias_add(x, b)
    gy = torch.randn(y.shape, device=device, generator=g)
    y.backward(gy)
    assert torch.equal(y, x.detach() + b.detach()[None, :, None])
    assert torch.equal(x.grad, gy)
    torch.testing.assert_close(b.grad.double(), gy.double().sum((0, 2)), rtol=1e-5, atol=1e-3)
