"""Module structure and numerics on CPU: the bm2f_amd modules with the oracle's MSDA core patched in,
against the golden outputs of the reference modules (tests/golden/*.npz)."""
import numpy as np
import pytest
import torch

from conftest import golden
from module_cases import build_decoder, build_pixdec, build_video_decoder, oracle_msda, rel_err, run_pixdec


def test_pixdec_state_dict_keys_match_reference():
    m = build_pixdec()
    assert sorted(m.state_dict().keys()) == list(golden("pixdec.npz")["state_dict_keys"])
    assert sum(p.numel() for p in m.parameters()) == 6035904  # SURVEY §8(b), measured on the reference


def test_decoder_state_dict_keys_match_reference():
    d = build_decoder()
    assert sorted(d.state_dict().keys()) == list(golden("decoder.npz")["state_dict_keys"])
    assert sum(p.numel() for p in d.parameters()) == 14493062


def test_video_decoder_state_dict_keys_match_reference():
    d = build_video_decoder()
    assert sorted(d.state_dict().keys()) == list(golden("video_decoder.npz")["state_dict_keys"])


def test_pixdec_forward_backward_cpu():
    m = build_pixdec()
    with oracle_msda():
        g, feats, outs = run_pixdec(m, torch.device("cpu"))
    names = ["out_mask_features", "out_out0", "out_ms0", "out_ms1", "out_ms2"]
    for name, o in zip(names, outs):
        assert rel_err(o.detach(), g[name]) < 1e-4, name
    for k, v in feats.items():
        assert rel_err(v.grad, g[f"ingrad_{k}"]) < 1e-4, k
    params = dict(m.named_parameters())
    for key in g.files:
        if key.startswith("pgrad_"):
            assert rel_err(params[key[6:]].grad, g[key]) < 1e-4, key


@pytest.mark.parametrize("fixture", ["decoder.npz", "decoder_q200.npz", "video_decoder.npz", "video_decoder_t5.npz"])
def test_decoder_forward_backward_cpu(fixture):
    from module_cases import DECODER_CASES, run_decoder
    from oracle.decoder_ref import torch_decoder_ops, unpack_bits
    build, video = DECODER_CASES[fixture]
    d = build()
    with torch_decoder_ops():
        g, x, mf, logits, masks, captured = run_decoder(d, torch.device("cpu"), fixture, video)
    assert rel_err(torch.stack([t.detach() for t in logits]), g["pred_logits"]) < 1e-4
    assert rel_err(torch.stack([t.detach() for t in masks]), g["pred_masks"]) < 1e-4
    for i, bits in enumerate(captured):
        want = g[f"attn_mask{i}"]
        got = unpack_bits(bits, want.shape[-1]).numpy()
        assert (got == want).all(), f"attn mask of layer {i} differs"
    for i, t in enumerate(x):
        assert rel_err(t.grad, g[f"ingrad_x{i}"]) < 1e-4
    assert rel_err(mf.grad, g["ingrad_mask_features"]) < 1e-4
    if not video:
        params = dict(d.named_parameters())
        for key in g.files:
            if key.startswith("pgrad_"):
                assert rel_err(params[key[6:]].grad, g[key]) < 1e-4, key


def test_flat_cast_leaves_unreached_parameters_without_grad():
    """The decoder's one-buffer weight cast (decoder_ops._FlatCast) returns the cast gradients of the parameters an
    output reached and None for the others (autocast's per-call casts leave those None, and AdamW skips them)."""
    from bm2f_amd.decoder_ops import _FlatCast
    a = torch.randn(3, 4, requires_grad=True)
    b = torch.randn(5, requires_grad=True)
    c = torch.randn(2, 2, requires_grad=True)
    la, lb, lc = _FlatCast.apply(torch.float16, a, b, c)
    assert la.dtype == torch.float16 and torch.equal(la, a.detach().half())
    (la.float().sum() * 2 + lc.float().pow(2).sum()).backward()
    assert b.grad is None
    torch.testing.assert_close(a.grad, torch.full_like(a, 2.0))
    torch.testing.assert_close(c.grad, (2 * c.detach().half().float()).half().float())
