"""The teacher-forced decoder-parity harness (tests/decoder_parity.py) on CPU at a small size: with the restatements
standing in for the HIP path, every tensor must pass its bars, the forced run must reproduce the fp32 reference
exactly, and a deliberately wrong run must fail them (the harness can fail)."""
import torch

from decoder_parity import decoder_parity


def _small_decoder(q=20, k=10, video_frames=None):
    if video_frames:
        from bm2f_amd.video_decoder import VideoMultiScaleMaskedTransformerDecoder
        return VideoMultiScaleMaskedTransformerDecoder(256, True, num_classes=k, hidden_dim=256, num_queries=q,
                                                       nheads=8, dim_feedforward=512, dec_layers=3, pre_norm=False,
                                                       mask_dim=256, enforce_input_project=False,
                                                       num_frames=video_frames)
    from bm2f_amd.transformer_decoder import MultiScaleMaskedTransformerDecoder
    return MultiScaleMaskedTransformerDecoder(256, True, num_classes=k, hidden_dim=256, num_queries=q, nheads=8,
                                              dim_feedforward=512, dec_layers=3, pre_norm=False, mask_dim=256,
                                              enforce_input_project=False)


def test_decoder_parity_harness_cpu():
    torch.manual_seed(0)
    dec = _small_decoder()
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(2, 256, h, h, generator=g) for h in (4, 8, 16)]
    mf = torch.randn(2, 256, 32, 32, generator=g)
    lines, bad, n_bits, n_diff = decoder_parity(dec, xs, mf, "cpu", hip=False)
    assert not bad, "\n".join(lines)
    assert n_bits > 0 and n_diff >= 0
    assert any(k.startswith("pgrad_") for k in (ln.split()[0] for ln in lines))


def test_decoder_parity_harness_video_cpu():
    torch.manual_seed(0)
    T = 2
    dec = _small_decoder(video_frames=T)
    g = torch.Generator().manual_seed(4)
    xs = [torch.randn(2 * T, 256, h, w, generator=g) for h, w in ((3, 5), (6, 10), (12, 20))]
    mf = torch.randn(2 * T, 256, 24, 40, generator=g)
    lines, bad, n_bits, _ = decoder_parity(dec, xs, mf, "cpu", hip=False)
    assert not bad, "\n".join(lines)
    assert n_bits > 0


def test_decoder_parity_harness_detects_a_wrong_path(monkeypatch):
    """A masked attention that drops one head's scale factor must fail the bars."""
    from oracle import decoder_ref
    torch.manual_seed(0)
    dec = _small_decoder()
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(2, 256, h, h, generator=g) for h in (4, 8, 16)]
    mf = torch.randn(2, 256, 32, 32, generator=g)
    real = decoder_ref.ref_masked_attention
    calls = {"n": 0}

    def skewed(q, k, v, blocked, num_heads, scale=None):
        calls["n"] += 1
        out = real(q, k, v, blocked, num_heads, scale)
        return out * 1.01 if q.dtype == torch.float32 and calls["n"] > 9 else out   # the last run only
    monkeypatch.setattr(decoder_ref, "ref_masked_attention", skewed)
    _, bad, _, _ = decoder_parity(dec, xs, mf, "cpu", hip=False)
    assert bad
