"""Shared builders for module-level parity tests (CPU with the oracle MSDA patched in, or GPU)."""
import contextlib

import numpy as np
import torch

from conftest import golden
from filler import fill_module

PIXDEC_SHAPES = {"res2": (256, 4), "res3": (512, 8), "res4": (1024, 16), "res5": (2048, 32)}


def build_pixdec():
    from bm2f_amd.pixel_decoder import MSDeformAttnPixelDecoder
    from bm2f_amd.registry import ShapeSpec
    shape = {k: ShapeSpec(channels=c, stride=s) for k, (c, s) in PIXDEC_SHAPES.items()}
    m = MSDeformAttnPixelDecoder(shape, transformer_dropout=0.0, transformer_nheads=8, transformer_dim_feedforward=1024,
                                 transformer_enc_layers=6, conv_dim=256, mask_dim=256, norm="GN",
                                 transformer_in_features=["res3", "res4", "res5"], common_stride=4)
    return fill_module(m).train()


def build_decoder(num_queries=100, num_classes=133):
    from bm2f_amd.transformer_decoder import MultiScaleMaskedTransformerDecoder
    d = MultiScaleMaskedTransformerDecoder(256, True, num_classes=num_classes, hidden_dim=256, num_queries=num_queries,
                                           nheads=8, dim_feedforward=2048, dec_layers=9, pre_norm=False, mask_dim=256,
                                           enforce_input_project=False)
    return fill_module(d).train()


def build_video_decoder(T=3, num_queries=20):
    from bm2f_amd.video_decoder import VideoMultiScaleMaskedTransformerDecoder
    d = VideoMultiScaleMaskedTransformerDecoder(256, True, num_classes=40, hidden_dim=256, num_queries=num_queries,
                                                nheads=8, dim_feedforward=2048, dec_layers=9, pre_norm=False,
                                                mask_dim=256, enforce_input_project=False, num_frames=T)
    return fill_module(d).train()


# decoder fixtures (tests/golden/gen_golden.py): name -> (builder, video)
DECODER_CASES = {
    "decoder.npz": (lambda: build_decoder(), False),
    "decoder_q200.npz": (lambda: build_decoder(num_queries=200, num_classes=80), False),     # config 4 shape
    "video_decoder.npz": (lambda: build_video_decoder(T=3), True),
    "video_decoder_t5.npz": (lambda: build_video_decoder(T=5), True),                        # config 5 layout
}


@contextlib.contextmanager
def oracle_msda():
    """Route MSDeformAttnFunction through the oracle's CPU core (tests only)."""
    from bm2f_amd import msda
    from oracle.msda_ref import core_pytorch

    orig = msda.MSDeformAttnFunction.apply

    def fake(value, shapes, lsi, loc, attn, step):
        return core_pytorch(value, shapes.cpu(), loc, attn)

    msda.MSDeformAttnFunction.apply = staticmethod(fake)
    try:
        yield
    finally:
        msda.MSDeformAttnFunction.apply = orig


def run_pixdec(m, device):
    g = golden("pixdec.npz")
    feats = {k: torch.from_numpy(g[f"in_{k}"]).to(device).requires_grad_() for k in PIXDEC_SHAPES}
    mf, o0, ms = m.forward_features(feats)
    outs = [mf, o0] + list(ms)
    grads = [torch.from_numpy(g[f"outgrad_{i}"]).to(device) for i in range(len(outs))]
    torch.autograd.backward(outs, grads)
    return g, feats, outs


def rel_err(got, want):
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    return np.abs(got - want).max() / max(np.abs(want).max(), 1e-30)


def run_decoder(d, device, fixture="decoder.npz", video=False):
    g = golden(fixture)
    x = [torch.from_numpy(g[f"in_x{i}"]).to(device).requires_grad_() for i in range(3)]
    mf = torch.from_numpy(g["in_mask_features"]).to(device).requires_grad_()
    captured = []
    for layer in d.transformer_cross_attention_layers:
        layer.register_forward_pre_hook(lambda m, a, kw: captured.append(kw["memory_mask"].clone()),
                                        with_kwargs=True)
    o = d(x, mf)
    logits = [a["pred_logits"] for a in o["aux_outputs"]] + [o["pred_logits"]]
    masks = [a["pred_masks"] for a in o["aux_outputs"]] + [o["pred_masks"]]
    loss = sum(lg.float().mean() + 0.5 * (mk.float() ** 2).mean() for lg, mk in zip(logits, masks))
    loss.backward()
    return g, x, mf, logits, masks, captured
