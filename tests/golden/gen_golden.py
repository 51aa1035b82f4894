"""Generate the golden fixtures in tests/golden/*.npz by importing the REFERENCE code (this container only).

Run:  python tests/golden/gen_golden.py [--ref /root/reference]

It never runs on the GPU box and nothing under /root/reference is copied: the reference modules are
imported in place with test-only stand-ins for the third-party pieces that are absent here
(detectron2 config/layers/registry, fvcore weight_init, and an empty ``MultiScaleDeformableAttention``
module so that ``MSDeformAttn.forward`` takes its CPU fallback ``ms_deform_attn_core_pytorch``,
ops/modules/ms_deform_attn.py:116-121).  The stand-in ``Conv2d`` applies conv -> norm -> activation,
detectron2's order (msdeformattn.py:269-281 relies on it).  Weights come from tests/golden/filler.py,
so the fixtures hold only inputs and outputs.

Fixtures:
  msda_testpy.npz   the ops/test.py fixture (N=1,M=2,D=2,Lq=2,L=2,P=2, shapes [(6,4),(3,2)], seed 3,
                    test.py:24-31,34-63) in fp64 and fp32: ms_deform_attn_core_pytorch output and, for a
                    seeded grad_output, its autograd gradients.
  msda_slice.npz    production-shaped slice: shapes [[4,4],[8,8],[16,16]], S=Lq=336, N=2, M=8, D=32,
                    L=3, P=4; variant "uniform" (loc ~ U[-0.1,1.1]) and "local" (encoder-like: reference
                    point + N(0,2px) offsets); fp32 inputs; outputs/grads computed in fp64, stored as fp32.
  pixdec.npz        MSDeformAttnPixelDecoder.forward_features (msdeformattn.py:314-358) on a 64x64 image's
                    R50-shaped features, full channel widths; outputs, input grads, selected param grads.
  decoder.npz       MultiScaleMaskedTransformerDecoder.forward (mask2former_transformer_decoder.py:363-435),
                    B=2, Q=100, K=133, 3 levels (2x2,4x4,8x8), mask features 16x16; all 10 heads' outputs,
                    the attn_mask handed to every cross-attention layer (bit-exact bookkeeping), input grads.
  video_decoder.npz VideoMultiScaleMaskedTransformerDecoder (video_mask2former_transformer_decoder.py:370-461),
                    B=1 clip, T=3 frames, Q=20.
"""
from __future__ import annotations

import argparse
import importlib
import os
import sys
import types
from collections import namedtuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from filler import fill_module  # noqa: E402


# ---------------------------------------------------------------------------------------------
# stand-ins for absent third-party packages (test-only)
# ---------------------------------------------------------------------------------------------
def install_stubs():
    class Registry:
        def __init__(self, name):
            self._name, self._map = name, {}

        def register(self, obj=None):
            def deco(o):
                self._map[o.__name__] = o
                return o
            return deco(obj) if obj is not None else deco

        def get(self, name):
            return self._map[name]

    def configurable(init_func=None, *, from_config=None):
        if init_func is not None:
            return init_func
        return lambda f: f

    class Conv2d(nn.Conv2d):
        def __init__(self, *args, **kwargs):
            norm = kwargs.pop("norm", None)
            activation = kwargs.pop("activation", None)
            super().__init__(*args, **kwargs)
            self.norm = norm
            self.activation = activation

        def forward(self, x):
            x = F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
            if self.norm is not None:
                x = self.norm(x)
            if self.activation is not None:
                x = self.activation(x)
            return x

    def get_norm(norm, out_channels):
        if norm is None or norm == "":
            return None
        assert norm == "GN", norm
        return nn.GroupNorm(32, out_channels)

    ShapeSpec = namedtuple("ShapeSpec", ["channels", "height", "width", "stride"], defaults=[None] * 4)

    mods = {}
    for name in ["detectron2", "detectron2.config", "detectron2.layers", "detectron2.modeling", "detectron2.utils",
                 "detectron2.utils.registry", "fvcore", "fvcore.nn", "fvcore.nn.weight_init",
                 "MultiScaleDeformableAttention"]:
        mods[name] = types.ModuleType(name)
    mods["detectron2.config"].configurable = configurable
    mods["detectron2.layers"].Conv2d = Conv2d
    mods["detectron2.layers"].ShapeSpec = ShapeSpec
    mods["detectron2.layers"].get_norm = get_norm
    mods["detectron2.layers"].DeformConv = None
    mods["detectron2.modeling"].SEM_SEG_HEADS_REGISTRY = Registry("SEM_SEG_HEADS")
    mods["detectron2.utils.registry"].Registry = Registry
    mods["fvcore.nn.weight_init"].c2_xavier_fill = lambda m: None
    mods["fvcore.nn"].weight_init = mods["fvcore.nn.weight_init"]
    sys.modules.update(mods)
    return ShapeSpec


def import_reference(ref_root):
    ShapeSpec = install_stubs()
    sys.path.insert(0, ref_root)
    # pre-seed the package objects so their data/eval-heavy __init__.py files are not executed
    for pkg, rel in [("mask2former", "mask2former"), ("mask2former.modeling", "mask2former/modeling"),
                     ("mask2former.modeling.pixel_decoder", "mask2former/modeling/pixel_decoder"),
                     ("mask2former.modeling.transformer_decoder", "mask2former/modeling/transformer_decoder"),
                     ("mask2former_video", "mask2former_video"),
                     ("mask2former_video.modeling", "mask2former_video/modeling"),
                     ("mask2former_video.modeling.transformer_decoder",
                      "mask2former_video/modeling/transformer_decoder")]:
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(ref_root, rel)]
        sys.modules[pkg] = m
    ref = types.SimpleNamespace(ShapeSpec=ShapeSpec)
    ref.func = importlib.import_module("mask2former.modeling.pixel_decoder.ops.functions.ms_deform_attn_func")
    ref.msdeform = importlib.import_module("mask2former.modeling.pixel_decoder.msdeformattn")
    ref.dec = importlib.import_module("mask2former.modeling.transformer_decoder.mask2former_transformer_decoder")
    ref.vdec = importlib.import_module(
        "mask2former_video.modeling.transformer_decoder.video_mask2former_transformer_decoder")
    return ref


def npf(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------------------------------------
def gen_msda_testpy(ref, out):
    core = ref.func.ms_deform_attn_core_pytorch
    N, M, D, Lq, L, P = 1, 2, 2, 2, 2, 2
    shapes = torch.as_tensor([(6, 4), (3, 2)], dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(sum(h * w for h, w in shapes.tolist()))
    torch.manual_seed(3)  # test.py:31; CPU rand then .cuda() in test.py, so these are its exact inputs
    res = {"shapes": shapes.numpy(), "level_start_index": lsi.numpy()}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        value = torch.rand(N, S, M, D) * 0.01
        loc = torch.rand(N, Lq, M, L, P, 2)
        attn = torch.rand(N, Lq, M, L, P) + 1e-5
        attn /= attn.sum(-1, keepdim=True).sum(-2, keepdim=True)
        v, lo, a = (x.to(dt).requires_grad_() for x in (value, loc, attn))
        o = core(v, shapes, lo, a)
        g = torch.rand(o.shape, generator=torch.Generator().manual_seed(11), dtype=torch.float64).to(dt)
        o.backward(g)
        res.update({f"{tag}_value": npf(v), f"{tag}_loc": npf(lo), f"{tag}_attn": npf(a), f"{tag}_out": npf(o),
                    f"{tag}_grad_out": npf(g), f"{tag}_grad_value": npf(v.grad), f"{tag}_grad_loc": npf(lo.grad),
                    f"{tag}_grad_attn": npf(a.grad)})
    np.savez_compressed(os.path.join(out, "msda_testpy.npz"), **res)


def gen_msda_slice(ref, out):
    core = ref.func.ms_deform_attn_core_pytorch
    N, M, D, L, P = 2, 8, 32, 3, 4
    shapes = torch.as_tensor([[4, 4], [8, 8], [16, 16]], dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(shapes.prod(1).sum())
    Lq = S
    gen = torch.Generator().manual_seed(2024)
    res = {"shapes": shapes.numpy(), "level_start_index": lsi.numpy()}
    # reference points of a flattened pyramid (msdeformattn.py:141-153 with valid ratio 1)
    refs = []
    for h, w in shapes.tolist():
        ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h), torch.linspace(0.5, w - 0.5, w), indexing="ij")
        refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
    refp = torch.cat(refs, 0)  # (S, 2)
    norm = torch.stack([shapes[:, 1], shapes[:, 0]], -1).float()  # (L, 2) = (W, H)
    for variant in ("uniform", "local"):
        value = torch.randn(N, S, M, D, generator=gen)
        if variant == "uniform":
            loc = torch.rand(N, Lq, M, L, P, 2, generator=gen) * 1.2 - 0.1
        else:
            off = torch.randn(N, Lq, M, L, P, 2, generator=gen) * 2.0
            loc = refp[None, :, None, None, None, :] + off / norm[None, None, None, :, None, :]
        logits = torch.randn(N, Lq, M, L * P, generator=gen)
        attn = logits.softmax(-1).view(N, Lq, M, L, P)
        gout = torch.randn(N, Lq, M * D, generator=gen)
        v, lo, a = (x.double().requires_grad_() for x in (value, loc, attn))
        o = core(v, shapes, lo, a)
        o.backward(gout.double())
        f32 = lambda t: npf(t).astype(np.float32)  # noqa: E731  (fp64-computed, stored rounded to fp32)
        res.update({f"{variant}_value": npf(value), f"{variant}_loc": npf(loc), f"{variant}_attn": npf(attn),
                    f"{variant}_grad_out": npf(gout), f"{variant}_out": f32(o), f"{variant}_grad_value": f32(v.grad),
                    f"{variant}_grad_loc": f32(lo.grad), f"{variant}_grad_attn": f32(a.grad)})
    np.savez_compressed(os.path.join(out, "msda_slice.npz"), **res)


PIXDEC_PARAM_GRADS = [
    "input_proj.2.1.weight", "input_proj.0.0.bias", "transformer.level_embed",
    "transformer.encoder.layers.0.self_attn.sampling_offsets.weight",
    "transformer.encoder.layers.0.self_attn.attention_weights.weight",
    "transformer.encoder.layers.0.self_attn.value_proj.weight",
    "transformer.encoder.layers.5.norm2.weight", "adapter_1.weight", "layer_1.norm.weight", "mask_features.weight",
]


def gen_pixdec(ref, out):
    S = ref.ShapeSpec
    input_shape = {"res2": S(channels=256, stride=4), "res3": S(channels=512, stride=8),
                   "res4": S(channels=1024, stride=16), "res5": S(channels=2048, stride=32)}
    torch.manual_seed(0)
    m = ref.msdeform.MSDeformAttnPixelDecoder(
        input_shape, transformer_dropout=0.0, transformer_nheads=8, transformer_dim_feedforward=1024,
        transformer_enc_layers=6, conv_dim=256, mask_dim=256, norm="GN",
        transformer_in_features=["res3", "res4", "res5"], common_stride=4)
    fill_module(m)
    m.train()
    img = 64
    gen = torch.Generator().manual_seed(7)
    feats = {k: torch.randn(1, s.channels, img // s.stride, img // s.stride, generator=gen).requires_grad_()
             for k, s in input_shape.items()}
    mask_features, out0, ms = m.forward_features(feats)
    outs = [mask_features, out0] + list(ms)
    grads = [torch.randn(o.shape, generator=gen) for o in outs]
    torch.autograd.backward(outs, grads)
    pnames = dict(m.named_parameters())
    res = {f"in_{k}": npf(v) for k, v in feats.items()}
    res.update({f"ingrad_{k}": npf(v.grad) for k, v in feats.items()})
    res.update({"out_mask_features": npf(mask_features), "out_out0": npf(out0)})
    res.update({f"out_ms{i}": npf(t) for i, t in enumerate(ms)})
    res.update({f"outgrad_{i}": npf(g) for i, g in enumerate(grads)})
    res.update({f"pgrad_{k}": npf(pnames[k].grad) for k in PIXDEC_PARAM_GRADS})
    res["state_dict_keys"] = np.array(sorted(k for k in m.state_dict().keys()))
    np.savez_compressed(os.path.join(out, "pixdec.npz"), **res)


def _capture_masks(dec):
    captured = []

    def hook(mod, args, kwargs):
        captured.append(kwargs["memory_mask"].clone())

    handles = [layer.register_forward_pre_hook(hook, with_kwargs=True)
               for layer in dec.transformer_cross_attention_layers]
    return captured, handles


DEC_PARAM_GRADS = [
    "query_feat.weight", "query_embed.weight", "level_embed.weight", "class_embed.weight",
    "mask_embed.layers.2.weight", "transformer_cross_attention_layers.0.multihead_attn.in_proj_bias",
    "transformer_cross_attention_layers.8.multihead_attn.out_proj.weight",
    "transformer_self_attention_layers.4.self_attn.in_proj_bias", "transformer_ffn_layers.3.linear2.bias",
    "decoder_norm.weight",
]


def gen_decoder(ref, out, num_queries=100, num_classes=133, name="decoder.npz", amp=None):
    """amp: None (fp32) or torch.float16 -- the reference's training precision (SOLVER.AMP.ENABLED), run
    under CPU autocast here."""
    torch.manual_seed(0)
    dec = ref.dec.MultiScaleMaskedTransformerDecoder(
        256, True, num_classes=num_classes, hidden_dim=256, num_queries=num_queries, nheads=8, dim_feedforward=2048,
        dec_layers=9, pre_norm=False, mask_dim=256, enforce_input_project=False)
    fill_module(dec)
    dec.train()
    gen = torch.Generator().manual_seed(5)
    B = 2
    x = [torch.randn(B, 256, s, s, generator=gen).requires_grad_() for s in (2, 4, 8)]
    mf = torch.randn(B, 256, 16, 16, generator=gen).requires_grad_()
    captured, handles = _capture_masks(dec)
    with torch.autocast("cpu", dtype=amp or torch.float32, enabled=amp is not None):
        o = dec(x, mf)
    for h in handles:
        h.remove()
    logits = [a["pred_logits"] for a in o["aux_outputs"]] + [o["pred_logits"]]
    masks = [a["pred_masks"] for a in o["aux_outputs"]] + [o["pred_masks"]]
    loss = sum(l.float().mean() + 0.5 * (mk.float() ** 2).mean() for l, mk in zip(logits, masks))
    loss.backward()
    pnames = dict(dec.named_parameters())
    res = {f"in_x{i}": npf(t) for i, t in enumerate(x)}
    res["in_mask_features"] = npf(mf)
    res.update({f"ingrad_x{i}": npf(t.grad) for i, t in enumerate(x)})
    res["ingrad_mask_features"] = npf(mf.grad)
    res["pred_logits"] = np.stack([npf(t.float()) for t in logits])
    res["pred_masks"] = np.stack([npf(t.float()) for t in masks])
    # attn_mask handed to cross-attn layer i, (B*h, Q, HW) bool; heads are identical copies -> keep head 0
    for i, mk in enumerate(captured):
        bq = mk.view(B, 8, mk.shape[1], mk.shape[2])
        assert torch.equal(bq, bq[:, :1].expand_as(bq))
        res[f"attn_mask{i}"] = npf(bq[:, 0])
    res.update({f"pgrad_{k}": npf(pnames[k].grad) for k in DEC_PARAM_GRADS})
    res["state_dict_keys"] = np.array(sorted(dec.state_dict().keys()))
    np.savez_compressed(os.path.join(out, name), **res)


def gen_decoder_q200(ref, out):
    """Config 4's decoder shape (COCO instance, Swin-L: Q=200, K=80), reduced spatial size."""
    gen_decoder(ref, out, num_queries=200, num_classes=80, name="decoder_q200.npz")


def gen_decoder_amp16(ref, out):
    """The decoder under fp16 autocast, the reference's training precision."""
    gen_decoder(ref, out, name="decoder_amp16.npz", amp=torch.float16)


def gen_video_decoder(ref, out, T=3, B=1, num_queries=20, levels=((2, 3), (4, 5), (8, 9)), mf_hw=(16, 18),
                      name="video_decoder.npz"):
    torch.manual_seed(0)
    dec = ref.vdec.VideoMultiScaleMaskedTransformerDecoder(
        256, True, num_classes=40, hidden_dim=256, num_queries=num_queries, nheads=8, dim_feedforward=2048,
        dec_layers=9, pre_norm=False, mask_dim=256, enforce_input_project=False, num_frames=T)
    fill_module(dec)
    dec.train()
    gen = torch.Generator().manual_seed(9)
    x = [torch.randn(B * T, 256, h, w, generator=gen).requires_grad_() for h, w in levels]
    mf = torch.randn(B * T, 256, *mf_hw, generator=gen).requires_grad_()
    captured, handles = _capture_masks(dec)
    o = dec(x, mf)
    for h in handles:
        h.remove()
    logits = [a["pred_logits"] for a in o["aux_outputs"]] + [o["pred_logits"]]
    masks = [a["pred_masks"] for a in o["aux_outputs"]] + [o["pred_masks"]]
    loss = sum(l.mean() + 0.5 * (mk ** 2).mean() for l, mk in zip(logits, masks))
    loss.backward()
    res = {f"in_x{i}": npf(t) for i, t in enumerate(x)}
    res["in_mask_features"] = npf(mf)
    res.update({f"ingrad_x{i}": npf(t.grad) for i, t in enumerate(x)})
    res["ingrad_mask_features"] = npf(mf.grad)
    res["pred_logits"] = np.stack([npf(t) for t in logits])
    res["pred_masks"] = np.stack([npf(t) for t in masks])
    for i, mk in enumerate(captured):
        bq = mk.view(B, 8, mk.shape[1], mk.shape[2])
        res[f"attn_mask{i}"] = npf(bq[:, 0])
    res["state_dict_keys"] = np.array(sorted(dec.state_dict().keys()))
    np.savez_compressed(os.path.join(out, name), **res)


def gen_video_decoder_t5(ref, out):
    """Config 5's clip layout (youtubevis_2019: T=5 frames, 384x640 -> a non-square 3:5 pyramid) at 1/4 of its
    spatial size: levels 3x5 / 6x10 / 12x20, mask features 12x20; one clip, Q=20 (fixture size)."""
    gen_video_decoder(ref, out, T=5, B=1, num_queries=20, levels=((3, 5), (6, 10), (12, 20)), mf_hw=(12, 20),
                      name="video_decoder_t5.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref = import_reference(args.ref)
    for fn in (gen_msda_testpy, gen_msda_slice, gen_pixdec, gen_decoder, gen_decoder_q200, gen_decoder_amp16,
               gen_video_decoder, gen_video_decoder_t5):
        if args.only and args.only not in fn.__name__:
            continue
        fn(ref, args.out)
        print("wrote", fn.__name__)


if __name__ == "__main__":
    main()
