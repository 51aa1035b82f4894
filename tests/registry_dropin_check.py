"""Drop-in check of INTEGRATION.md §2, run in a fresh interpreter by tests/test_registry_dropin.py (CPU, this
container only: it imports the reference from /root/reference, which never travels to the GPU box).

The order is the one the documented recipe produces: the reference's registry module
(maskformer_transformer_decoder.py:16) and its own decoder / pixel decoder register first, then bm2f's
classes are imported -- as the edited ``__init__.py`` files would import them -- and replace those entries.
Then the reference's OWN builders, ``build_pixel_decoder`` (pixel_decoder/fpn.py:21-33) and
``build_transformer_decoder`` (maskformer_transformer_decoder.py:22-27), are called with a config; they must
return the bm2f classes.  A reference module's state_dict (filled by tests/golden/filler.py, as the fixtures
were made) loads strictly into each, and the outputs match the reference's golden fixtures on CPU (the
oracle's MSDA / decoder restatements stand in for the HIP kernels here).

Stand-ins for the absent detectron2 / fvcore mirror their behaviour where the check depends on it: the
registry raises on a duplicate name like detectron2's Registry, and ``configurable`` routes a cfg through
``from_config``.
"""
import functools
import os
import sys
import types
from collections import namedtuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE, os.path.join(HERE, "golden")]


def install_detectron2_standins():
    class Registry:
        def __init__(self, name):
            self._name, self._obj_map = name, {}

        def _do_register(self, name, obj):
            if name in self._obj_map:  # detectron2/fvcore Registry behaviour
                raise AssertionError(f"An object named '{name}' was already registered in '{self._name}' registry!")
            self._obj_map[name] = obj

        def register(self, obj=None):
            if obj is None:
                def deco(o):
                    self._do_register(o.__name__, o)
                    return o
                return deco
            self._do_register(obj.__name__, obj)
            return obj

        def get(self, name):
            return self._obj_map[name]

    def configurable(init_func=None, *, from_config=None):
        def wrap(init):
            @functools.wraps(init)
            def wrapped(self, *args, **kwargs):
                if args and hasattr(args[0], "MODEL"):
                    init(self, **type(self).from_config(*args, **kwargs))
                else:
                    init(self, *args, **kwargs)
            return wrapped
        return wrap(init_func) if init_func is not None else wrap

    class Conv2d(nn.Conv2d):
        def __init__(self, *args, **kwargs):
            norm, activation = kwargs.pop("norm", None), kwargs.pop("activation", None)
            super().__init__(*args, **kwargs)
            self.norm, self.activation = norm, activation

        def forward(self, x):
            x = F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
            if self.norm is not None:
                x = self.norm(x)
            if self.activation is not None:
                x = self.activation(x)
            return x

    def get_norm(norm, out_channels):
        return None if not norm else nn.GroupNorm(32, out_channels)

    ShapeSpec = namedtuple("ShapeSpec", ["channels", "height", "width", "stride"], defaults=[None] * 4)
    mods = {n: types.ModuleType(n) for n in [
        "detectron2", "detectron2.config", "detectron2.layers", "detectron2.modeling", "detectron2.utils",
        "detectron2.utils.registry", "fvcore", "fvcore.nn", "fvcore.nn.weight_init"]}
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


def main(ref_root):
    ShapeSpec = install_detectron2_standins()
    # bm2f's module stands in for the compiled MultiScaleDeformableAttention
    import bm2f_amd.msda
    sys.modules["MultiScaleDeformableAttention"] = bm2f_amd.msda
    sys.path.insert(0, ref_root)
    for pkg, rel in [("mask2former", "mask2former"), ("mask2former.modeling", "mask2former/modeling"),
                     ("mask2former.modeling.pixel_decoder", "mask2former/modeling/pixel_decoder"),
                     ("mask2former.modeling.transformer_decoder", "mask2former/modeling/transformer_decoder")]:
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(ref_root, rel)]
        sys.modules[pkg] = m
    import importlib
    td = importlib.import_module("mask2former.modeling.transformer_decoder.maskformer_transformer_decoder")
    ref_dec = importlib.import_module("mask2former.modeling.transformer_decoder.mask2former_transformer_decoder")
    ref_pd = importlib.import_module("mask2former.modeling.pixel_decoder.msdeformattn")
    fpn = importlib.import_module("mask2former.modeling.pixel_decoder.fpn")
    RefDecoder, RefPixdec = ref_dec.MultiScaleMaskedTransformerDecoder, ref_pd.MSDeformAttnPixelDecoder
    assert td.TRANSFORMER_DECODER_REGISTRY.get("MultiScaleMaskedTransformerDecoder") is RefDecoder

    # the edited __init__.py files import bm2f's classes here
    from bm2f_amd.pixel_decoder import MSDeformAttnPixelDecoder
    from bm2f_amd.transformer_decoder import MultiScaleMaskedTransformerDecoder
    from bm2f_amd.bench_model import default_cfg

    cfg = default_cfg()
    shapes = {"res2": ShapeSpec(channels=256, stride=4), "res3": ShapeSpec(channels=512, stride=8),
              "res4": ShapeSpec(channels=1024, stride=16), "res5": ShapeSpec(channels=2048, stride=32)}
    pd = fpn.build_pixel_decoder(cfg, shapes)                       # the reference's own builder
    dec = td.build_transformer_decoder(cfg, 256, mask_classification=True)
    assert type(pd) is MSDeformAttnPixelDecoder, type(pd)
    assert type(dec) is MultiScaleMaskedTransformerDecoder, type(dec)

    from filler import fill_module
    from module_cases import oracle_msda, rel_err, run_decoder, run_pixdec
    from oracle.decoder_ref import torch_decoder_ops
    torch.manual_seed(0)
    ref_m = fill_module(RefPixdec(shapes, transformer_dropout=0.0, transformer_nheads=8,
                                  transformer_dim_feedforward=1024, transformer_enc_layers=6, conv_dim=256,
                                  mask_dim=256, norm="GN", transformer_in_features=["res3", "res4", "res5"],
                                  common_stride=4))
    pd.load_state_dict(ref_m.state_dict(), strict=True)
    pd.train()
    with oracle_msda():
        g, feats, outs = run_pixdec(pd, torch.device("cpu"))
    for name, o in zip(["out_mask_features", "out_out0", "out_ms0", "out_ms1", "out_ms2"], outs):
        assert rel_err(o.detach(), g[name]) < 1e-4, name

    ref_d = fill_module(RefDecoder(256, True, num_classes=133, hidden_dim=256, num_queries=100, nheads=8,
                                   dim_feedforward=2048, dec_layers=9, pre_norm=False, mask_dim=256,
                                   enforce_input_project=False))
    dec.load_state_dict(ref_d.state_dict(), strict=True)
    dec.train()
    with torch_decoder_ops():
        g, x, mf, logits, masks, _ = run_decoder(dec, torch.device("cpu"), "decoder.npz", False)
    assert rel_err(torch.stack([t.detach() for t in logits]), g["pred_logits"]) < 1e-4
    assert rel_err(torch.stack([t.detach() for t in masks]), g["pred_masks"]) < 1e-4
    print("registry drop-in ok")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
