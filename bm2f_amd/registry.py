"""Detectron2 surface the hot-path modules plug into.

When detectron2 is importable its real ``configurable`` / ``Conv2d`` / ``ShapeSpec`` / ``get_norm`` and
``SEM_SEG_HEADS_REGISTRY`` are used, so ``build_pixel_decoder`` (reference pixel_decoder/fpn.py:21-33) and
``build_transformer_decoder`` (transformer_decoder/maskformer_transformer_decoder.py:22-27) find the
modules exactly as they find the reference's.  The transformer-decoder registry is the reference's own
``TRANSFORMER_DECODER_REGISTRY`` object whenever its module
(``mask2former.modeling.transformer_decoder.maskformer_transformer_decoder``, :16) is loaded when a bm2f
class is defined -- as it is when the reference's ``transformer_decoder/__init__.py`` imports bm2f in place of
its own decoder.  :func:`register` replaces a same-name entry (the reference's class
registered first) instead of raising, so both import orders work.  Without detectron2 (this image) the same
names are provided here with the same calling conventions:

* ``configurable``: ``Cls(cfg, *args)`` routes through ``Cls.from_config(cfg, *args)``; explicit
  keyword construction works unchanged.
* ``Conv2d(..., norm=, activation=)``: conv -> norm -> activation (detectron2's order).
* ``Registry``: ``register()`` decorator + ``get(name)``.
"""
from __future__ import annotations

import functools
import sys
from collections import namedtuple

import torch.nn.functional as F
from torch import nn

try:  # pragma: no cover - detectron2 is absent in this image
    from detectron2.config import configurable  # type: ignore
    from detectron2.layers import Conv2d, ShapeSpec, get_norm  # type: ignore
    from detectron2.modeling import SEM_SEG_HEADS_REGISTRY  # type: ignore
    from detectron2.utils.registry import Registry  # type: ignore
    HAVE_DETECTRON2 = True
except Exception:  # noqa: BLE001
    HAVE_DETECTRON2 = False

    class Registry:
        def __init__(self, name: str):
            self._name = name
            self._obj_map = {}

        def _do_register(self, name, obj):
            if name in self._obj_map:
                raise KeyError(f"An object named '{name}' was already registered in '{self._name}' registry!")
            self._obj_map[name] = obj

        def register(self, obj=None):
            if obj is None:
                def deco(func_or_class):
                    self._do_register(func_or_class.__name__, func_or_class)
                    return func_or_class
                return deco
            self._do_register(obj.__name__, obj)
            return obj

        def get(self, name):
            if name not in self._obj_map:
                raise KeyError(f"No object named '{name}' found in '{self._name}' registry!")
            return self._obj_map[name]

        def __contains__(self, name):
            return name in self._obj_map

    def _is_cfg(x) -> bool:
        return hasattr(x, "MODEL")

    def configurable(init_func=None, *, from_config=None):
        def wrap(init):
            @functools.wraps(init)
            def wrapped(self, *args, **kwargs):
                if (args and _is_cfg(args[0])) or _is_cfg(kwargs.get("cfg")):
                    fc = type(self).from_config
                    explicit = fc(*args, **kwargs)
                    init(self, **explicit)
                else:
                    init(self, *args, **kwargs)
            return wrapped
        if init_func is not None:
            return wrap(init_func)
        return wrap

    ShapeSpec = namedtuple("ShapeSpec", ["channels", "height", "width", "stride"], defaults=[None] * 4)

    class Conv2d(nn.Conv2d):
        """nn.Conv2d + optional norm and activation, applied in detectron2's order."""

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
        if isinstance(norm, str):
            if norm != "GN":
                raise ValueError(f"norm {norm!r} is not supported by the bm2f_amd shim (only 'GN')")
            return nn.GroupNorm(32, out_channels)
        return norm(out_channels)

    SEM_SEG_HEADS_REGISTRY = Registry("SEM_SEG_HEADS")

REFERENCE_TD_MODULE = "mask2former.modeling.transformer_decoder.maskformer_transformer_decoder"

# Same name and role as mask2former/modeling/transformer_decoder/maskformer_transformer_decoder.py:16; used
# when the reference's module is not loaded
_LOCAL_TD_REGISTRY = Registry("TRANSFORMER_MODULE")


def transformer_decoder_registry():
    """The reference's TRANSFORMER_DECODER_REGISTRY if its module is loaded, else bm2f's own."""
    mod = sys.modules.get(REFERENCE_TD_MODULE)
    reg = getattr(mod, "TRANSFORMER_DECODER_REGISTRY", None) if mod is not None else None
    return reg if reg is not None else _LOCAL_TD_REGISTRY


def _entries(registry):
    # detectron2 / fvcore Registry and the local one keep their map in ``_obj_map``
    return getattr(registry, "_obj_map", None)


def register(registry_fn):
    """Class decorator: register into ``registry_fn()`` (resolved now, at class definition), replacing an
    entry of the same name -- e.g. the reference's own MSDeformAttnPixelDecoder when its module was imported
    first -- instead of raising "already registered"."""
    def deco(cls):
        _register_replacing(registry_fn(), cls)
        return cls
    return deco


def _register_replacing(registry, cls):
    entries = _entries(registry)
    if entries is not None and cls.__name__ in entries:
        entries[cls.__name__] = cls
    else:
        registry.register(cls)


def install():
    """(Re)register the bm2f classes into the registries visible now: call after importing the reference's
    modules in an order where bm2f was imported first."""
    from .pixel_decoder import MSDeformAttnPixelDecoder
    from .transformer_decoder import MultiScaleMaskedTransformerDecoder
    from .video_decoder import VideoMultiScaleMaskedTransformerDecoder
    _register_replacing(SEM_SEG_HEADS_REGISTRY, MSDeformAttnPixelDecoder)
    for cls in (MultiScaleMaskedTransformerDecoder, VideoMultiScaleMaskedTransformerDecoder):
        _register_replacing(transformer_decoder_registry(), cls)
        if transformer_decoder_registry() is not _LOCAL_TD_REGISTRY:
            _register_replacing(_LOCAL_TD_REGISTRY, cls)


def __getattr__(name):
    if name == "TRANSFORMER_DECODER_REGISTRY":
        return transformer_decoder_registry()
    raise AttributeError(name)


def build_pixel_decoder(cfg, input_shape):
    """reference pixel_decoder/fpn.py:21-33"""
    name = cfg.MODEL.SEM_SEG_HEAD.PIXEL_DECODER_NAME
    model = SEM_SEG_HEADS_REGISTRY.get(name)(cfg, input_shape)
    if not callable(getattr(model, "forward_features", None)):
        raise ValueError("Only SEM_SEG_HEADS with forward_features method can be used as pixel decoder. "
                         f"Please implement forward_features for {name} to only return mask features.")
    return model


def build_transformer_decoder(cfg, in_channels, mask_classification=True):
    """reference transformer_decoder/maskformer_transformer_decoder.py:22-27"""
    name = cfg.MODEL.MASK_FORMER.TRANSFORMER_DECODER_NAME
    return transformer_decoder_registry().get(name)(cfg, in_channels, mask_classification)


def c2_xavier_fill(module: nn.Module) -> None:
    """fvcore.nn.weight_init.c2_xavier_fill: kaiming_uniform(a=1) weights, zero bias."""
    nn.init.kaiming_uniform_(module.weight, a=1)
    if module.bias is not None:
        nn.init.constant_(module.bias, 0)


__all__ = ["Registry", "configurable", "ShapeSpec", "Conv2d", "get_norm", "SEM_SEG_HEADS_REGISTRY",
           "TRANSFORMER_DECODER_REGISTRY", "transformer_decoder_registry", "register", "install",
           "build_pixel_decoder", "build_transformer_decoder", "c2_xavier_fill", "HAVE_DETECTRON2"]
