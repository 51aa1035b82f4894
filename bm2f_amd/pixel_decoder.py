"""MSDeformAttn pixel decoder (reference mask2former/modeling/pixel_decoder/msdeformattn.py).

Same classes, constructor arguments, ``from_config`` keys, ``forward_features`` contract and state-dict
keys as the reference, so ``build_pixel_decoder`` and existing checkpoints work unchanged.  The
deformable attention runs on the gfx950 kernels (``bm2f_amd.msda``).  MI355X-side changes that do not
alter results:

* the all-False padding mask and valid ratios (msdeformattn.py:62, :84) are constants: the no-op
  ``masked_fill`` is skipped and reference points / sine embeddings are computed once per shape;
* the host copy of ``spatial_shapes`` rides along with the device tensor, so the MSDA backward can
  use its spatially tiled grad_value accumulation without a device->host sync.
"""
from __future__ import annotations

import copy
from typing import Callable, Dict, List, Optional, Union

import numpy as np
import torch
from torch import nn
from torch.nn import functional as F
from torch.nn.init import normal_

from .msda import MSDeformAttn, attach_host_shapes
from . import conv_ops, linear_ops
from .decoder_ops import row_bias_add
from .norm_ops import add_layernorm, group_norm_act
from .position_encoding import PositionEmbeddingSine
from .registry import SEM_SEG_HEADS_REGISTRY, Conv2d, ShapeSpec, c2_xavier_fill, configurable, get_norm, register


# encoder layers hand their residual inputs through the projection / FFN autograd nodes so gradient sums
# ride in GEMM epilogues (False: plain autograd sums, for A/B measurements and tests)
RESIDUAL_FUSED = True


def _get_clones(module, N):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def _get_activation_fn(activation):
    if activation == "relu":
        return F.relu
    if activation == "gelu":
        return F.gelu
    if activation == "glu":
        return F.glu
    raise RuntimeError(f"activation should be relu/gelu, not {activation}.")


class MSDeformAttnTransformerEncoderLayer(nn.Module):
    """Post-norm layer: MSDA -> add & LN -> FFN -> add & LN (msdeformattn.py:92-131)."""

    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        self.self_attn = MSDeformAttn(d_model, n_levels, n_heads, n_points)
        self.dropout1 = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.linear1 = nn.Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation)
        self.dropout2 = nn.Dropout(dropout)
        self.linear2 = nn.Linear(d_ffn, d_model)
        self.dropout3 = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(d_model)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def _add_norm(self, src, src2, dropout, norm):
        # residual + LayerNorm in one kernel when the dropout is an identity (p = 0, as configured, or eval)
        if dropout.p == 0.0 or not self.training:
            return add_layernorm(src, src2, norm)
        return norm(src + dropout(src2))

    def forward_ffn(self, src):
        if self.activation is F.relu and (self.dropout2.p == 0.0 or not self.training):
            src2 = linear_ops.ffn(src, self.linear1, self.linear2)   # bias+ReLU / ReLU mask fused in the GEMMs
        else:
            src2 = self.linear2(self.dropout2(self.activation(self.linear1(src))))
        return self._add_norm(src, src2, self.dropout3, self.norm2)

    def forward(self, src, pos, reference_points, spatial_shapes, level_start_index, padding_mask=None):
        if self._residual_fused():
            # src's three consumers (value_proj, the query, the residual) and the FFN input's two (linear1,
            # the residual) have their gradients summed inside the input-gradient GEMMs (linear_ops)
            src2, src = self.self_attn.forward_src_pos(src, pos, reference_points, spatial_shapes,
                                                       level_start_index, padding_mask)
            src = self._add_norm(src, src2, self.dropout1, self.norm1)
            src2, src = linear_ops.ffn_residual(src, self.linear1, self.linear2)
            return self._add_norm(src, src2, self.dropout3, self.norm2)
        src2 = self.self_attn(self.with_pos_embed(src, pos), reference_points, src, spatial_shapes,
                              level_start_index, padding_mask)
        src = self._add_norm(src, src2, self.dropout1, self.norm1)
        return self.forward_ffn(src)

    def _residual_fused(self):
        return (self.activation is F.relu and RESIDUAL_FUSED
                and all(d.p == 0.0 or not self.training for d in (self.dropout1, self.dropout2, self.dropout3)))


class MSDeformAttnTransformerEncoder(nn.Module):
    def __init__(self, encoder_layer, num_layers):
        super().__init__()
        self.layers = _get_clones(encoder_layer, num_layers)
        self.num_layers = num_layers
        self._ref_cache = {}

    @staticmethod
    def get_reference_points(spatial_shapes, valid_ratios, device):
        """Pixel centres normalised by the valid extent (msdeformattn.py:141-153)."""
        reference_points_list = []
        for lvl, (H_, W_) in enumerate(spatial_shapes):
            H_, W_ = int(H_), int(W_)
            ref_y, ref_x = torch.meshgrid(torch.linspace(0.5, H_ - 0.5, H_, dtype=torch.float32, device=device),
                                          torch.linspace(0.5, W_ - 0.5, W_, dtype=torch.float32, device=device),
                                          indexing="ij")
            ref_y = ref_y.reshape(-1)[None] / (valid_ratios[:, None, lvl, 1] * H_)
            ref_x = ref_x.reshape(-1)[None] / (valid_ratios[:, None, lvl, 0] * W_)
            reference_points_list.append(torch.stack((ref_x, ref_y), -1))
        reference_points = torch.cat(reference_points_list, 1)
        return reference_points[:, :, None] * valid_ratios[:, None]

    def reference_points_for(self, host_shapes, batch, device):
        key = (tuple(host_shapes), device)
        ref = self._ref_cache.get(key)
        if ref is None:
            ones = torch.ones((1, len(host_shapes), 2), dtype=torch.float32, device=device)
            with torch.no_grad():
                ref = self.get_reference_points(host_shapes, ones, device).contiguous()
            self._ref_cache[key] = ref
        return ref.expand(batch, -1, -1, -1)

    def forward(self, src, spatial_shapes, level_start_index, valid_ratios, pos=None, padding_mask=None,
                host_shapes=None):
        output = src
        if host_shapes is not None and valid_ratios is None:
            reference_points = self.reference_points_for(host_shapes, src.shape[0], src.device)
        else:
            reference_points = self.get_reference_points(
                host_shapes if host_shapes is not None else spatial_shapes.tolist(), valid_ratios, src.device)
        for layer in self.layers:
            output = layer(output, pos, reference_points, spatial_shapes, level_start_index, padding_mask)
        return output


class MSDeformAttnTransformerEncoderOnly(nn.Module):
    def __init__(self, d_model=256, nhead=8, num_encoder_layers=6, dim_feedforward=1024, dropout=0.1,
                 activation="relu", num_feature_levels=4, enc_n_points=4):
        super().__init__()
        self.d_model = d_model
        self.nhead = nhead
        encoder_layer = MSDeformAttnTransformerEncoderLayer(d_model, dim_feedforward, dropout, activation,
                                                            num_feature_levels, nhead, enc_n_points)
        self.encoder = MSDeformAttnTransformerEncoder(encoder_layer, num_encoder_layers)
        self.level_embed = nn.Parameter(torch.Tensor(num_feature_levels, d_model))
        self._reset_parameters()
        self._shape_cache = {}

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)
        for m in self.modules():
            if isinstance(m, MSDeformAttn):
                m._reset_parameters()
        normal_(self.level_embed)

    def _shapes(self, host_shapes, device):
        key = (tuple(host_shapes), device)
        hit = self._shape_cache.get(key)
        if hit is None:
            st = torch.as_tensor(host_shapes, dtype=torch.long, device=device)
            lsi = torch.cat((st.new_zeros((1,)), st.prod(1).cumsum(0)[:-1]))
            attach_host_shapes(st, host_shapes, lsi)     # checked once per shape set (cached)
            hit = (st, lsi)
            self._shape_cache[key] = hit
        return hit

    def forward(self, srcs, pos_embeds):
        """srcs / pos_embeds: lists of (N, C, H_l, W_l), coarse -> fine (msdeformattn.py:61-89)."""
        host_shapes = [(int(x.shape[2]), int(x.shape[3])) for x in srcs]
        src_flatten = conv_ops.flatten_levels(srcs)   # cat of the transposed levels, tiled transposes
        if all(p.dim() == 4 and p.stride(0) == 0 for p in pos_embeds):
            # batch-broadcast embeddings (PositionEmbeddingSine without a padding mask): keep one (1, S, C)
            # copy; the layers broadcast it, and its gradient is (1, S, C) instead of (N, S, C) per layer
            pos_embeds = [p[:1] for p in pos_embeds]
        lvl_pos_embed_flatten = torch.cat(
            [row_bias_add(p.flatten(2).transpose(1, 2), self.level_embed[lvl]) for lvl, p in enumerate(pos_embeds)],
            1)
        spatial_shapes, level_start_index = self._shapes(host_shapes, src_flatten.device)
        memory = self.encoder(src_flatten, spatial_shapes, level_start_index, None, lvl_pos_embed_flatten, None,
                              host_shapes=host_shapes)
        return memory, spatial_shapes, level_start_index


class _F32Contiguous(torch.autograd.Function):
    """``x.float()`` as a contiguous NCHW tensor in one copy (a channels_last backbone output would otherwise be
    cast, then transposed by the first conv), and the gradient handed back in x's dtype and memory layout in
    one copy (so the backbone's gradient sums see one layout)."""

    @staticmethod
    def forward(ctx, x):
        ctx.dtype = x.dtype
        ctx.cl = (x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last))
        return x.to(dtype=torch.float32, memory_format=torch.contiguous_format)

    @staticmethod
    def backward(ctx, g):
        fmt = torch.channels_last if ctx.cl else torch.contiguous_format
        return g.to(dtype=ctx.dtype, memory_format=fmt)


def _as_f32_nchw(x):
    """The reference's ``features[f].float()`` (msdeformattn.py:320, 336), contiguous NCHW."""
    if x.dtype == torch.float32 and x.is_contiguous():
        return x
    return _F32Contiguous.apply(x)


def _conv_input(x, conv):
    """The input of a conv on a backbone feature: a 16-bit feature into a 1x1 conv the x3 kernels take goes in as it
    is (they read it converted, exactly the ``.float()`` of the reference), anything else through
    :func:`_as_f32_nchw`."""
    if x.dtype in (torch.float16, torch.bfloat16) and conv_ops.eligible(x, conv):
        return x
    return _as_f32_nchw(x)


@register(lambda: SEM_SEG_HEADS_REGISTRY)
class MSDeformAttnPixelDecoder(nn.Module):
    """Deformable-encoder pixel decoder (msdeformattn.py:164-358)."""

    @configurable
    def __init__(
        self,
        input_shape: Dict[str, ShapeSpec],
        *,
        transformer_dropout: float,
        transformer_nheads: int,
        transformer_dim_feedforward: int,
        transformer_enc_layers: int,
        conv_dim: int,
        mask_dim: int,
        norm: Optional[Union[str, Callable]] = None,
        transformer_in_features: List[str],
        common_stride: int,
    ):
        super().__init__()
        transformer_input_shape = {k: v for k, v in input_shape.items() if k in transformer_in_features}
        input_shape = sorted(input_shape.items(), key=lambda x: x[1].stride)
        self.in_features = [k for k, v in input_shape]
        self.feature_strides = [v.stride for k, v in input_shape]
        self.feature_channels = [v.channels for k, v in input_shape]

        transformer_input_shape = sorted(transformer_input_shape.items(), key=lambda x: x[1].stride)
        self.transformer_in_features = [k for k, v in transformer_input_shape]
        transformer_in_channels = [v.channels for k, v in transformer_input_shape]
        self.transformer_feature_strides = [v.stride for k, v in transformer_input_shape]

        self.transformer_num_feature_levels = len(self.transformer_in_features)
        in_list = transformer_in_channels[::-1] if self.transformer_num_feature_levels > 1 else transformer_in_channels[-1:]
        self.input_proj = nn.ModuleList([
            nn.Sequential(nn.Conv2d(c, conv_dim, kernel_size=1), nn.GroupNorm(32, conv_dim)) for c in in_list])
        for proj in self.input_proj:
            nn.init.xavier_uniform_(proj[0].weight, gain=1)
            nn.init.constant_(proj[0].bias, 0)

        self.transformer = MSDeformAttnTransformerEncoderOnly(
            d_model=conv_dim, dropout=transformer_dropout, nhead=transformer_nheads,
            dim_feedforward=transformer_dim_feedforward, num_encoder_layers=transformer_enc_layers,
            num_feature_levels=self.transformer_num_feature_levels)
        self.pe_layer = PositionEmbeddingSine(conv_dim // 2, normalize=True)

        self.mask_dim = mask_dim
        self.mask_features = Conv2d(conv_dim, mask_dim, kernel_size=1, stride=1, padding=0)
        c2_xavier_fill(self.mask_features)

        self.maskformer_num_feature_levels = 3  # always use 3 scales
        self.common_stride = common_stride
        stride = min(self.transformer_feature_strides)
        self.num_fpn_levels = int(np.log2(stride) - np.log2(self.common_stride))

        lateral_convs, output_convs = [], []
        use_bias = norm == ""
        for idx, in_channels in enumerate(self.feature_channels[:self.num_fpn_levels]):
            lateral_conv = Conv2d(in_channels, conv_dim, kernel_size=1, bias=use_bias, norm=get_norm(norm, conv_dim))
            output_conv = Conv2d(conv_dim, conv_dim, kernel_size=3, stride=1, padding=1, bias=use_bias,
                                 norm=get_norm(norm, conv_dim), activation=F.relu)
            c2_xavier_fill(lateral_conv)
            c2_xavier_fill(output_conv)
            self.add_module("adapter_{}".format(idx + 1), lateral_conv)
            self.add_module("layer_{}".format(idx + 1), output_conv)
            lateral_convs.append(lateral_conv)
            output_convs.append(output_conv)
        self.lateral_convs = lateral_convs[::-1]
        self.output_convs = output_convs[::-1]

    @classmethod
    def from_config(cls, cfg, input_shape: Dict[str, ShapeSpec]):
        """Same keys as msdeformattn.py:294-312 (FFN fixed at 1024 there too)."""
        return {
            "input_shape": {k: v for k, v in input_shape.items() if k in cfg.MODEL.SEM_SEG_HEAD.IN_FEATURES},
            "conv_dim": cfg.MODEL.SEM_SEG_HEAD.CONVS_DIM,
            "mask_dim": cfg.MODEL.SEM_SEG_HEAD.MASK_DIM,
            "norm": cfg.MODEL.SEM_SEG_HEAD.NORM,
            "transformer_dropout": cfg.MODEL.MASK_FORMER.DROPOUT,
            "transformer_nheads": cfg.MODEL.MASK_FORMER.NHEADS,
            "transformer_dim_feedforward": 1024,
            "transformer_enc_layers": cfg.MODEL.SEM_SEG_HEAD.TRANSFORMER_ENC_LAYERS,
            "transformer_in_features": cfg.MODEL.SEM_SEG_HEAD.DEFORMABLE_TRANSFORMER_ENCODER_IN_FEATURES,
            "common_stride": cfg.MODEL.SEM_SEG_HEAD.COMMON_STRIDE,
        }

    def forward_features(self, features):
        # the reference runs this method with autocast disabled and upcasts to fp32 (msdeformattn.py:314,320)
        with torch.autocast(device_type="cuda", enabled=False), torch.autocast(device_type="cpu", enabled=False):
            return self._forward_features(features)

    def _forward_features(self, features):
        srcs, pos = [], []
        for idx, f in enumerate(self.transformer_in_features[::-1]):
            proj = self.input_proj[idx]
            x = _conv_input(features[f], proj[0])
            srcs.append(group_norm_act(conv_ops.conv2d(x, proj[0]), proj[1]))   # 1x1 conv (x3) + GroupNorm
            pos.append(self.pe_layer(x))

        y, spatial_shapes, level_start_index = self.transformer(srcs, pos)
        bs = y.shape[0]
        host_shapes = [(int(s.shape[2]), int(s.shape[3])) for s in srcs]
        sizes = [h * w for h, w in host_shapes]
        out = [z.transpose(1, 2).view(bs, -1, h, w) for z, (h, w) in zip(torch.split(y, sizes, dim=1), host_shapes)]

        for idx, f in enumerate(self.in_features[:self.num_fpn_levels][::-1]):
            x = _conv_input(features[f], self.lateral_convs[idx])
            cur_fpn = conv_ops.conv_norm_act(x, self.lateral_convs[idx])
            y = conv_ops.upsample_add(out[-1], cur_fpn)   # cur_fpn + bilinear resize of out[-1], one pass
            out.append(conv_ops.conv_norm_act(y, self.output_convs[idx]))

        multi_scale_features = out[:self.maskformer_num_feature_levels]
        return conv_ops.conv_norm_act(out[-1], self.mask_features), out[0], multi_scale_features
