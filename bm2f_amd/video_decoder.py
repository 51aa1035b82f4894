"""Spatio-temporal masked-attention decoder (reference
mask2former_video/modeling/transformer_decoder/video_mask2former_transformer_decoder.py:208-474).

Identical to the image decoder except for the memory (T*HW_l tokens per level, frame-major,
:390-393), the 3-D sine embedding, and the per-frame mask einsum ``bqc,btchw->bqthw`` (:449) whose
resize runs per frame (:453-458) — the bitmask kernel takes the T frames of a row at once.
"""
from __future__ import annotations

import torch
from torch import nn

from . import decoder_ops
from .position_encoding import PositionEmbeddingSine3D
from .registry import configurable, register, transformer_decoder_registry
from .transformer_decoder import MultiScaleMaskedTransformerDecoder


@register(transformer_decoder_registry)
class VideoMultiScaleMaskedTransformerDecoder(MultiScaleMaskedTransformerDecoder):
    _version = 2

    @configurable
    def __init__(self, in_channels, mask_classification=True, *, num_classes: int, hidden_dim: int,
                 num_queries: int, nheads: int, dim_feedforward: int, dec_layers: int, pre_norm: bool,
                 mask_dim: int, enforce_input_project: bool, num_frames):
        super().__init__(in_channels, mask_classification, num_classes=num_classes, hidden_dim=hidden_dim,
                         num_queries=num_queries, nheads=nheads, dim_feedforward=dim_feedforward,
                         dec_layers=dec_layers, pre_norm=pre_norm, mask_dim=mask_dim,
                         enforce_input_project=enforce_input_project)
        self.num_frames = num_frames
        self.pe_layer = PositionEmbeddingSine3D(hidden_dim // 2, normalize=True)

    @classmethod
    def from_config(cls, cfg, in_channels, mask_classification):
        ret = MultiScaleMaskedTransformerDecoder.from_config(cfg, in_channels, mask_classification)
        ret["num_frames"] = cfg.INPUT.SAMPLING_FRAME_NUM
        return ret

    def forward(self, x, mask_features, mask=None):
        with decoder_ops.lowp_scope(self):
            return self._forward(x, mask_features, mask)

    def _forward(self, x, mask_features, mask=None):
        bt, c_m, h_m, w_m = mask_features.shape
        bs = bt // self.num_frames if self.training else 1
        t = bt // bs
        mask_features = mask_features.view(bs, t, c_m, h_m, w_m)
        assert len(x) == self.num_feature_levels
        del mask
        src, pos, key, size_list = [], [], [], []
        for i in range(self.num_feature_levels):
            h, w = x[i].shape[-2:]
            size_list.append((h, w))
            p = self.pe_layer(x[i].view(bs, t, -1, h, w), None).flatten(3)  # (bs, t, c, hw)
            s = decoder_ops.chan_bias_add(self.input_proj[i](x[i]).flatten(2), self.level_embed.weight[i])  # (bt, c, hw)
            c = s.shape[1]
            # (bs, t, c, hw) -> (bs, t*hw, c): frame-major keys, as (T*HW, B, C) in the reference
            p = p.permute(0, 1, 3, 2).reshape(bs, t * h * w, c)
            s = s.view(bs, t, c, h * w).permute(0, 1, 3, 2).reshape(bs, t * h * w, c)
            src.append(s)
            pos.append(p)
            key.append(s + p)

        query_embed = self.query_embed.weight.unsqueeze(0).expand(bs, -1, -1)
        output = self.query_feat.weight.unsqueeze(0).repeat(bs, 1, 1)
        mf_lp = self._lowp_features(mask_features).detach().transpose(1, 2).reshape(bs, c_m, t * h_m * w_m)
        # (B, C, T*H*W) gradient -> (B, T, C, H, W)
        fold = decoder_ops.MaskFeatureFold(
            mask_features, mf_lp, (t, h_m, w_m),
            lambda df, shape: df.view(shape[0], shape[2], shape[1], shape[3], shape[4]).transpose(1, 2))

        predictions_class, predictions_mask = [], []
        outputs_class, outputs_mask, attn_mask = self._heads(output, fold, size_list[0])
        predictions_class.append(outputs_class)
        predictions_mask.append(outputs_mask)
        for i in range(self.num_layers):
            li = i % self.num_feature_levels
            output = self.transformer_cross_attention_layers[i](
                output, src[li], memory_mask=attn_mask, memory_key_padding_mask=None, pos=pos[li],
                query_pos=query_embed, memory_plus_pos=key[li])
            output = self.transformer_self_attention_layers[i](output, tgt_mask=None, tgt_key_padding_mask=None,
                                                               query_pos=query_embed)
            output = self.transformer_ffn_layers[i](output)
            outputs_class, outputs_mask, attn_mask = self._heads(
                output, fold, size_list[(i + 1) % self.num_feature_levels],
                need_mask=i < self.num_layers - 1)
            predictions_class.append(outputs_class)
            predictions_mask.append(outputs_mask)
        assert len(predictions_class) == self.num_layers + 1
        return {
            "pred_logits": predictions_class[-1],
            "pred_masks": predictions_mask[-1],
            "aux_outputs": self._set_aux_loss(predictions_class if self.mask_classification else None,
                                              predictions_mask),
        }

    def _heads(self, output, fold, size, need_mask=True):
        decoder_output = self.decoder_norm(output)
        outputs_class = decoder_ops.linear(decoder_output, self.class_embed)
        mask_embed = self.mask_embed(decoder_output)
        # (b, q, t, h, w): einsum "bqc,btchw->bqthw" (:449) and the per-frame resized bitmask (:453-458)
        outputs_mask, attn_mask = decoder_ops.mask_heads(fold, mask_embed, size if need_mask else None)
        return outputs_class, outputs_mask, attn_mask
