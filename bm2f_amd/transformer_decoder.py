"""Masked-attention transformer decoder (reference
mask2former/modeling/transformer_decoder/mask2former_transformer_decoder.py).

Same class names, constructor / ``from_config`` arguments, forward contract and state-dict keys as the
reference (``nn.MultiheadAttention`` sub-modules are kept as parameter holders so checkpoints load).
What runs differs, not what is computed:

* tensors stay batch-first ``(B, L, C)`` internally (the reference permutes to ``(L, B, C)``);
* the attention mask is a per-(b, q, pixel) bitmask from :func:`decoder_ops.attn_mask_bits`
  (resize + ``sigmoid() < 0.5`` + fully-masked-row fix in one kernel, shared by all heads);
* cross-attention runs :class:`decoder_ops.MaskedAttention` (flash style HIP kernels) between the
  in/out projections; the 10 mask einsums reuse one low-precision copy of ``mask_features``;
* positional encodings / ``mem + pos`` per level are computed once per forward;
* the last prediction head's attention mask, which the reference computes and discards, is skipped.
"""
from __future__ import annotations

import logging
import math
from typing import Optional

import torch
from torch import Tensor, nn
from torch.nn import functional as F

from . import decoder_ops
from .position_encoding import PositionEmbeddingSine
from .registry import Conv2d, c2_xavier_fill, configurable, register, transformer_decoder_registry


def _get_activation_fn(activation):
    if activation == "relu":
        return F.relu
    if activation == "gelu":
        return F.gelu
    if activation == "glu":
        return F.glu
    raise RuntimeError(f"activation should be relu/gelu, not {activation}.")


class SelfAttentionLayer(nn.Module):
    """Self-attention over the queries (reference :17-72); batch-first tensors (B, Q, C)."""

    def __init__(self, d_model, nhead, dropout=0.0, activation="relu", normalize_before=False):
        super().__init__()
        self.self_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout)
        self.norm = nn.LayerNorm(d_model)
        self.dropout = nn.Dropout(dropout)
        self.activation = _get_activation_fn(activation)
        self.normalize_before = normalize_before
        self._reset_parameters()

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def _attend(self, q_in, v_in):
        a = self.self_attn
        B, L, C = q_in.shape
        H = a.num_heads
        w, b = decoder_ops.lp(a.in_proj_weight), decoder_ops.lp(a.in_proj_bias)
        # split, not slices: the in-projection's gradient is then one cat of the pieces (SplitBackward) instead of
        # a zero-filled full-size tensor per slice, added up
        (w_qk, w_v), (b_qk, b_v) = w.split([2 * C, C]), (b.split([2 * C, C]) if b is not None else (None, None))
        qk = F.linear(q_in, w_qk, b_qk)
        v = F.linear(v_in, w_v, b_v)
        q, k = qk.split(C, dim=-1)
        heads = lambda t: t.view(B, L, H, C // H).transpose(1, 2)  # noqa: E731
        drop = a.dropout if self.training else 0.0
        o = F.scaled_dot_product_attention(heads(q), heads(k), heads(v), dropout_p=drop)
        return decoder_ops.linear(o.transpose(1, 2).reshape(B, L, C), a.out_proj)

    def forward(self, tgt, tgt_mask: Optional[Tensor] = None, tgt_key_padding_mask: Optional[Tensor] = None,
                query_pos: Optional[Tensor] = None):
        if tgt_mask is not None or tgt_key_padding_mask is not None:
            raise NotImplementedError("the decoder never masks self-attention (reference :409-413)")
        if self.normalize_before:
            t2 = self.norm(tgt)
            q = t2 if query_pos is None else t2 + query_pos
            return tgt + self.dropout(self._attend(q, t2))
        q = tgt if query_pos is None else tgt + query_pos
        return self.norm(tgt + self.dropout(self._attend(q, tgt)))


class CrossAttentionLayer(nn.Module):
    """Masked cross-attention (reference :75-135) on the bitmask kernels; batch-first tensors."""

    def __init__(self, d_model, nhead, dropout=0.0, activation="relu", normalize_before=False):
        super().__init__()
        self.multihead_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout)
        self.norm = nn.LayerNorm(d_model)
        self.dropout = nn.Dropout(dropout)
        self.activation = _get_activation_fn(activation)
        self.normalize_before = normalize_before
        self._reset_parameters()

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def _attend(self, query, key, value, bits, lowp=None):
        a = self.multihead_attn
        if a.dropout and self.training:
            raise NotImplementedError("attention dropout > 0 is not supported by the masked-attention kernel")
        C = query.shape[-1]
        w, b = decoder_ops.lp(a.in_proj_weight), decoder_ops.lp(a.in_proj_bias)
        (w_q, w_k, w_v) = w.split(C)   # one SplitBackward (see SelfAttentionLayer)
        b_q, b_k, b_v = b.split(C) if b is not None else (None, None, None)
        q = F.linear(query, w_q, b_q)
        if lowp is not None and len(lowp) == 3:
            # (key_lp, memory_lp, sink): both projections' input gradients go to the fp32 memory (value) through the
            # level's sink (decoder_ops.GradSink); the key's pos is a constant
            k_lp, v_lp, sink = lowp
            k = decoder_ops.token_linear_sink(value, w_k, b_k, k_lp, sink)
            v = decoder_ops.token_linear_sink(value, w_v, b_v, v_lp, sink)
        else:
            k_lp, v_lp = lowp if lowp is not None else (None, None)
            k = decoder_ops.token_linear(key, w_k, b_k, x_lp=k_lp)
            v = decoder_ops.token_linear(value, w_v, b_v, x_lp=v_lp)
        o = decoder_ops.masked_attention(q, k, v, bits, a.num_heads)
        return decoder_ops.linear(o, a.out_proj)

    def forward(self, tgt, memory, memory_mask=None, memory_key_padding_mask=None, pos=None, query_pos=None,
                memory_plus_pos=None, memory_lowp=None):
        """memory_mask: bits (B, Q, words) from decoder_ops.attn_mask_bits.  memory_lowp: optional detached
        autocast-dtype copies (key, memory) made once per forward for the layers sharing a level."""
        if memory_key_padding_mask is not None:
            raise NotImplementedError("the decoder passes no key padding mask (reference :405)")
        if memory_lowp is not None and len(memory_lowp) == 3:
            key = None   # the projections read the once-cast memory + pos (decoder_ops.lowp_memory)
        else:
            key = memory_plus_pos if memory_plus_pos is not None else (memory if pos is None else memory + pos)
        if self.normalize_before:
            t2 = self.norm(tgt)
            q = t2 if query_pos is None else t2 + query_pos
            return tgt + self.dropout(self._attend(q, key, memory, memory_mask, memory_lowp))
        q = tgt if query_pos is None else tgt + query_pos
        return self.norm(tgt + self.dropout(self._attend(q, key, memory, memory_mask, memory_lowp)))


class FFNLayer(nn.Module):
    def __init__(self, d_model, dim_feedforward=2048, dropout=0.0, activation="relu", normalize_before=False):
        super().__init__()
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm = nn.LayerNorm(d_model)
        self.activation = _get_activation_fn(activation)
        self.normalize_before = normalize_before
        self._reset_parameters()

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def forward(self, tgt):
        if self.normalize_before:
            t2 = decoder_ops.linear(self.dropout(self.activation(decoder_ops.linear(self.norm(tgt), self.linear1))),
                                    self.linear2)
            return tgt + self.dropout(t2)
        t2 = decoder_ops.linear(self.dropout(self.activation(decoder_ops.linear(tgt, self.linear1))), self.linear2)
        return self.norm(tgt + self.dropout(t2))


class MLP(nn.Module):
    def __init__(self, input_dim, hidden_dim, output_dim, num_layers):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(nn.Linear(n, k) for n, k in zip([input_dim] + h, h + [output_dim]))

    def forward(self, x):
        for i, layer in enumerate(self.layers):
            x = F.relu(decoder_ops.linear(x, layer)) if i < self.num_layers - 1 else decoder_ops.linear(x, layer)
        return x


def _migrate_static_query(module, state_dict, prefix, local_metadata):
    """Old checkpoints name query_feat 'static_query' (reference :212-233)."""
    version = local_metadata.get("version", None)
    if version is None or version < 2:
        changed = False
        for k in list(state_dict.keys()):
            if k.startswith(prefix) and "static_query" in k:
                state_dict[k.replace("static_query", "query_feat")] = state_dict.pop(k)
                changed = True
        if changed:
            logging.getLogger(__name__).warning(
                f"Weight format of {module.__class__.__name__} have changed! "
                "Please upgrade your models. Applying automatic conversion now ...")


@register(transformer_decoder_registry)
class MultiScaleMaskedTransformerDecoder(nn.Module):
    _version = 2
    # under CUDA autocast: K / V memory projections on once-cast copies with one fp32 gradient sink per level
    # (decoder_ops.lowp_memory); False restores the per-level cast copies with autograd's gradient sums
    sink_memory_grads = True

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        _migrate_static_query(self, state_dict, prefix, local_metadata)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    @configurable
    def __init__(self, in_channels, mask_classification=True, *, num_classes: int, hidden_dim: int,
                 num_queries: int, nheads: int, dim_feedforward: int, dec_layers: int, pre_norm: bool,
                 mask_dim: int, enforce_input_project: bool):
        super().__init__()
        assert mask_classification, "Only support mask classification model"
        self.mask_classification = mask_classification
        self.pe_layer = PositionEmbeddingSine(hidden_dim // 2, normalize=True)
        self.num_heads = nheads
        self.num_layers = dec_layers
        self.transformer_self_attention_layers = nn.ModuleList()
        self.transformer_cross_attention_layers = nn.ModuleList()
        self.transformer_ffn_layers = nn.ModuleList()
        for _ in range(self.num_layers):
            self.transformer_self_attention_layers.append(
                SelfAttentionLayer(d_model=hidden_dim, nhead=nheads, dropout=0.0, normalize_before=pre_norm))
            self.transformer_cross_attention_layers.append(
                CrossAttentionLayer(d_model=hidden_dim, nhead=nheads, dropout=0.0, normalize_before=pre_norm))
            self.transformer_ffn_layers.append(
                FFNLayer(d_model=hidden_dim, dim_feedforward=dim_feedforward, dropout=0.0,
                         normalize_before=pre_norm))
        self.decoder_norm = nn.LayerNorm(hidden_dim)
        self.num_queries = num_queries
        self.query_feat = nn.Embedding(num_queries, hidden_dim)
        self.query_embed = nn.Embedding(num_queries, hidden_dim)
        self.num_feature_levels = 3
        self.level_embed = nn.Embedding(self.num_feature_levels, hidden_dim)
        self.input_proj = nn.ModuleList()
        for _ in range(self.num_feature_levels):
            if in_channels != hidden_dim or enforce_input_project:
                self.input_proj.append(Conv2d(in_channels, hidden_dim, kernel_size=1))
                c2_xavier_fill(self.input_proj[-1])
            else:
                self.input_proj.append(nn.Sequential())
        if self.mask_classification:
            self.class_embed = nn.Linear(hidden_dim, num_classes + 1)
        self.mask_embed = MLP(hidden_dim, hidden_dim, mask_dim, 3)

    @classmethod
    def from_config(cls, cfg, in_channels, mask_classification):
        """Same keys as the reference (:336-361); DEC_LAYERS counts the query-feature head too."""
        assert cfg.MODEL.MASK_FORMER.DEC_LAYERS >= 1
        return {
            "in_channels": in_channels,
            "mask_classification": mask_classification,
            "num_classes": cfg.MODEL.SEM_SEG_HEAD.NUM_CLASSES,
            "hidden_dim": cfg.MODEL.MASK_FORMER.HIDDEN_DIM,
            "num_queries": cfg.MODEL.MASK_FORMER.NUM_OBJECT_QUERIES,
            "nheads": cfg.MODEL.MASK_FORMER.NHEADS,
            "dim_feedforward": cfg.MODEL.MASK_FORMER.DIM_FEEDFORWARD,
            "dec_layers": cfg.MODEL.MASK_FORMER.DEC_LAYERS - 1,
            "pre_norm": cfg.MODEL.MASK_FORMER.PRE_NORM,
            "enforce_input_project": cfg.MODEL.MASK_FORMER.ENFORCE_INPUT_PROJ,
            "mask_dim": cfg.MODEL.SEM_SEG_HEAD.MASK_DIM,
        }

    # -- memory / positional inputs: (B, HW_l, C) per level, mem + pos precomputed once --------------
    def _levels(self, x, with_key=True):
        src, pos, key, size_list = [], [], [], []
        for i in range(self.num_feature_levels):
            size_list.append(tuple(x[i].shape[-2:]))
            pe = self.pe_layer(x[i], None)
            if pe.stride(0) == 0:
                # batch-shared embedding: one contiguous (1, HW, C) copy, so the adds below vectorise
                p = pe[:1].flatten(2).transpose(1, 2).contiguous().expand(pe.shape[0], -1, -1)
            else:
                p = pe.flatten(2).transpose(1, 2)
            s = decoder_ops.row_bias_add(self.input_proj[i](x[i]).flatten(2).transpose(1, 2), self.level_embed.weight[i])
            src.append(s)
            pos.append(p)
            key.append(s + p if with_key else None)
        return src, pos, key, size_list

    @staticmethod
    def _lowp_levels(src, key):
        """Per level, (key, memory) cast once to the autocast dtype for the K/V projections of the layers
        that read the level (3 each at 9 layers / 3 levels); gradients still return in fp32 per layer."""
        dev = src[0].device.type
        if dev != "cuda" or not torch.is_autocast_enabled(dev):
            return [None] * len(src)
        dt = torch.get_autocast_dtype(dev)
        if src[0].dtype == dt:
            return [None] * len(src)
        return [(k.detach().to(dt), s.detach().to(dt)) for s, k in zip(src, key)]

    @staticmethod
    def _lowp_features(mask_features):
        """The einsum operand under autocast: cast once per forward, outside the autograd graph (the
        einsum's backward returns the features' gradient in their own dtype)."""
        if torch.is_autocast_enabled(mask_features.device.type):
            dt = torch.get_autocast_dtype(mask_features.device.type)
            if dt != mask_features.dtype:
                return mask_features.detach().to(dt)
        return mask_features

    def forward(self, x, mask_features, mask=None):
        # under autocast the GEMM weights are cast once per forward in a few kernels (decoder_ops.lowp_scope)
        with decoder_ops.lowp_scope(self):
            return self._forward(x, mask_features, mask)

    def _forward(self, x, mask_features, mask=None):
        assert len(x) == self.num_feature_levels
        del mask
        lowp = None
        if self.sink_memory_grads and x[0].device.type == "cuda" and torch.is_autocast_enabled("cuda"):
            # K / V projections on once-cast memory (and memory + pos) whose fp32 gradients collect in one sink per
            # level (decoder_ops.lowp_memory): the fp32 memory + pos itself is then never formed
            src, pos, key, size_list = self._levels(x, with_key=False)
            lowp = decoder_ops.lowp_memory(src, pos)
            if any(lv is None for lv in lowp):
                key, lowp = [s + p for s, p in zip(src, pos)], None
        else:
            src, pos, key, size_list = self._levels(x)
        if lowp is None:
            lowp = self._lowp_levels(src, key)
        bs = src[0].shape[0]
        query_embed = self.query_embed.weight.unsqueeze(0).expand(bs, -1, -1)
        output = self.query_feat.weight.unsqueeze(0).repeat(bs, 1, 1)
        # every head's einsum against one fold: the features' gradient is one GEMM over all heads
        fold = decoder_ops.image_mask_fold(mask_features, self._lowp_features(mask_features))

        predictions_class, predictions_mask = [], []
        outputs_class, outputs_mask, attn_mask = self.forward_prediction_heads(
            output, mask_features, size_list[0], fold)
        predictions_class.append(outputs_class)
        predictions_mask.append(outputs_mask)

        for i in range(self.num_layers):
            level_index = i % self.num_feature_levels
            output = self.transformer_cross_attention_layers[i](
                output, src[level_index], memory_mask=attn_mask, memory_key_padding_mask=None,
                pos=pos[level_index], query_pos=query_embed, memory_plus_pos=key[level_index],
                memory_lowp=lowp[level_index])
            output = self.transformer_self_attention_layers[i](output, tgt_mask=None, tgt_key_padding_mask=None,
                                                               query_pos=query_embed)
            output = self.transformer_ffn_layers[i](output)
            last = i == self.num_layers - 1
            outputs_class, outputs_mask, attn_mask = self.forward_prediction_heads(
                output, mask_features, size_list[(i + 1) % self.num_feature_levels], fold, need_mask=not last)
            predictions_class.append(outputs_class)
            predictions_mask.append(outputs_mask)

        assert len(predictions_class) == self.num_layers + 1
        return {
            "pred_logits": predictions_class[-1],
            "pred_masks": predictions_mask[-1],
            "aux_outputs": self._set_aux_loss(predictions_class if self.mask_classification else None,
                                              predictions_mask),
        }

    def forward_prediction_heads(self, output, mask_features, attn_mask_target_size, fold=None, need_mask=True):
        """output (B, Q, C) -> class logits (B, Q, K+1), mask logits (B, Q, H, W), attention bits.
        ``fold`` is the forward's :class:`~bm2f_amd.decoder_ops.MaskFeatureFold` (one is made if absent)."""
        decoder_output = self.decoder_norm(output)
        outputs_class = decoder_ops.linear(decoder_output, self.class_embed)
        mask_embed = self.mask_embed(decoder_output)
        if fold is None:
            fold = decoder_ops.image_mask_fold(mask_features, self._lowp_features(mask_features))
        outputs_mask, attn_mask = decoder_ops.mask_heads(fold, mask_embed,
                                                         attn_mask_target_size if need_mask else None)
        return outputs_class, outputs_mask, attn_mask

    @torch.jit.unused
    def _set_aux_loss(self, outputs_class, outputs_seg_masks):
        if self.mask_classification:
            return [{"pred_logits": a, "pred_masks": b} for a, b in zip(outputs_class[:-1], outputs_seg_masks[:-1])]
        return [{"pred_masks": b} for b in outputs_seg_masks[:-1]]
