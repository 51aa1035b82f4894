"""Sine position embeddings (reference transformer_decoder/position_encoding.py:12-52 and
mask2former_video/modeling/transformer_decoder/position_encoding.py:12-57).

The hot path only ever calls them with ``mask=None`` (msdeformattn.py:322, decoder :375), so the
embedding depends on the feature map's spatial size alone.  It is computed with the reference's exact
fp32 op sequence once per (shape, device) and cached; the cached tensor is returned expanded over the
batch (no per-step recomputation, no grad).
"""
from __future__ import annotations

import math

import torch
from torch import nn


def _embed(not_mask: torch.Tensor, num_pos_feats, temperature, normalize, scale):
    y_embed = not_mask.cumsum(1, dtype=torch.float32)
    x_embed = not_mask.cumsum(2, dtype=torch.float32)
    if normalize:
        eps = 1e-6
        y_embed = y_embed / (y_embed[:, -1:, :] + eps) * scale
        x_embed = x_embed / (x_embed[:, :, -1:] + eps) * scale
    dim_t = torch.arange(num_pos_feats, dtype=torch.float32, device=not_mask.device)
    dim_t = temperature ** (2 * (dim_t // 2) / num_pos_feats)
    pos_x = x_embed[:, :, :, None] / dim_t
    pos_y = y_embed[:, :, :, None] / dim_t
    pos_x = torch.stack((pos_x[:, :, :, 0::2].sin(), pos_x[:, :, :, 1::2].cos()), dim=4).flatten(3)
    pos_y = torch.stack((pos_y[:, :, :, 0::2].sin(), pos_y[:, :, :, 1::2].cos()), dim=4).flatten(3)
    return torch.cat((pos_y, pos_x), dim=3).permute(0, 3, 1, 2)


class PositionEmbeddingSine(nn.Module):
    def __init__(self, num_pos_feats=64, temperature=10000, normalize=False, scale=None):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        if scale is not None and normalize is False:
            raise ValueError("normalize should be True if scale is passed")
        self.scale = 2 * math.pi if scale is None else scale
        self._cache = {}

    def forward(self, x, mask=None):
        if mask is not None:
            return _embed(~mask, self.num_pos_feats, self.temperature, self.normalize, self.scale)
        key = (x.shape[-2], x.shape[-1], x.device)
        pe = self._cache.get(key)
        if pe is None:
            ones = torch.ones((1, x.shape[-2], x.shape[-1]), device=x.device, dtype=torch.bool)
            with torch.no_grad():
                pe = _embed(ones, self.num_pos_feats, self.temperature, self.normalize, self.scale).contiguous()
            self._cache[key] = pe
        return pe.expand(x.shape[0], -1, -1, -1)


class PositionEmbeddingSine3D(nn.Module):
    """(B, T, C, H, W) -> (B, T, 2*num_pos_feats, H, W); z (time) term added to the cat(y, x) term."""

    def __init__(self, num_pos_feats=64, temperature=10000, normalize=False, scale=None):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        if scale is not None and normalize is False:
            raise ValueError("normalize should be True if scale is passed")
        self.scale = 2 * math.pi if scale is None else scale
        self._cache = {}

    def _compute(self, not_mask):
        z_embed = not_mask.cumsum(1, dtype=torch.float32)
        y_embed = not_mask.cumsum(2, dtype=torch.float32)
        x_embed = not_mask.cumsum(3, dtype=torch.float32)
        if self.normalize:
            eps = 1e-6
            z_embed = z_embed / (z_embed[:, -1:, :, :] + eps) * self.scale
            y_embed = y_embed / (y_embed[:, :, -1:, :] + eps) * self.scale
            x_embed = x_embed / (x_embed[:, :, :, -1:] + eps) * self.scale
        npf = self.num_pos_feats
        dev = not_mask.device
        dim_t = torch.arange(npf, dtype=torch.float32, device=dev)
        dim_t = self.temperature ** (2 * (dim_t // 2) / npf)
        dim_t_z = torch.arange(npf * 2, dtype=torch.float32, device=dev)
        dim_t_z = self.temperature ** (2 * (dim_t_z // 2) / (npf * 2))
        pos_x = x_embed[:, :, :, :, None] / dim_t
        pos_y = y_embed[:, :, :, :, None] / dim_t
        pos_z = z_embed[:, :, :, :, None] / dim_t_z
        pos_x = torch.stack((pos_x[..., 0::2].sin(), pos_x[..., 1::2].cos()), dim=5).flatten(4)
        pos_y = torch.stack((pos_y[..., 0::2].sin(), pos_y[..., 1::2].cos()), dim=5).flatten(4)
        pos_z = torch.stack((pos_z[..., 0::2].sin(), pos_z[..., 1::2].cos()), dim=5).flatten(4)
        return (torch.cat((pos_y, pos_x), dim=4) + pos_z).permute(0, 1, 4, 2, 3)

    def forward(self, x, mask=None):
        if x.dim() != 5:
            raise AssertionError(f"{x.shape} should be a 5-dimensional Tensor, got {x.dim()}-dimensional Tensor instead")
        if mask is not None:
            return self._compute(~mask)
        key = (x.shape[1], x.shape[3], x.shape[4], x.device)
        pe = self._cache.get(key)
        if pe is None:
            ones = torch.ones((1, x.shape[1], x.shape[3], x.shape[4]), device=x.device, dtype=torch.bool)
            with torch.no_grad():
                pe = self._compute(ones).contiguous()
            self._cache[key] = pe
        return pe.expand(x.shape[0], -1, -1, -1, -1)
