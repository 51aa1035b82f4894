"""Deterministic per-parameter-name weight filler shared by the golden generator and the tests.

Fixtures store only inputs and outputs; the weights of any module are re-created from the state-dict
key names, so the reference modules (in this container, via gen_golden.py) and the bm2f_amd modules
(anywhere) see bit-identical parameters.

Rule for a tensor named ``key`` with shape ``shape``: u ~ U[-1, 1) from a CPU generator seeded with
crc32(key), then
  * ``*.sampling_offsets.bias``  -> the reference init grid (ms_deform_attn.py:66-75) + 0.25*u
  * ``*.sampling_offsets.weight``-> 0.02*u
  * 1-D ``*.weight`` (LayerNorm / GroupNorm affine scales)  -> 1 + 0.1*u
  * other 1-D tensors (biases, level embeddings as 1-D)  -> 0.05*u
  * tensors with dim >= 2        -> u * sqrt(3 / fan_in), fan_in = prod(shape[1:])
"""
from __future__ import annotations

import math
import zlib

import torch


def _u(key: str, shape) -> torch.Tensor:
    g = torch.Generator().manual_seed(zlib.crc32(key.encode("utf-8")) & 0x7FFFFFFF)
    return torch.rand(tuple(shape), generator=g, dtype=torch.float64) * 2.0 - 1.0


def _offset_grid(numel: int, n_heads: int = 8, n_points: int = 4) -> torch.Tensor:
    n_levels = numel // (n_heads * n_points * 2)
    thetas = torch.arange(n_heads, dtype=torch.float64) * (2.0 * math.pi / n_heads)
    grid = torch.stack([thetas.cos(), thetas.sin()], -1)
    grid = grid / grid.abs().max(-1, keepdim=True)[0]
    grid = grid.view(n_heads, 1, 1, 2).repeat(1, n_levels, n_points, 1)
    grid = grid * torch.arange(1, n_points + 1, dtype=torch.float64).view(1, 1, -1, 1)
    return grid.reshape(-1)


def fill_value(key: str, shape) -> torch.Tensor:
    u = _u(key, shape)
    if key.endswith("sampling_offsets.bias"):
        return _offset_grid(u.numel()) + 0.25 * u
    if key.endswith("sampling_offsets.weight"):
        return 0.02 * u
    if len(shape) == 1:
        if key.endswith(".weight"):
            return 1.0 + 0.1 * u
        return 0.05 * u
    fan_in = 1
    for s in shape[1:]:
        fan_in *= int(s)
    return u * math.sqrt(3.0 / max(fan_in, 1))


@torch.no_grad()
def fill_module(module: torch.nn.Module) -> torch.nn.Module:
    """Overwrite every parameter (not buffers) of ``module`` in place."""
    for key, p in module.named_parameters():
        p.copy_(fill_value(key, p.shape).to(p.dtype))
    return module


def state_dict_for(module: torch.nn.Module) -> dict:
    return {k: fill_value(k, p.shape).to(torch.float32) for k, p in module.named_parameters()}
