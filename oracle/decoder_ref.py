"""TEST INFRASTRUCTURE ONLY — torch restatements of the decoder ops' reference semantics.

Used as the GPU kernels' checkers (tests/), to exercise the bm2f_amd decoder modules on CPU (patched in
place of the HIP ops), and by bench.py's cpu_baseline leg (the reference's CPU path).  Pinned by the
reference's golden decoder outputs (tests/golden/decoder.npz, video_decoder.npz: bit-exact masks).

* ref_attn_bool: F.interpolate(bilinear, align_corners=False) -> sigmoid -> < 0.5 in the logits' dtype,
  then the fully-masked-row fix (mask2former_transformer_decoder.py:446-449, :400).
* ref_masked_attention: nn.MultiheadAttention's math with a bool mask (True = blocked), per head.
"""
import contextlib
import math

import torch
import torch.nn.functional as F


def ref_attn_bool(logits, size, row_fix=True):
    """(B,Q,H,W) or (B,Q,T,H,W) -> bool (B, Q, T*h*w), True = blocked."""
    if logits.dim() == 4:
        m = F.interpolate(logits, size=size, mode="bilinear", align_corners=False)
    else:
        b, q, t = logits.shape[:3]
        m = F.interpolate(logits.flatten(0, 1), size=size, mode="bilinear", align_corners=False)
        m = m.view(b, q, t, size[0], size[1])
    m = (m.sigmoid().flatten(2) < 0.5)
    if row_fix:
        m[torch.where(m.sum(-1) == m.shape[-1])] = False
    return m


def pack_bits(mask_bool):
    B, Q, N = mask_bool.shape
    nw = (N + 31) // 32
    pad = torch.zeros((B, Q, nw * 32), dtype=torch.int64, device=mask_bool.device)
    pad[..., :N] = mask_bool.long()
    w = (pad.view(B, Q, nw, 32) << torch.arange(32, device=mask_bool.device)).sum(-1)
    w = torch.where(w >= 2 ** 31, w - 2 ** 32, w)
    return w.to(torch.int32)


def unpack_bits(bits, n):
    shifts = torch.arange(32, device=bits.device, dtype=torch.int32)
    return ((bits.unsqueeze(-1) >> shifts) & 1).bool().flatten(2)[..., :n]


def ref_masked_attention(q, k, v, blocked, num_heads, scale=None):
    """q (B,Lq,C), k/v (B,Lk,C), blocked (B,Lq,Lk) bool -> (B,Lq,C); computed in fp32 (fp64 for fp64 inputs)."""
    B, Lq, C = q.shape
    Lk = k.shape[1]
    d = C // num_heads
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    ct = torch.float64 if q.dtype == torch.float64 else torch.float32
    qh = q.to(ct).view(B, Lq, num_heads, d).transpose(1, 2)
    kh = k.to(ct).view(B, Lk, num_heads, d).transpose(1, 2)
    vh = v.to(ct).view(B, Lk, num_heads, d).transpose(1, 2)
    s = (qh * scale) @ kh.transpose(-1, -2)
    s = s.masked_fill(blocked[:, None], float("-inf"))
    p = s.softmax(-1)
    return (p @ vh).transpose(1, 2).reshape(B, Lq, C)


@contextlib.contextmanager
def torch_decoder_ops():
    """Route bm2f_amd.decoder_ops through the restatements above (CPU tests only)."""
    from bm2f_amd import decoder_ops

    saved = (decoder_ops.attn_mask_bits, decoder_ops.masked_attention)

    def bits_fn(logits, size, row_fix=True):
        return pack_bits(ref_attn_bool(logits.detach(), size, row_fix))

    def attn_fn(q, k, v, bits, num_heads, scale=None):
        return ref_masked_attention(q, k, v, unpack_bits(bits, k.shape[1]), num_heads, scale).to(q.dtype)

    decoder_ops.attn_mask_bits, decoder_ops.masked_attention = bits_fn, attn_fn
    try:
        yield
    finally:
        decoder_ops.attn_mask_bits, decoder_ops.masked_attention = saved
