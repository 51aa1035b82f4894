"""Worst elements of the mask-head embed gradient (G F^T) against fp64, for the failing test shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bm2f_amd import decoder_ops

dev = torch.device("cuda")
for (B, Q, N) in [(2, 37, 65536), (2, 100, 65536), (2, 100, 4096)]:
    gen = torch.Generator(device=dev).manual_seed(Q + N)
    g = torch.randn(B, Q, N, device=dev, generator=gen).to(torch.bfloat16)
    f = (torch.randn(B, 256, N, device=dev, generator=gen) / 16).to(torch.bfloat16)
    de = decoder_ops.mask_heads_bwd_embed(g, f)
    exact = torch.bmm(g.double(), f.double().transpose(1, 2))
    f32 = torch.bmm(g.float(), f.float().transpose(1, 2))
    ref = exact.to(torch.bfloat16)
    d = (de.double() - exact).abs()
    rel = d / exact.abs().clamp_min(1e-30)
    i = torch.argmax(d - exact.abs() * 2 ** -8)
    idx = torch.unravel_index(i, d.shape)
    print((B, Q, N), "max|de-exact|", d.max().item(), "at", [int(x) for x in idx], "exact", exact[idx].item(),
          "kernel", de[idx].item(), "ref", ref[idx].item(), "f32 bmm", f32[idx].item())
    print("   n(>1 ulp of ref)", int(((de.float() - ref.float()).abs() > ref.float().abs() * 2 ** -7 + 1e-6).sum()),
          " max |f32 bmm - exact|", (f32.double() - exact).abs().max().item())
