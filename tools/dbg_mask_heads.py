"""Where do the mask-heads logits and torch's fp32 bmm differ? Compares both with an fp64 product of the same
low-precision operands, per dtype, for the Q=200 64x96 case."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")]
import torch

from test_mask_heads_gpu import _case, _fold
from bm2f_amd import decoder_ops

dev = torch.device("cuda")
for dt, T in [("f16", torch.float16), ("bf16", torch.bfloat16)]:
    for case in [(1, 200, 256, 1, 64, 96), (2, 100, 256, 1, 64, 64)]:
        B, Q, C, Tf, H, W = case
        e, f = _case(dev, B, Q, C, Tf, H, W, dt)
        out, _ = decoder_ops.mask_heads(_fold(f, 1), e, None)
        exact = torch.bmm(e.double(), f.double().reshape(B, C, -1)).view(out.shape)
        bmm32 = torch.bmm(e.float(), f.float().reshape(B, C, -1)).view(out.shape)
        r_ex = exact.to(T)
        print(dt, case, "subnormal f:", (f.float().abs() < 6.1e-5).float().mean().item() if dt == "f16" else 0)
        for name, v in [("kernel", out), ("bmm32->dt", bmm32.to(T)), ("bmm32 raw", bmm32)]:
            d = (v.double() - r_ex.double()).abs()
            bad = d > r_ex.double().abs() * (2 ** -10 if dt == "f16" else 2 ** -7) + 1e-6
            print(f"  {name:10s} max|d| {d.max().item():.3g}  n>1ulp {int(bad.sum())}  "
                  f"max|v-exact| {(v.double() - exact).abs().max().item():.3g}")
            if bad.any() and name == "kernel":
                idx = bad.nonzero()[:5].tolist()
                for i in idx:
                    print("    at", i, "kernel", v[tuple(i)].item(), "exact", exact[tuple(i)].item(),
                          "bmm32", bmm32[tuple(i)].item())
