"""FPN merge of the pixel decoder (msdeformattn.py:343-349): lateral + bilinear 2x upsample of the encoder's
finest map, which arrives as a transposed (N, HW, C) view.  Times the layout variants, fwd + bwd.
python tools/fpn_bench.py"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bm2f_amd import conv_ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    N, C, h, w = 16, 256, 128, 128
    z = torch.randn(N, h * w, C, device=dev, requires_grad=True)
    lat = torch.randn(N, C, 2 * h, 2 * w, device=dev, requires_grad=True)
    g = torch.randn(N, C, 2 * h, 2 * w, device=dev)
    variants = {
        "view (current)": lambda src: F.interpolate(src, size=(2 * h, 2 * w), mode="bilinear", align_corners=False),
        "contiguous in": lambda src: F.interpolate(src.contiguous(), size=(2 * h, 2 * w), mode="bilinear",
                                                   align_corners=False),
        "contiguous out": lambda src: F.interpolate(src, size=(2 * h, 2 * w), mode="bilinear",
                                                    align_corners=False).contiguous(),
    }
    variants["fused (upsample.hip)"] = None
    variants["fused, contiguous in"] = "c"
    ref = None
    for name, up in variants.items():
        def fwd():
            if up is None:
                return conv_ops.upsample_add(z.transpose(1, 2).view(N, C, h, w), lat)
            if up == "c":
                return conv_ops.upsample_add(z.transpose(1, 2).contiguous().view(N, C, h, w), lat)
            return lat + up(z.transpose(1, 2).view(N, C, h, w))
        y = fwd()
        if ref is None:
            ref = y.detach()
        torch.testing.assert_close(y.detach(), ref, rtol=1e-5, atol=1e-5)
        tf = timeit(fwd)
        tb = timeit(lambda: torch.autograd.grad(fwd(), (z, lat), g))
        print(f"{name:16s} fwd {tf:.3f} ms  fwd+bwd {tb:.3f} ms  out contiguous={y.is_contiguous()}", flush=True)


if __name__ == "__main__":
    main()
