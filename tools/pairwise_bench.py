"""Ablation timing of the matcher's fused pairwise pass (csrc/weaksup.hip match_cost_kernel) at config-2
shapes: B=16 images x Q=100 masks of 256^2, G targets per image.

    python tools/pairwise_bench.py [--targets 12]

Variants: full; no targets (drops the box-weighted sums); no neighbour bits and no targets (staging +
axis maxima only); and the plain per-pixel map kernel (mode 0) for comparison.  Prints ms per launch.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bm2f_amd import weaksup  # noqa: E402


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--queries", type=int, default=100)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--targets", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, Q, H, G = a.batch, a.queries, a.hw, a.targets
    x = torch.randn(B, Q, H, H, device=dev) * 3
    sim = torch.rand(B, 8, H, H, device=dev)
    bits = weaksup.threshold_bits(sim, 0.3)
    nobits = torch.zeros_like(bits)
    # rectangular boxes up to half the image per side (box_masks are rasterised gt boxes)
    lo = torch.randint(0, H // 2, (B, G, 2), device=dev)
    hi = lo + torch.randint(4, H // 2, (B, G, 2), device=dev)
    ar = torch.arange(H, device=dev)
    iny = (ar >= lo[..., 0:1]) & (ar < hi[..., 0:1])
    inx = (ar >= lo[..., 1:2]) & (ar < hi[..., 1:2])
    box = (iny[..., :, None] & inx[..., None, :]).float().contiguous()
    gc = torch.full((B,), G, dtype=torch.int32, device=dev)
    g0 = torch.zeros_like(gc)
    rows = torch.arange(B * Q, device=dev, dtype=torch.int32) // Q
    xf = x.view(B * Q, H, H)
    res = {
        "full": timed(lambda: weaksup.match_cost(x, bits, box, gc, 2)),
        "no_targets": timed(lambda: weaksup.match_cost(x, bits, box, g0, 2)),
        "no_bits_no_targets": timed(lambda: weaksup.match_cost(x, nobits, box, g0, 2)),
        "map_mode0": timed(lambda: weaksup.pairwise_map(xf, bits, rows, 2)),
        "x_bytes_GB": x.numel() * 4 / 1e9,
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
