"""Time the mask-heads kernel against torch.bmm + m2f_attn_mask_bits at the bench's decoder shapes
(bs16, Q=100, 256 channels, 256^2 mask features, the three pyramid targets), bf16.

    python tools/mask_heads_bench.py [--batch 16] [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--queries", type=int, default=100)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None, help="another build of libbm2f.so to load (A/B against a baseline build)")
    a = ap.parse_args()
    import torch
    from bm2f_amd import _native, decoder_ops
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
        print("lib:", os.path.basename(a.lib))
    dev = torch.device("cuda")
    B, Q, C, H = a.batch, a.queries, 256, a.res
    g = torch.Generator(device=dev).manual_seed(0)
    e = torch.randn(B, Q, C, device=dev, generator=g).bfloat16()
    f = (torch.randn(B, C, H, H, device=dev, generator=g) / 16).bfloat16()
    fold = decoder_ops.MaskFeatureFold(f, f.reshape(B, C, -1), (H, H), lambda df, s: df.view(s))

    def timeit(fn):
        for _ in range(3):
            fn()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.iters):
            fn()
        t.record()
        torch.cuda.synchronize()
        return s.elapsed_time(t) / a.iters

    res = {}
    nbytes = 2 * B * H * H * (C + Q) + 2 * B * Q * C
    for size in [None, (H // 8, H // 8), (H // 4, H // 4), (H // 2, H // 2)]:
        fused = timeit(lambda: decoder_ops.mask_heads(fold, e, size))
        if size is None:
            base = timeit(lambda: fold(e))
        else:
            base = timeit(lambda: decoder_ops.attn_mask_bits(fold(e), size))
        key = "einsum" if size is None else f"target{size[0]}"
        res[key] = {"fused_ms": round(fused, 4), "bmm_plus_bits_ms": round(base, 4),
                    "fused_GBps": round(nbytes / fused / 1e6, 1), "fused_frac_hbm": round(nbytes / fused / 1e6 / 8000, 3),
                    "fused_mfma_tflops": round(2 * B * Q * C * H * H / fused / 1e9, 1)}
        print(key, res[key], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
