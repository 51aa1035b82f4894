"""Mask-einsum feature gradient (m2f_mask_heads_bwd_feats) at config 2: 10 heads, B=16, Q=100, 256^2, fp16 G,
fp32 output; per-call ms, algorithmic GB/s and TFLOP/s, for each k-steps-per-stage option.

    python tools/mask_df_bench.py [--b 16] [--q 100] [--n 65536] [--stages 4,1] [--lib tools/lib/libbm2f_X.so]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bm2f_amd import _native, decoder_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--q", type=int, default=100)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--heads", type=int, default=10)
    ap.add_argument("--stages", default="4,1", help="k-steps-per-stage options to time, comma separated")
    ap.add_argument("--lib", default=None, help="another build of libbm2f.so to load (A/B against a baseline build)")
    a = ap.parse_args()
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device("cuda")
    dt = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    es = [torch.randn(a.b, a.q, 256, device=dev, generator=g).to(dt) for _ in range(a.heads)]
    gs = [torch.randn(a.b, a.q, a.n, device=dev, generator=g).to(dt) for _ in range(a.heads)]
    nbytes = a.heads * a.b * a.q * a.n * 2 + a.b * 256 * a.n * 4
    flops = 2 * a.b * 256 * a.n * a.heads * a.q
    lib = os.path.basename(a.lib) if a.lib else "-"
    for stage in [int(x) for x in a.stages.split(",")] * 2:
        with _native.options(mask_df_stage=stage):
            for _ in range(3):
                decoder_ops.mask_heads_bwd_feats(es, gs, torch.float32)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                decoder_ops.mask_heads_bwd_feats(es, gs, torch.float32)
            e.record()
            torch.cuda.synchronize()
            t = s.elapsed_time(e) / 10
        print(f"lib={lib} stage {stage}: {t:.3f} ms  {nbytes / t / 1e6:.0f} GB/s alg  {flops / t / 1e9:.0f} TF", flush=True)


if __name__ == "__main__":
    main()
