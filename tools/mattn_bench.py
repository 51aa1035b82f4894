"""Masked cross-attention fwd / bwd at the decoder shapes (B=16 Q=100 and config 4's B=2 Q=200, the three
pyramid levels of 1024^2), fp16, ~60 % of the keys blocked; per-call ms and algorithmic GB/s.

    python tools/mattn_bench.py [--dq-atomic]      (--dq-atomic: option mattn_dq_atomic = 1, the LDS-atomic dQ)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bm2f_amd import _native, decoder_ops  # noqa: E402


def bits_for(B, Q, Lk, device, p=0.6):
    g = torch.Generator(device=device).manual_seed(Q + Lk)
    blocked = torch.rand(B, Q, Lk, device=device, generator=g) < p
    blocked[:, :, 0] = False
    nw = (Lk + 31) // 32
    pad = torch.zeros(B, Q, nw * 32, dtype=torch.int64, device=device)
    pad[..., :Lk] = blocked.long()
    w = (pad.view(B, Q, nw, 32) << torch.arange(32, device=device)).sum(-1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--dq-atomic", action="store_true")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library option (m2f_set_option) for this run, repeatable; e.g. --opt mattn_bwd_minblk=4")
    ap.add_argument("--lib", default=None, help="another build of libbm2f.so to load (A/B against a baseline build)")
    a = ap.parse_args()
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
        print("lib:", os.path.basename(a.lib))
    if a.dq_atomic:
        _native.set_option("mattn_dq_atomic", 1)
    for kv in a.opt:
        k_, v_ = kv.split("=")
        _native.set_option(k_, int(v_))
    print(f"opts: {','.join(a.opt) or '-'}", flush=True)
    dev = torch.device("cuda")
    dt = torch.float16
    for B, Q in ((16, 100), (2, 200)):
        for Lk in (1024, 4096, 16384):
            g = torch.Generator(device=dev).manual_seed(Lk)
            q = torch.randn(B, Q, 256, device=dev, generator=g).to(dt).requires_grad_()
            k = torch.randn(B, Lk, 256, device=dev, generator=g).to(dt).requires_grad_()
            v = torch.randn(B, Lk, 256, device=dev, generator=g).to(dt).requires_grad_()
            bits = bits_for(B, Q, Lk, dev)
            go = torch.randn(B, Q, 256, device=dev, generator=g).to(dt)
            tf = timeit(lambda: decoder_ops.masked_attention(q, k, v, bits, 8))
            tfb = timeit(lambda: decoder_ops.masked_attention(q, k, v, bits, 8).backward(go))
            kv = 2 * B * Lk * 256 * 2
            print(f"B={B} Q={Q} Lk={Lk}: fwd {tf:.4f} ms ({(kv + 2 * B * Q * 512) / tf / 1e6:.0f} GB/s alg), "
                  f"bwd {tfb - tf:.4f} ms ({(2 * kv + 4 * B * Q * 512) / (tfb - tf) / 1e6:.0f} GB/s alg)", flush=True)


if __name__ == "__main__":
    main()
