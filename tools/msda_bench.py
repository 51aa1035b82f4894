"""MSDA kernel microbenchmark at the config-2 layer shape (N images of a 1024^2 pyramid).

    python tools/msda_bench.py [--n 16] [--iters 20] [--stress]

Inputs follow SURVEY §8(d): sampling locations from the reference init (8 rays, 1..P px per level)
plus N(0, 1 px) noise around each query's reference point (``--stress``: loc ~ U(0,1)).
Reports ms per call and algorithmic GB/s (68.81 MB fwd / 115.60 MB bwd per 1024^2 image).
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bm2f_amd import msda  # noqa: E402


def make_inputs(N, shapes, M=8, D=32, P=4, stress=False, device="cuda", seed=0, noise=1.0):
    g = torch.Generator(device=device).manual_seed(seed)
    st = torch.tensor(shapes, dtype=torch.int64, device=device)
    msda.attach_host_shapes(st, shapes)
    lsi = torch.cat((st.new_zeros(1), st.prod(1).cumsum(0)[:-1]))
    S = int(st.prod(1).sum().item())
    L = len(shapes)
    value = torch.randn(N, S, M, D, device=device, generator=g)
    if stress:
        loc = torch.rand(N, S, M, L, P, 2, device=device, generator=g)
    else:
        refs = []
        for h, w in shapes:
            ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h, device=device),
                                    torch.linspace(0.5, w - 0.5, w, device=device), indexing="ij")
            refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
        ref = torch.cat(refs, 0)
        th = torch.arange(M, device=device) * (2 * math.pi / M)
        grid = torch.stack([th.cos(), th.sin()], -1)
        grid = grid / grid.abs().max(-1, keepdim=True)[0]
        off = grid.view(M, 1, 1, 2) * torch.arange(1, P + 1, device=device).view(1, 1, P, 1)
        off = off.expand(M, L, P, 2)
        off = off[None, None] + noise * torch.randn(N, S, M, L, P, 2, device=device, generator=g)
        norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32, device=device)
        loc = ref[None, :, None, None, None, :] + off / norm[None, None, None, :, None, :]
    attn = torch.rand(N, S, M, L, P, device=device, generator=g)
    attn = attn / attn.sum((-1, -2), keepdim=True)
    gout = torch.randn(N, S, M * D, device=device, generator=g)
    return value, st, lsi, loc.contiguous(), attn, gout


def timeit(fn, iters):
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
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stress", action="store_true")
    ap.add_argument("--no-host-shapes", action="store_true")
    ap.add_argument("--noise", type=float, default=1.0, help="px std of the offsets around the init rays")
    ap.add_argument("--bwd-only", action="store_true")
    a = ap.parse_args()
    r = a.res
    shapes = [(r // 32, r // 32), (r // 16, r // 16), (r // 8, r // 8)]
    v, st, lsi, loc, attn, gout = make_inputs(a.n, shapes, stress=a.stress, noise=a.noise)
    if a.no_host_shapes:
        delattr(st, "_bm2f_host_shapes")
    per_img = (r / 1024) ** 2
    fwd_bytes = 68.81e6 * per_img * a.n
    bwd_bytes = 115.60e6 * per_img * a.n
    tf = 0.0 if a.bwd_only else timeit(lambda: msda.ms_deform_attn_forward(v, st, lsi, loc, attn, 64), a.iters)
    tb = timeit(lambda: msda.ms_deform_attn_backward(v, st, lsi, loc, attn, gout, 64), a.iters)
    tf = tf or float("nan")
    print(f"N={a.n} res={r} stress={a.stress} noise={a.noise} env={ {k: v for k, v in os.environ.items() if k.startswith('M2F_')} }: fwd {tf:.3f} ms ({fwd_bytes / tf / 1e6:.0f} GB/s alg), "
          f"bwd {tb:.3f} ms ({bwd_bytes / tb / 1e6:.0f} GB/s alg)")


if __name__ == "__main__":
    main()
