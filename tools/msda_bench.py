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


HEAD_MAJOR = False


def fused_calls(value, shapes, gout, noise, M=8, P=4, seed=1):
    """Forward / backward closures of the fused-front-end kernels (m2f_msda_fused_{fwd,bwd}_f32) on the
    encoder layout: reference points at the pixel centres, offsets on the reference init rays (pixel units,
    ms_deform_attn.py:_reset_parameters) plus N(0, noise) px, random logits."""
    import ctypes
    from bm2f_amd import _native
    N, S = value.shape[:2]
    L = len(shapes)
    dev = value.device
    g = torch.Generator(device=dev).manual_seed(seed)
    refs = []
    for h, w in shapes:
        ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h, device=dev),
                                torch.linspace(0.5, w - 0.5, w, device=dev), indexing="ij")
        refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
    ref = torch.cat(refs, 0)[None, :, None, :].expand(N, S, L, 2).contiguous()
    th = torch.arange(M, device=dev) * (2 * math.pi / M)
    grid = torch.stack([th.cos(), th.sin()], -1)
    grid = grid / grid.abs().max(-1, keepdim=True)[0]
    off = (grid.view(M, 1, 1, 2) * torch.arange(1, P + 1, device=dev).view(1, 1, P, 1)).expand(M, L, P, 2)
    off = off[None, None] + noise * torch.randn(N, S, M, L, P, 2, device=dev, generator=g)
    logits = torch.randn(N, S, M * L * P, device=dev, generator=g)
    proj = torch.cat([off.reshape(N, S, -1), logits], -1).contiguous()
    if HEAD_MAJOR:  # one [offsets | logits] record per (query, head): the m2f_msda_fused_*_hm_f32 entry points
        proj = torch.cat([off.reshape(N, S, M, -1), logits.view(N, S, M, -1)], -1).reshape(N, S, -1).contiguous()
    hs = msda._host_shape_buffer(shapes)
    out = torch.empty(N, S, M * 32, device=dev)
    gv = torch.empty_like(value)
    gp = torch.empty_like(proj)
    st = msda._stream(dev)
    D = value.shape[-1]

    def fwd():
        _native.call("m2f_msda_fused_fwd_hm_f32" if HEAD_MAJOR else "m2f_msda_fused_fwd_f32", msda._ptr(value), msda._ptr(proj), proj.stride(1), msda._ptr(ref),
                     ref.stride(0), ctypes.cast(hs, ctypes.c_void_p), N, S, M, D, L, S, P, msda._ptr(out), st)

    wsb = ctypes.c_int64(0)  # deterministic mode (--opt msda_bwd_det=1) needs a workspace
    _native.call("m2f_msda_fused_bwd_workspace", ctypes.cast(hs, ctypes.c_void_p), N, S, M, D, L, P, ctypes.byref(wsb))
    ws = torch.empty(wsb.value, dtype=torch.uint8, device=dev) if wsb.value else None

    def bwd():
        _native.call("m2f_msda_fused_bwd_hm_f32" if HEAD_MAJOR else "m2f_msda_fused_bwd_f32", msda._ptr(value), msda._ptr(proj), proj.stride(1), msda._ptr(ref),
                     ref.stride(0), ctypes.cast(hs, ctypes.c_void_p), msda._ptr(gout), N, S, M, D, L, S, P,
                     msda._ptr(gv), msda._ptr(gp), None if ws is None else msda._ptr(ws), ctypes.c_int64(wsb.value), st)
    fwd.tensors = {"out": out, "grad_value": gv, "grad_proj": gp, "M": M, "LP": len(shapes) * P}
    return fwd, bwd


def digest(fwd):
    """Hashes of the fused calls' outputs, the projection gradient in the reference layout (A/B builds compare)."""
    import hashlib
    t = fwd.tensors
    gp = t["grad_proj"]
    if HEAD_MAJOR:
        M, LP = t["M"], t["LP"]
        r = gp.view(*gp.shape[:2], M, 3 * LP)
        gp = torch.cat([r[..., :2 * LP].reshape(*gp.shape[:2], -1), r[..., 2 * LP:].reshape(*gp.shape[:2], -1)], -1)
    return {k: hashlib.sha1(v.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]
            for k, v in (("out", t["out"]), ("grad_value", t["grad_value"]), ("grad_proj", gp))}


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
    ap.add_argument("--levels", type=int, default=3, choices=[3, 4],
                    help="4: add the 1/64 level (the reference module's default n_levels = 4)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stress", action="store_true")
    ap.add_argument("--no-host-shapes", action="store_true")
    ap.add_argument("--noise", type=float, default=1.0, help="px std of the offsets around the init rays")
    ap.add_argument("--bwd-only", action="store_true")
    ap.add_argument("--fwd-only", action="store_true")
    ap.add_argument("--fused", action="store_true", help="the fused front-end kernels (the path the bench step runs)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library option (m2f_set_option) for this run, repeatable; e.g. --opt msda_fwd_quad=0")
    ap.add_argument("--lib", default=None, help="another build of libbm2f.so to load (A/B against a baseline build)")
    ap.add_argument("--ab", default=None, metavar="NAME=V1,V2",
                    help="time the backward with option NAME at each value, alternating, --rounds times (one process)")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--digest", action="store_true", help="print hashes of the fused outputs after timing")
    ap.add_argument("--head-major", action="store_true",
                    help="projection rows as one [offsets | logits] record per head (the _hm_ entry points, as the "
                         "module calls them)")
    a = ap.parse_args()
    global HEAD_MAJOR
    HEAD_MAJOR = a.head_major
    from bm2f_amd import _native
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
    for kv in a.opt:
        k, v_ = kv.split("=")
        _native.set_option(k, int(v_))
    r = a.res
    shapes = [(r // s, r // s) for s in ((64, 32, 16, 8) if a.levels == 4 else (32, 16, 8))]
    v, st, lsi, loc, attn, gout = make_inputs(a.n, shapes, stress=a.stress, noise=a.noise)
    if a.no_host_shapes:
        delattr(st, "_bm2f_host_shapes")
    per_img = (r / 1024) ** 2
    fwd_bytes = 68.81e6 * per_img * a.n
    bwd_bytes = 115.60e6 * per_img * a.n
    if a.fused:
        fwd, bwd = fused_calls(v, shapes, gout, a.noise)
    else:
        fwd = lambda: msda.ms_deform_attn_forward(v, st, lsi, loc, attn, 64)  # noqa: E731
        bwd = lambda: msda.ms_deform_attn_backward(v, st, lsi, loc, attn, gout, 64)  # noqa: E731
    if a.ab:
        name, vals = a.ab.split("=")
        res = {v_: [] for v_ in vals.split(",")}
        for _ in range(a.rounds):
            for v_ in res:
                _native.set_option(name, int(v_))
                res[v_].append(timeit(bwd, a.iters))
        _native.set_option(name, -1)
        for v_, ts in res.items():
            print(f"ab {name}={v_} fused={a.fused} noise={a.noise} N={a.n}: bwd ms per round {[round(t, 4) for t in ts]} "
                  f"min {min(ts):.4f} median {sorted(ts)[len(ts) // 2]:.4f}", flush=True)
        return
    tf = 0.0 if a.bwd_only else timeit(fwd, a.iters)
    tb = float("nan") if a.fwd_only else timeit(bwd, a.iters)
    tf = tf or float("nan")
    print(f"lib={os.path.basename(a.lib) if a.lib else '-'} N={a.n} res={r} fused={a.fused} opts={','.join(a.opt) or '-'} stress={a.stress} noise={a.noise} : fwd {tf:.3f} ms ({fwd_bytes / tf / 1e6:.0f} GB/s alg), "
          f"bwd {tb:.3f} ms ({bwd_bytes / tb / 1e6:.0f} GB/s alg)")
    if a.fused and a.digest:
        fwd()
        bwd()
        torch.cuda.synchronize()
        print("digest", digest(fwd), flush=True)


if __name__ == "__main__":
    main()
