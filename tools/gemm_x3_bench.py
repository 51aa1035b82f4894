"""x3 (split-bf16) vs exact-f32 MFMA vs hipBLASLt fp32 GEMMs on the encoder-layer shapes: time + error vs fp64.
python tools/gemm_x3_bench.py [--rows 344064]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bm2f_amd import _native, linear_ops  # noqa: E402


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


def rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16 * 21504)
    ap.add_argument("--cfgs", default="0,2,3", help="x3_nt_cfg option values to time")
    ap.add_argument("--lib", default=None, help="another build of libbm2f.so (A/B)")
    ap.add_argument("--x3-only", action="store_true", help="time only the x3 engine (A/B runs)")
    ap.add_argument("--tn-nw", default="", help="x3_tn_nw option values to time the wgrad with, e.g. 4,41")
    ap.add_argument("--shapes", default="256x256,256x288,256x1024,1024x256", help="KxN forward shapes")
    a = ap.parse_args()
    if a.lib:
        from bm2f_amd import _native as _nat
        _nat._LIB_PATH = os.path.abspath(a.lib)
    M = a.rows
    dev = torch.device("cuda")
    torch.manual_seed(0)
    sub = slice(0, 4096)
    for (K, N) in [tuple(int(v) for v in sh.split("x")) for sh in a.shapes.split(",")]:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        g = torch.randn(M, N, device=dev)
        fl = 2.0 * M * N * K
        ref = x[sub].double() @ w.double().t() + b.double()
        res = {}
        if not a.x3_only:
            res["blas"] = (timeit(lambda: torch.nn.functional.linear(x, w, b)),
                           rel(torch.nn.functional.linear(x, w, b)[sub], ref))
            res["exact"] = (timeit(lambda: linear_ops.gemm_nt(x, w, b, engine="exact")),
                            rel(linear_ops.gemm_nt(x, w, b, engine="exact")[sub], ref))
        res["x3"] = (timeit(lambda: linear_ops.gemm_nt(x, w, b, engine="x3")),
                     rel(linear_ops.gemm_nt(x, w, b, engine="x3")[sub], ref))
        for c in [c for c in a.cfgs.split(",") if c]:
            _native.set_option("x3_nt_cfg", int(c))
            try:
                res[f"x3c{c}"] = (timeit(lambda: linear_ops.gemm_nt(x, w, b, engine="x3")),
                                  rel(linear_ops.gemm_nt(x, w, b, engine="x3")[sub], ref))
            finally:
                _native.set_option("x3_nt_cfg", -1)
        print(f"fwd   M={M} K={K} N={N}: " + "  ".join(f"{k} {t:.3f}ms {fl / t / 1e9:.0f}TF err {e:.1e}" for k, (t, e) in res.items()), flush=True)
        wt = w.t().contiguous()
        ref = g[sub].double() @ w.double()
        mk = torch.randn(M, K, device=dev)
        res = {"x3": (timeit(lambda: linear_ops.gemm_nt(g, w, engine="x3", b_kn=True)),
                      rel(linear_ops.gemm_nt(g, w, engine="x3", b_kn=True)[sub], ref)),
               "x3mask": (timeit(lambda: linear_ops.gemm_nt(g, w, mask=mk, engine="x3", b_kn=True)), 0.0)}
        if not a.x3_only:
            res["blas"] = (timeit(lambda: g @ w), rel((g @ w)[sub], ref))
            res["exact"] = (timeit(lambda: linear_ops.gemm_nt(g, wt, engine="exact")),
                            rel(linear_ops.gemm_nt(g, wt, engine="exact")[sub], ref))
            res["exactmask"] = (timeit(lambda: linear_ops.gemm_nt(g, wt, mask=mk, engine="exact")), 0.0)
        print(f"dgrad M={M} K={N} N={K}: " + "  ".join(f"{k} {t:.3f}ms {fl / t / 1e9:.0f}TF err {e:.1e}" for k, (t, e) in res.items()), flush=True)
        del mk
        ref = g.double().t() @ x.double()
        refb = g.double().sum(0)
        res = {} if a.x3_only else {"blas": (timeit(lambda: (g.t() @ x, g.sum(0))), rel(g.t() @ x, ref))}
        for eng in (("x3",) if a.x3_only else ("exact", "x3")):
            dw, db = linear_ops.gemm_tn(g, x, colsum=True, engine=eng)
            res[eng] = (timeit(lambda: linear_ops.gemm_tn(g, x, colsum=True, engine=eng)), rel(dw, ref))
            res[eng + "_bias"] = (0.0, rel(db, refb))
        for rnd, nw in enumerate([v for v in a.tn_nw.split(",") if v]):
            _native.set_option("x3_tn_nw", int(nw))
            try:
                dw, db = linear_ops.gemm_tn(g, x, colsum=True, engine="x3")
                res[f"nw{nw}.{rnd}"] = (timeit(lambda: linear_ops.gemm_tn(g, x, colsum=True, engine="x3")), rel(dw, ref))
                res[f"nw{nw}_bias.{rnd}"] = (0.0, rel(db, refb))
            finally:
                _native.set_option("x3_tn_nw", -1)
        print(f"wgrad M={M} N1={N} N2={K}: " + "  ".join(f"{k} {t:.3f}ms {fl / max(t, 1e-9) / 1e9:.0f}TF err {e:.1e}" for k, (t, e) in res.items()), flush=True)
        del x, w, g


if __name__ == "__main__":
    main()
