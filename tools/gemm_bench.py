"""fp32 GEMM kernels (csrc/gemm.hip) vs torch (hipBLASLt) on the encoder-layer shapes: time + error vs fp64.
python tools/gemm_bench.py [--rows 344064]"""
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
    ap.add_argument("--sweep", default="", help="comma list of gemm_nt_cfg option values to time for fwd/dgrad")
    a = ap.parse_args()
    M = a.rows
    dev = torch.device("cuda")
    torch.manual_seed(0)
    print(f"{'shape':28s} {'op':6s} {'torch ms':>9s} {'TF':>6s} {'ours ms':>9s} {'TF':>6s} {'err torch':>10s} {'err ours':>10s}")
    for (K, N) in [(256, 256), (256, 288), (256, 1024), (1024, 256)]:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        g = torch.randn(M, N, device=dev)
        flops = 2.0 * M * N * K
        # forward
        t0 = timeit(lambda: torch.nn.functional.linear(x, w, b))
        t1 = timeit(lambda: linear_ops.gemm_nt(x, w, b))
        sub = slice(0, 4096)
        ref = x[sub].double() @ w.double().t() + b.double()
        e0 = rel(torch.nn.functional.linear(x, w, b)[sub], ref)
        e1 = rel(linear_ops.gemm_nt(x, w, b)[sub], ref)
        print(f"M={M} K={K} N={N}".ljust(28), "fwd".ljust(6), f"{t0:9.3f} {flops / t0 / 1e9:6.1f} {t1:9.3f} {flops / t1 / 1e9:6.1f} {e0:10.2e} {e1:10.2e}")
        # dgrad: g (M,N) @ w (N,K)
        wt = w.t().contiguous()
        t0 = timeit(lambda: g @ w)
        t1 = timeit(lambda: linear_ops.gemm_nt(g, wt))
        ref = g[sub].double() @ w.double()
        e0 = rel((g @ w)[sub], ref)
        e1 = rel(linear_ops.gemm_nt(g, wt)[sub], ref)
        print(" " * 28, "dgrad".ljust(6), f"{t0:9.3f} {flops / t0 / 1e9:6.1f} {t1:9.3f} {flops / t1 / 1e9:6.1f} {e0:10.2e} {e1:10.2e}")
        mk = torch.randn(M, K, device=dev)
        tm = timeit(lambda: linear_ops.gemm_nt(g, wt, mask=mk))
        tw = timeit(lambda: torch.where(mk > 0, g @ w, 0.0))
        print(" " * 28, "dg+msk".ljust(6), f"{tw:9.3f} {flops / tw / 1e9:6.1f} {tm:9.3f} {flops / tm / 1e9:6.1f}")
        del mk
        # wgrad: g^T (N,M) @ x (M,K) + colsum
        t0 = timeit(lambda: (g.t() @ x, g.sum(0)))
        t1 = timeit(lambda: linear_ops.gemm_tn(g, x, colsum=True))
        ref = g.double().t() @ x.double()
        e0 = rel(g.t() @ x, ref)
        dw, db = linear_ops.gemm_tn(g, x, colsum=True)
        e1 = rel(dw, ref)
        eb = rel(db, g.double().sum(0))
        print(" " * 28, "wgrad".ljust(6), f"{t0:9.3f} {flops / t0 / 1e9:6.1f} {t1:9.3f} {flops / t1 / 1e9:6.1f} {e0:10.2e} {e1:10.2e} bias {eb:.1e}")
        for cfg in [c for c in a.sweep.split(",") if c]:
            _native.set_option("gemm_nt_cfg", int(cfg))
            tf = timeit(lambda: linear_ops.gemm_nt(x, w, b))
            td = timeit(lambda: linear_ops.gemm_nt(g, wt))
            ef = rel(linear_ops.gemm_nt(x, w, b)[sub], x[sub].double() @ w.double().t() + b.double())
            print(" " * 28, f"cfg{cfg}".ljust(6), f"fwd {tf:7.3f} ms {flops / tf / 1e9:6.1f} TF  dgrad {td:7.3f} ms "
                  f"{flops / td / 1e9:6.1f} TF  err {ef:.1e}")
            _native.set_option("gemm_nt_cfg", -1)
        del x, w, g


if __name__ == "__main__":
    main()
