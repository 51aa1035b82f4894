"""bf16 weight-gradient GEMM dW = G^T X over a long reduction (the decoder's cross-attention K/V
projections: rows = B*HW_l up to 262144), hipBLASLt formulations.  python tools/wgrad_bf16_bench.py"""
import torch


def timeit(fn, iters=20):
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
    for rows in (262144, 65536, 16384):
        g = torch.randn(rows, 256, device=dev, dtype=torch.bfloat16)
        x = torch.randn(rows, 256, device=dev, dtype=torch.bfloat16)
        fl = 2 * rows * 256 * 256
        res = {"gT@x": timeit(lambda: g.t() @ x), "(xT@g)T": timeit(lambda: (x.t() @ g).t())}
        for ch in (2048, 4096, 8192):
            if rows % ch == 0 and rows // ch >= 2:
                res[f"bmm{ch}"] = timeit(lambda: torch.bmm(g.view(-1, ch, 256).transpose(1, 2),
                                                            x.view(-1, ch, 256)).sum(0, dtype=torch.float32))

        print(f"rows={rows}: " + "  ".join(f"{k} {t * 1e3:.1f}us ({fl / t / 1e9:.0f} TF)" for k, t in res.items()), flush=True)


if __name__ == "__main__":
    main()
