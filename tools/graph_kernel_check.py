"""HIP-graph replay of single library calls (diagnostic): each call captured alone, with its buffers allocated
inside the capture (as the ops do) or outside (static), replayed three times against an eager call.

    python tools/graph_kernel_check.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bm2f_amd import _native, linear_ops, norm_ops  # noqa: E402
from torch import nn  # noqa: E402


def check(name, fn, n=3):
    torch.cuda.synchronize()
    want = fn().clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    res = []
    for _ in range(n):
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        res.append((out - want).abs().max().item())
    print(f"{name}: max |replay - eager| over {n} replays: {res}", flush=True)


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(4096, 256, device=dev)
    lin = nn.Linear(256, 256).to(dev)
    check("gemm_nt alloc-in-capture", lambda: linear_ops.gemm_nt(x, lin.weight, lin.bias))
    check("gemm_nt b_kn", lambda: linear_ops.gemm_nt(x, lin.weight, b_kn=True))
    check("gemm_tn", lambda: linear_ops.gemm_tn(x, x[:, :128].contiguous(), colsum=True)[0])
    out_s = torch.empty(4096, 256, device=dev)
    check("gemm_nt static out", lambda: linear_ops.gemm_nt(x, lin.weight, lin.bias, out=out_s))
    ln = nn.LayerNorm(256).to(dev)
    check("add_layernorm", lambda: norm_ops.add_layernorm(x, x * 0.5, ln))
    # torch reference op in a graph, for the harness itself
    check("torch addmm", lambda: torch.addmm(lin.bias, x, lin.weight.t()))


if __name__ == "__main__":
    main()


def autograd_checks():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(4096, 256, device=dev, requires_grad=True)
    lin = nn.Linear(256, 256).to(dev)
    import torch.nn.functional as F

    def mk(kind):
        def fn():
            x.grad = None
            lin.weight.grad = None
            lin.bias.grad = None
            if kind == "ours-fwd":
                with torch.no_grad():
                    return linear_ops.linear(x, lin).square().mean()
            y = linear_ops.linear(x, lin) if kind.startswith("ours") else F.linear(x, lin.weight, lin.bias)
            loss = y.square().mean()
            loss.backward()
            if kind == "ours-grad":
                return lin.weight.grad
            return loss.detach()
        return fn
    for kind in ("ours-fwd", "torch", "ours", "ours-grad"):
        check("autograd " + kind, mk(kind))


if __name__ == "__main__":
    autograd_checks()
