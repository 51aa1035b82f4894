"""Does a HIP graph replay re-run memset nodes? (diagnostic): torch reductions over many blocks (semaphore memset)
and the library's hipMemsetAsync (m2f_msda_fused_bwd zeroes grad_value) captured and replayed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from graph_kernel_check import check  # noqa: E402


def main():
    dev = torch.device("cuda")
    x = torch.randn(4096, 256, device=dev)
    check("sum 1M", lambda: x.sum())
    check("sum 1M dim", lambda: x.sum(0))
    check("mean 64K", lambda: x[:256].mean())
    check("norm", lambda: torch.linalg.vector_norm(x))
    from bm2f_amd.bench_model import graph_safe_sum
    xb = torch.randn(2, 200, 64, 64, device=dev).bfloat16()
    check("graph_safe_sum 1.6M bf16", lambda: graph_safe_sum(xb))
    ps = [torch.nn.Parameter(torch.randn(s_, device=dev)) for s_ in ([256, 256], [1024], [2048, 256], [96, 256]) * 80]
    for p_ in ps:
        p_.grad = torch.randn_like(p_)
    gsave = [p_.grad.clone() for p_ in ps]

    def clip():
        for p_, g_ in zip(ps, gsave):
            p_.grad.copy_(g_)
        torch.nn.utils.clip_grad_norm_(ps, 0.01, foreach=True)
        return ps[0].grad
    check("clip_grad_norm_ foreach (320 tensors)", clip)
    buf = torch.empty(1 << 20, device=dev)
    check("zero_ + add", lambda: buf.zero_().add_(1.0))
    check("memset via cudart", lambda: memset_then_add(buf))


def memset_then_add(buf):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    rc = hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, buf.numel() * 4,
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    return buf.add_(1.0)


if __name__ == "__main__":
    main()
