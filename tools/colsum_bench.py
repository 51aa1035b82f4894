"""m2f_colsum (decoder_ops.colsum_f32) against torch's column sum at the config-2 step's shapes: per-call ms.

    python tools/colsum_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bm2f_amd.decoder_ops import colsum_f32  # noqa: E402


def t(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    dev = torch.device("cuda")
    for rows, dt in ((262144, torch.float16), (65536, torch.float16), (16384, torch.float16), (262144, torch.float32),
                     (21504, torch.float32)):
        x = torch.randn(rows, 256, device=dev).to(dt)
        a = t(lambda: colsum_f32(x))
        b = t(lambda: x.sum(0, dtype=torch.float32))
        gb = rows * 256 * x.element_size() / 1e9
        print(f"rows {rows:7d} {str(dt):14s} m2f_colsum {a * 1e3:7.1f} us ({gb / a * 1e3:6.0f} GB/s)   torch {b * 1e3:7.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
