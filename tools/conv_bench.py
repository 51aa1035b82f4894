"""x3 fp32 convs (conv_ops) vs MIOpen F.conv2d on the pixel decoder's conv shapes at bs16, 1024^2 input.
python tools/conv_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bm2f_amd.miopen_tuning import use_shipped_find_db  # noqa: E402

use_shipped_find_db()
import torch  # noqa: E402
from torch import nn  # noqa: E402

from bm2f_amd import conv_ops  # noqa: E402


def timeit(fn, iters=5):
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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="shapes whose name contains this")
    ap.add_argument("--lib", default=None, help="another build of libbm2f.so (A/B)")
    ap.add_argument("--x3-only", action="store_true", help="skip the MIOpen timings (A/B runs)")
    a = ap.parse_args()
    if a.lib:
        from bm2f_amd import _native as _nat
        _nat._LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device("cuda")
    shapes = [("layer_1 3x3", 16, 256, 256, 256, 256, 3, False), ("adapter_1 1x1", 16, 256, 256, 256, 256, 1, False),
              ("mask_features 1x1", 16, 256, 256, 256, 256, 1, True), ("input_proj res3", 16, 512, 256, 128, 128, 1, True),
              ("input_proj res4", 16, 1024, 256, 64, 64, 1, True), ("input_proj res5", 16, 2048, 256, 32, 32, 1, True)]
    for name, N, Ci, Co, H, W, k, b in shapes:
        if a.only not in name:
            continue
        conv = nn.Conv2d(Ci, Co, k, padding=k // 2, bias=b).to(dev)
        x = torch.randn(N, Ci, H, W, device=dev, requires_grad=True)
        g = torch.randn(N, Co, H, W, device=dev)
        fl = 2.0 * N * H * W * Ci * Co * k * k
        res = {}
        engines = (("miopen", lambda: conv(x)), ("x3", lambda: conv_ops.conv2d(x, conv)),
                   ("x3+tn", lambda: conv_ops.conv2d(x, conv)))
        for eng, fn in engines[2:] if a.x3_only else engines:
            conv_ops.WGRAD3 = "tn" if eng == "x3+tn" else "miopen"
            tf = timeit(fn)
            y = fn()
            tb = timeit(lambda: torch.autograd.grad(y, (x, conv.weight), g, retain_graph=True))
            res[eng] = (tf, tb)
        print(f"{name:18s} " + "  ".join(f"{e}: fwd {tf:.3f} ms ({fl / tf / 1e9:.0f} TF) bwd {tb:.3f} ms ({2 * fl / tb / 1e9:.0f} TF)"
                                         for e, (tf, tb) in res.items()), flush=True)
        del x, g, conv


if __name__ == "__main__":
    main()
