"""Phase shares of the tiled MSDA backward from s_memtime stamps (diagnostic build, M2F_DIAG).

    python tools/msda_stamps.py [--build] [--n 16]

Builds tools/lib/libbm2f_diag.so from bm2f_amd/csrc (msda.hip with -DM2F_DIAG) when --build is given (on the CPU
container), then on the GPU runs the stamped kernel at config 2 shapes (reference-init sampling, as
tools/msda_bench.py) and prints, over workgroups, the median cycles of each phase and the kernel time.  The
stamped build adds one barrier; read its shares, not its length.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "lib", "libbm2f_diag.so")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    csrc = os.path.join(ROOT, "bm2f_amd", "csrc")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950", "-DM2F_DIAG",
           "-munsafe-fp-atomics", "-I" + os.path.join(ROOT, "include"), "-I" + csrc, os.path.join(csrc, "msda.hip"),
           os.path.join(csrc, "eltwise.hip"), "-o", LIB]   # eltwise.hip: m2f::zero_async
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--lib", default=LIB, help="diagnostic library to load (default: the --build output)")
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--threads", type=int, default=512)
    ap.add_argument("--tile", type=int, default=0, help="tile edge on the finest level (0: the default)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE", help="library option, repeatable")
    a = ap.parse_args()
    if a.build:
        build()
        return
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from msda_bench import make_inputs
    shapes = [(32, 32), (64, 64), (128, 128)]
    v, st, lsi, loc, attn, gout = make_inputs(a.n, shapes, noise=a.noise)
    lib = ctypes.CDLL(a.lib)
    p, i = ctypes.c_void_p, ctypes.c_int
    fn = lib.m2f_diag_msda_bwd_stamps_f32
    fn.argtypes = [p, p, p, p, i, i, i, i, p, p, p, p, p, i, p]
    N, S, M = v.shape[0], v.shape[1], v.shape[2]
    gv = torch.empty_like(v)
    gl = torch.empty_like(loc)
    ga = torch.empty_like(attn)
    import math as _m
    thr = a.threads
    th = a.tile or (16 if thr >= 1024 else 12)
    tw = th
    lib.m2f_set_option.argtypes = [ctypes.c_char_p, ctypes.c_int64]
    lib.m2f_set_option(b"msda_threads", thr)
    lib.m2f_set_option(b"msda_tile", th)
    for kv in a.opt:
        k, v_ = kv.split("=")
        lib.m2f_set_option(k.encode(), int(v_))
    nwg = _m.ceil(128 / th) * _m.ceil(128 / tw) * M * N
    stamps = torch.zeros(nwg * 8, dtype=torch.int64, device=v.device)
    hs = (ctypes.c_int64 * 6)(*[x for hw in shapes for x in hw])
    stream = torch.cuda.current_stream().cuda_stream
    for noflush in (1, 0):
      ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
      for it in range(4):
        if it == 1:
            ev[0].record()
        rc = fn(v.data_ptr(), loc.data_ptr(), attn.data_ptr(), gout.data_ptr(), N, S, M, 3, ctypes.cast(hs, p),
                gv.data_ptr(), gl.data_ptr(), ga.data_ptr(), stamps.data_ptr(), noflush, stream)
        assert rc == 0
      ev[1].record()
      torch.cuda.synchronize()
      print(f"noflush={noflush}: {ev[0].elapsed_time(ev[1]) / 3:.3f} ms per launch (stamped build)")
      report(stamps, nwg)


def report(stamps, nwg):
    import torch
    st = stamps.view(nwg, 8).double()
    s = torch.stack([st[:, 5], st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4]], 1)  # entry, then phase ends
    d = (s[:, 1:] - s[:, :5])
    med = d.median(0).values
    tot = (s[:, 5] - s[:, 0]).median()
    names = ["setup", "phase0 g+desc+bbox", "window+sort", "phase2 gather+grads", "phase3 walk+flush"]
    for n_, m_ in zip(names, med.tolist()):
        print(f"{n_:28s} {m_:10.0f} cycles  {100 * m_ / tot:5.1f} %")
    span = (s[:, 5].max() - s[:, 0].min()).item()
    print(f"per-workgroup median {tot:.0f} cycles; kernel span {span:.0f} cycles (s_memtime ticks)")


if __name__ == "__main__":
    main()
