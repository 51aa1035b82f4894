"""Build ``bm2f_amd/lib/libbm2f.so`` from ``bm2f_amd/csrc/*.hip`` for gfx950 (in-tree, no JIT cache).

    python -m bm2f_amd.build [--force] [--verbose]

hipcc cross-compiles on a host without a GPU; the resulting .so travels with the repo snapshot.
Objects are rebuilt only when a source or header is newer than the object.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build_obj")
LIB = os.path.join(PKG, "lib", "libbm2f.so")
INCLUDE = os.path.join(ROOT, "include")
ARCH = "gfx950"
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I" + INCLUDE, "-I" + CSRC,
            "-Wno-pass-failed", "-munsafe-fp-atomics"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _newest_dep() -> float:
    deps = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return max((os.path.getmtime(d) for d in deps), default=0.0)


# per-file flags: the MFMA-dense x3 kernels must not get SLP-packed f32 VALU (v_pk_add_f32 beside MFMAs
# costs more issue than two scalar ops, MI355X_MICROARCH.md)
FILE_FLAGS = {"gemm_x3.hip": ["-fno-slp-vectorize"], "conv_x3.hip": ["-fno-slp-vectorize"]}


def _compile(src: str, force: bool, verbose: bool) -> str:
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if (not force and os.path.exists(obj)
            and os.path.getmtime(obj) >= max(os.path.getmtime(src), _newest_dep(), os.path.getmtime(__file__))):
        return obj
    cmd = [_hipcc(), *CXXFLAGS, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    jobs = min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, verbose), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(force=a.force, verbose=a.verbose))


if __name__ == "__main__":
    sys.exit(main())
