"""A/B builds: libbm2f.so with one source recompiled under extra defines, into tools/lib/libbm2f_<name>.so.

    python tools/build_variant.py NAME SOURCE.hip -DMACRO=VALUE ...

The other objects are the main build's (bm2f_amd/build_obj, built first).  Load a variant with the benches' --lib.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bm2f_amd import build as b  # noqa: E402


def main():
    name, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
    b.build()
    objs = [os.path.join(b.OBJ, f) for f in sorted(os.listdir(b.OBJ)) if f.endswith(".o")]
    vobj = os.path.join(b.OBJ, "variant_" + name + ".o")
    path = os.path.join(b.CSRC, src)
    subprocess.run([b._hipcc(), *b.CXXFLAGS, *b.FILE_FLAGS.get(src, []), *defs, "-c", path, "-o", vobj], check=True)
    objs = [o for o in objs if os.path.basename(o) != src + ".o" and not os.path.basename(o).startswith("variant_")]
    out = os.path.join(ROOT, "tools", "lib", f"libbm2f_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([b._hipcc(), f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", out, *objs, vobj], check=True)
    os.remove(vobj)
    print(out)


if __name__ == "__main__":
    main()
