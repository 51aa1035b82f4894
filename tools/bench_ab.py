"""bench.py with Python-level switches flipped first (A/B of host-side choices that have no library option).

    python tools/bench_ab.py --set bm2f_amd.bench_model.CONV1X1_GEMM=0 -- [bench.py arguments]

Each --set MODULE.ATTR=VALUE assigns VALUE converted to the attribute's type (int, bool or str) before bench.main()
runs; e.g. --set bm2f_amd._native._LIB_PATH=tools/lib/libbm2f_x.so times another build of the library."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    sets = []
    while argv and argv[0] == "--set":
        sets.append(argv[1])
        argv = argv[2:]
    if argv and argv[0] == "--":
        argv = argv[1:]
    for s in sets:
        path, val = s.split("=")
        mod, attr = path.rsplit(".", 1)
        m = importlib.import_module(mod)
        old = getattr(m, attr)
        setattr(m, attr, os.path.abspath(val) if isinstance(old, str) else type(old)(int(val)))
        print(f"[bench_ab] {path} = {getattr(m, attr)!r}", file=sys.stderr, flush=True)
    sys.argv = [os.path.join(ROOT, "bench.py")] + argv
    import bench
    bench.main()


if __name__ == "__main__":
    main()
