"""Reductions one eager training step of a bench config issues (aten sum / mean / norm / amax ...), with their input
shape, reduced size per output and the Python frame that called them: the large ones are where torch's reduce
kernel zeroes a semaphore with a memset, which a HIP graph replays wrongly under the runtime's packet capture.

    python tools/reduction_scan.py [--config 4|5] [--min-per-out 1024]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4, choices=[2, 4, 5])
    ap.add_argument("--min-per-out", type=int, default=1024)
    a = ap.parse_args()
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode
    from bm2f_amd.bench_model import HeadBench, head_features, make_optimizer, make_scaler, train_step
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if a.config == 4:
        model = HeadBench("swin_l", 200, 80).to(dev)
        feats = head_features("swin_l", 2, 1024, 1024, dev, seed=1000)
    else:
        model = HeadBench("swin_t", 100, 40, frames=5).to(dev)
        feats = head_features("swin_t", 10, 384, 640, dev, seed=1000)
    opt = make_optimizer(model, capturable=True)
    scaler = make_scaler(torch.float16)
    train_step(model, opt, feats, torch.float16, scaler=scaler)
    torch.cuda.synchronize()
    names = ("sum", "mean", "norm", "linalg_vector_norm", "amax", "amin", "max", "min", "var", "std", "_foreach_norm",
             "prod", "any", "all", "logsumexp", "native_layer_norm_backward", "native_group_norm_backward")
    seen = collections.Counter()
    where = {}

    class Scan(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            base = func.__name__.split(".")[0]
            if base in names and args and isinstance(args[0], torch.Tensor):
                x = args[0]
                outs = out if isinstance(out, (tuple, list)) else (out,)
                on = max(1, sum(o.numel() for o in outs if isinstance(o, torch.Tensor)))
                per = x.numel() // on
                if per >= a.min_per_out:
                    frames = [f for f in traceback.extract_stack() if "torch/" not in f.filename][-3:]
                    site = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(frames))
                    node = torch._C._current_autograd_node()
                    if node is not None:   # backward: the forward call that made the node (anomaly mode)
                        tb = node.metadata.get("traceback_", [])
                        lines = [ln.strip().splitlines()[0] for ln in tb if "bm2f_amd" in ln or "tools/" in ln]
                        site = f"bwd of {node.name()} from " + " <- ".join(
                            ln.split("File ")[-1].replace('"', "") for ln in reversed(lines[-3:]))
                    key = (str(func), tuple(x.shape), str(x.dtype), on, site)
                    seen[key] += 1
                    where[key] = site
            return out

    with torch.autograd.detect_anomaly(check_nan=False), Scan():
        train_step(model, opt, feats, torch.float16, scaler=scaler)
    torch.cuda.synchronize()
    for key, n in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(f"{n:3d}x {key[0]:40s} in {key[1]} {key[2]} -> {key[3]} outputs   {where[key]}")


if __name__ == "__main__":
    main()
