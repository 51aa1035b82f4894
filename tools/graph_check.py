"""Graph replay vs eager, step by step (diagnostic for bench_model.GraphStep).

    python tools/graph_check.py [--swin swin_l] [--frames 0] [--amp fp16|bf16] [--det 1]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bm2f_amd import _native  # noqa: E402
from bm2f_amd.bench_model import GraphStep, HeadBench, head_features, make_optimizer, make_scaler, train_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--swin", default="swin_l")
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--amp", default="fp16")
    ap.add_argument("--det", type=int, default=1)
    ap.add_argument("--scaler", type=int, default=1)
    ap.add_argument("--lr0", type=int, default=0, help="learning rate 0 (parameters constant: every step's loss equal)")
    ap.add_argument("--replays", type=int, default=0, help="replay this many times back to back first, no eager steps between")
    ap.add_argument("--dump", default=None, help="write the captured graph as a dot file here")
    ap.add_argument("--garbage", type=int, default=0, help="after the back-to-back replays: fill freed memory of the "
                    "normal pool with NaN, then replay again (does the graph read memory it does not own?)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    amp = {"fp16": torch.float16, "bf16": torch.bfloat16}[a.amp]
    frames = a.frames or None
    torch.manual_seed(0)
    n = 2 * (frames or 1)
    base = HeadBench(a.swin, 20, 10, frames=frames).to(dev)
    eager = copy.deepcopy(base)
    feats = head_features(a.swin, n, 256, 256, dev, seed=3)
    feats_e = {k: v.detach().clone().requires_grad_() for k, v in feats.items()}
    if a.det:
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.backends.cudnn.deterministic = True
    with _native.options(msda_bwd_det=a.det):
        opt_g, opt_e = make_optimizer(base, capturable=True), make_optimizer(eager, capturable=True)
        if a.lr0:
            for o in (opt_g, opt_e):
                for grp in o.param_groups:
                    grp["lr"] = 0.0
        sc_g = make_scaler(amp) if a.scaler else None
        sc_e = make_scaler(amp) if a.scaler else None
        g = GraphStep(base, opt_g, feats, amp, scaler=sc_g, warmup=2, debug_dump=a.dump)
        if a.replays:
            print("back-to-back replays", [g().item() for _ in range(a.replays)], flush=True)
        if a.garbage:
            junk = [torch.full((1 << k,), float("nan"), device=dev) for k in range(10, 28) for _ in range(3)]
            del junk
            print("after NaN-filled allocations", [g().item() for _ in range(2)], flush=True)
            torch.cuda.empty_cache()
            junk = [torch.full((1 << k,), float("nan"), device=dev) for k in range(10, 28) for _ in range(3)]
            del junk
            print("after empty_cache + NaN-filled allocations", [g().item() for _ in range(2)], flush=True)
            return
        le = [train_step(eager, opt_e, feats_e, amp, scaler=sc_e).item() for _ in range(2)]
        print("eager warm-up losses", le, flush=True)
        for i in range(4):
            lg = g().clone()
            l_e = train_step(eager, opt_e, feats_e, amp, scaler=sc_e)
            torch.cuda.synchronize()
            nd = sum(int(not torch.equal(pg, pe)) for pg, pe in zip(base.parameters(), eager.parameters()))
            sg = sc_g.get_scale() if sc_g else None
            se = sc_e.get_scale() if sc_e else None
            print(f"step {3 + i}: graph {lg.item():.6f} eager {l_e.item():.6f} params differing {nd} scale {sg} {se}", flush=True)


if __name__ == "__main__":
    main()
