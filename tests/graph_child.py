"""Child process of ``test_graph_step_packet_capture``: the bitwise graph-vs-eager check of
``test_graph_step_matches_eager`` run in a fresh process, so that ``DEBUG_CLR_GRAPH_PACKET_CAPTURE`` (read once when the
HIP runtime initialises) takes the value the parent put in the environment -- bench.py's graph runs of configs 4 / 5 keep
the runtime's graph packet capture on.  Exits 0 and prints ``GRAPH_OK`` when every replayed step's loss and every
parameter equal the eager copy's bit for bit.

    DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python tests/graph_child.py --swin swin_l --amp fp16 --replays 4
"""
import argparse
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--swin", default="swin_l")
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--amp", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--replays", type=int, default=4)
    a = ap.parse_args()
    import torch
    from torch.nn.attention import SDPBackend, sdpa_kernel

    from bm2f_amd import _native
    from bm2f_amd.bench_model import GraphStep, HeadBench, head_features, make_optimizer, make_scaler, train_step
    dev = torch.device("cuda:0")
    amp = {"fp16": torch.float16, "bf16": torch.bfloat16}[a.amp]
    frames = a.frames or None
    print(f"packet capture env: {os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')!r}", flush=True)
    torch.manual_seed(0)
    n = 2 * (frames or 1)
    base = HeadBench(a.swin, 20, 10, frames=frames).to(dev)
    eager = copy.deepcopy(base)
    feats = head_features(a.swin, n, 256, 256, dev, seed=3)
    feats_e = {k: v.detach().clone().requires_grad_() for k, v in feats.items()}
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    with _native.options(msda_bwd_det=1), sdpa_kernel([SDPBackend.MATH]):
        opt_g, opt_e = make_optimizer(base, capturable=True), make_optimizer(eager, capturable=True)
        sc_g, sc_e = make_scaler(amp), make_scaler(amp)
        g = GraphStep(base, opt_g, feats, amp, scaler=sc_g, warmup=2)
        print(f"captured nodes: {g.nodes}", flush=True)
        if g.nodes.get("memset"):
            print("FAIL: memset node in the captured step", flush=True)
            return 1
        for _ in range(2):
            train_step(eager, opt_e, feats_e, amp, scaler=sc_e)
        bad = 0
        for i in range(a.replays):
            lg = g().clone()
            le = train_step(eager, opt_e, feats_e, amp, scaler=sc_e)
            torch.cuda.synchronize()
            nd = sum(int(not torch.equal(pg, pe)) for pg, pe in zip(base.parameters(), eager.parameters()))
            same = bool(torch.isfinite(lg)) and torch.equal(lg, le)
            print(f"replay {i + 1}: graph loss {lg.item():.9g} eager {le.item():.9g} equal {same} "
                  f"params differing {nd}", flush=True)
            bad += int(not same) + nd
    if bad:
        print("FAIL", flush=True)
        return 1
    print("GRAPH_OK", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
