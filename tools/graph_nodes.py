"""Node types of the captured training-step graph (bench_model.GraphStep) at a bench config's full size, through
hipGraphGetNodes: a memset node is what the runtime's packet capture replays wrongly (tools/graph_memset_check.py).

    python tools/graph_nodes.py [--config 4|5] [--math]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4, choices=[4, 5])
    ap.add_argument("--math", action="store_true", help="self-attention on the math backend")
    a = ap.parse_args()
    import torch
    from bm2f_amd.bench_model import GraphStep, HeadBench, head_features, make_optimizer, make_scaler
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if a.config == 4:
        model = HeadBench("swin_l", 200, 80).to(dev)
        feats = head_features("swin_l", 2, 1024, 1024, dev, seed=1000)
    else:
        model = HeadBench("swin_t", 100, 40, frames=5).to(dev)
        feats = head_features("swin_t", 10, 384, 640, dev, seed=1000)
    opt = make_optimizer(model, capturable=True)
    g = GraphStep(model, opt, feats, torch.float16, scaler=make_scaler(torch.float16), warmup=2,
                  sdpa_math=a.math)
    torch.cuda.synchronize()
    print(f"config {a.config} (sdpa {'math' if a.math else 'default'}): {g.nodes}")


if __name__ == "__main__":
    main()
