"""torch.profiler op-level table of one training step (device time per aten op).
python tools/op_profile.py [--batch 16] [--part pixdec|all] [--rows 40]"""
import argparse
import os
import sys

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bm2f_amd.bench_model import MaskFormerR50, make_optimizer, train_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=45)
    ap.add_argument("--part", default="all")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = MaskFormerR50().to(dev)
    opt = make_optimizer(model)
    x = torch.randn(a.batch, 3, a.res, a.res, device=dev) * 57 + 117
    if a.part == "pixdec":
        feats = {k: torch.randn(a.batch, c, a.res // s, a.res // s, device=dev, requires_grad=True)
                 for k, (c, s) in {"res2": (256, 4), "res3": (512, 8), "res4": (1024, 16), "res5": (2048, 32)}.items()}

        def step():
            mf, o0, ms = model.pixel_decoder.forward_features(feats)
            (mf.mean() + sum(t.mean() for t in ms)).backward()
    else:
        def step():
            train_step(model, opt, x, torch.bfloat16)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=60))


if __name__ == "__main__":
    main()
