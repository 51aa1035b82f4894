"""Per-stage timing of the benchmark training step with HIP events (fwd per module, bwd per module via
grad hooks, clip + optimizer).  python tools/step_breakdown.py [--batch 16] [--res 1024] [--amp bf16]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bm2f_amd.miopen_tuning import use_shipped_find_db  # noqa: E402

use_shipped_find_db()
import torch  # noqa: E402

from bm2f_amd.bench_model import MaskFormerR50, make_optimizer, surrogate_loss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--amp", default="bf16")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = MaskFormerR50().to(dev)
    opt = make_optimizer(model)
    amp = {"bf16": torch.bfloat16, "fp16": torch.float16, "none": None}[a.amp]
    x = torch.randn(a.batch, 3, a.res, a.res, device=dev) * 57 + 117
    names = ["start", "backbone_fwd", "pixdec_fwd", "decoder_fwd", "loss", "decoder_bwd", "pixdec_bwd",
             "backbone_bwd", "clip", "opt"]
    tot = {n: 0.0 for n in names[1:]}
    for it in range(a.steps + 1):
        ev = {}

        def mark(name):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev[name] = e

        opt.zero_grad(set_to_none=True)
        mark("start")
        with torch.autocast("cuda", dtype=amp, enabled=amp is not None):
            xx = (x - model.pixel_mean) / model.pixel_std
            feats = model.backbone(xx)
            mark("backbone_fwd")
            mf, _, ms = model.pixel_decoder.forward_features(feats)
            mark("pixdec_fwd")
            out = model.predictor(ms, mf)
            mark("decoder_fwd")
            loss = surrogate_loss(out)
            mark("loss")
        mf.register_hook(lambda g: mark("decoder_bwd"))
        feats["res5"].register_hook(lambda g: mark("pixdec_bwd"))
        loss.backward()
        mark("backbone_bwd")
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.01, foreach=True)
        mark("clip")
        opt.step()
        mark("opt")
        torch.cuda.synchronize()
        if it == 0:
            continue
        for i in range(1, len(names)):
            tot[names[i]] += ev[names[i - 1]].elapsed_time(ev[names[i]]) / a.steps
    total = sum(tot.values())
    for n, v in tot.items():
        print(f"{n:14s} {v:8.2f} ms  {100 * v / total:5.1f}%")
    print(f"{'total':14s} {total:8.2f} ms  -> {a.batch / total * 1e3:.1f} img/s")
    print("peak mem GB", torch.cuda.max_memory_allocated() / 1e9)


if __name__ == "__main__":
    main()
