"""Weak-supervision criterion benchmark at the config-2 shapes (16 images of 1024^2, Q=100, K=133,
masks 256^2, 10 decoder heads), SURVEY 8(f) ranks 1 and 3.

    python tools/criterion_bench.py [--batch 16] [--queries 100] [--res 1024] [--iters 10]

Times on the GPU (HIP events around synchronised regions):
  prep      bm2f_amd.weaksup.prepare_weaksup_targets (Lab + colour similarity + box rasters)
  match     one HungarianMatcherProjPair call (batched costs + one LSAP launch)
  crit_fwd  SetCriterionProjPair forward over 10 heads (10 matcher calls + 30 losses)
  crit_fb   forward + backward of the summed losses
and, for the same cost matrices, the host work the reference does instead of the GPU LSAP
(matcher.py:309-311): per image per head a device->host copy of C and scipy's linear_sum_assignment.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bm2f_amd import weaksup  # noqa: E402
from bm2f_amd.criterion import HungarianMatcherProjPair, SetCriterionProjPair, WeakTargets  # noqa: E402


def synth_targets(B, res, gen, device):
    images, tg = [], []
    for _ in range(B):
        blocks = torch.rand(3, res // 64, res // 64, generator=gen) * 255
        img = torch.nn.functional.interpolate(blocks[None], size=(res, res), mode="bilinear",
                                              align_corners=False)[0]
        img = (img + torch.randint(-2, 3, (3, res, res), generator=gen)).clamp(0, 255).to(torch.uint8)
        G = int(torch.randint(1, 21, (1,), generator=gen))
        xy = torch.rand(G, 2, generator=gen) * (res - 64)
        wh = 16 + torch.rand(G, 2, generator=gen) * (res / 2)
        boxes = torch.cat([xy, torch.minimum(xy + wh, torch.tensor(res - 1.0))], 1)
        images.append(img.to(device))
        tg.append({"boxes": boxes, "labels": torch.randint(0, 133, (G,), generator=gen)})
    return images, tg


def timed(fn, iters):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        out = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--queries", type=int, default=100)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--heads", type=int, default=10)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(0)
    B, Q, K, h = a.batch, a.queries, 133, a.res // 4
    images, tg = synth_targets(B, a.res, gen, dev)
    heights = [a.res] * B
    prep = lambda: weaksup.prepare_weaksup_targets(tg, images, heights)  # noqa: E731
    prep()
    t_prep, targets = timed(prep, a.iters)
    heads = [{"pred_logits": (torch.randn(B, Q, K + 1, device=dev) * 2).requires_grad_(),
              "pred_masks": (torch.randn(B, Q, h, h, device=dev) * 3).requires_grad_()} for _ in range(a.heads)]
    outputs = dict(heads[-1], aux_outputs=heads[:-1])
    matcher = HungarianMatcherProjPair(2.0, 5.0, 5.0, pairwise_warmup_iters=1)
    crit = SetCriterionProjPair(K, matcher, {}, 0.1, 3, 2, 0.3, 1, ["labels", "projection_masks", "pairwise"],
                                False, 0, 3.0, 0.75).to(dev)
    tgw = WeakTargets(targets, dev, 0.3)
    with torch.no_grad():
        matcher(heads[0], targets, prepared=tgw)
        t_match, _ = timed(lambda: matcher(heads[0], targets, prepared=tgw), a.iters)
    for _ in range(2):
        sum(crit(outputs, targets).values()).backward()
    t_fwd, losses = timed(lambda: crit(outputs, targets), a.iters)
    total = sum(losses.values())

    def bwd():
        l = sum(crit(outputs, targets).values())
        l.backward()
    t_fb, _ = timed(bwd, a.iters)

    # the reference's host side for the same costs: C.cpu() per image then scipy, per head
    from scipy.optimize import linear_sum_assignment
    with torch.no_grad():
        Cs = [matcher.cost_matrix(hd, tgw, 1.0) for hd in heads]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for C in Cs:
        for b in range(B):
            c = C[b, :, :tgw.G[b]].cpu()
            linear_sum_assignment(c)
    t_host = (time.perf_counter() - t0) * 1e3
    res = {"batch": B, "queries": Q, "mask_hw": h, "heads": a.heads, "targets": tgw.G,
           "prep_ms": round(t_prep, 3), "match_ms_per_head": round(t_match, 3),
           "criterion_fwd_ms": round(t_fwd, 3), "criterion_fwd_bwd_ms": round(t_fb, 3),
           "reference_host_lsap_ms_per_step": round(t_host, 3), "loss": float(total)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
