"""AMP fp16 decoder vs decoder_amp16.npz, teacher-forced, with the mask-heads kernel on and off: prints
every gradient's relative error for both, to see what the kernel's rounding changes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch

from bm2f_amd import decoder_ops
from conftest import golden
from module_cases import build_decoder, rel_err, run_decoder
from oracle.decoder_ref import pack_bits

dev = torch.device("cuda")
g = golden("decoder_amp16.npz")
real_heads = decoder_ops.mask_heads
real_ok = decoder_ops.MaskFeatureFold.fused_ok
res = {}
for fused in (True, False):
    forced = iter([pack_bits(torch.from_numpy(g[f"attn_mask{i}"])).to(dev) for i in range(9)])

    def heads(fold, embed, size=None):
        out, _ = real_heads(fold, embed, size)
        return out, (next(forced) if size is not None else None)
    decoder_ops.mask_heads = heads
    decoder_ops.MaskFeatureFold.fused_ok = real_ok if fused else (lambda self, q, size=None: False)
    d = build_decoder().to(dev)
    with torch.autocast("cuda", dtype=torch.float16):
        gg, x, mf, logits, masks, _ = run_decoder(d, dev, "decoder_amp16.npz", False)
    r = {"logits": rel_err(torch.stack([t.detach().float().cpu() for t in logits]), g["pred_logits"]),
         "masks": rel_err(torch.stack([t.detach().float().cpu() for t in masks]), g["pred_masks"]),
         "mf": rel_err(mf.grad.cpu(), g["ingrad_mask_features"])}
    for i, t in enumerate(x):
        r[f"x{i}"] = rel_err(t.grad.cpu(), g[f"ingrad_x{i}"])
    params = dict(d.named_parameters())
    for key in g.files:
        if key.startswith("pgrad_"):
            r[key[6:]] = rel_err(params[key[6:]].grad.float().cpu(), g[key])
    res[fused] = r
for k in res[True]:
    print(f"{k:60s} fused {res[True][k]:.3g}  bmm {res[False][k]:.3g}")
