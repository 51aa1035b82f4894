"""Which op separates the HIP decoder path from the fp32 reference at full size (tests/decoder_parity.py)?
Runs the teacher-forced comparison with the self-attention's SDPA backend forced to MATH and/or the HIP masked
attention swapped for its torch restatement, and prints the failing / worst tensors of each arm.

    python tools/decoder_parity_diag.py [--config 5|2|4]"""
import argparse
import contextlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from torch.nn.attention import SDPBackend, sdpa_kernel  # noqa: E402

import decoder_parity as dp  # noqa: E402


def build(config, dev):
    torch.manual_seed(0)
    if config == 5:
        from bm2f_amd.video_decoder import VideoMultiScaleMaskedTransformerDecoder
        T, clips = 5, 2
        dec = VideoMultiScaleMaskedTransformerDecoder(256, True, num_classes=40, hidden_dim=256, num_queries=100,
                                                      nheads=8, dim_feedforward=2048, dec_layers=9, pre_norm=False,
                                                      mask_dim=256, enforce_input_project=False, num_frames=T).to(dev)
        g = torch.Generator(device=dev).manual_seed(4)
        xs = [torch.randn(clips * T, 256, h, w, device=dev, generator=g) for h, w in ((12, 20), (24, 40), (48, 80))]
        mf = torch.randn(clips * T, 256, 96, 160, device=dev, generator=g)
        return dec, xs, mf
    from bm2f_amd.transformer_decoder import MultiScaleMaskedTransformerDecoder
    Q, K = (100, 133) if config == 2 else (200, 80)
    dec = MultiScaleMaskedTransformerDecoder(256, True, num_classes=K, hidden_dim=256, num_queries=Q, nheads=8,
                                             dim_feedforward=2048, dec_layers=9, pre_norm=False, mask_dim=256,
                                             enforce_input_project=False).to(dev)
    g = torch.Generator(device=dev).manual_seed(9)
    xs = [torch.randn(2, 256, h, h, device=dev, generator=g) for h in (32, 64, 128)]
    mf = torch.randn(2, 256, 256, 256, device=dev, generator=g)
    return dec, xs, mf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for arm, math, hip in (("default", False, True), ("sdpa_math", True, True), ("ref_attention", False, False),
                           ("sdpa_math+ref_attention", True, False)):
        dec, xs, mf = build(a.config, dev)
        ctx = sdpa_kernel([SDPBackend.MATH]) if math else contextlib.nullcontext()
        with ctx:
            lines, bad, n_bits, n_diff = dp.decoder_parity(dec, xs, mf, dev, hip=hip)
        worst = sorted((ln for ln in lines if " hip max " in ln), key=lambda ln: -float(ln.split("hip max ")[1].split()[0]))
        print(f"== {arm}: failures {bad}; bits {n_diff}/{n_bits}", flush=True)
        for ln in worst[:6]:
            print("   " + ln, flush=True)


if __name__ == "__main__":
    main()
