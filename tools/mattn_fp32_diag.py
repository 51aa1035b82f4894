"""fp32 masked attention on the decoder's own inputs: the HIP kernels and the torch fp32 restatement, each against
fp64, per cross-attention call (out, dQ, dK, dV; max-normalised and norm errors).

    python tools/mattn_fp32_diag.py [--config 5|2|4]

The decoder (config 5: the video decoder at full per-rank size; 2 / 4: the image decoder) runs once in fp32 with a
wrapper around decoder_ops.masked_attention that records each call's q, k, v, bits and incoming gradient."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bm2f_amd import decoder_ops  # noqa: E402
from oracle.decoder_ref import ref_masked_attention, unpack_bits  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if a.config == 5:
        from bm2f_amd.video_decoder import VideoMultiScaleMaskedTransformerDecoder
        T, clips = 5, 2
        dec = VideoMultiScaleMaskedTransformerDecoder(256, True, num_classes=40, hidden_dim=256, num_queries=100,
                                                      nheads=8, dim_feedforward=2048, dec_layers=9, pre_norm=False,
                                                      mask_dim=256, enforce_input_project=False, num_frames=T).to(dev)
        g = torch.Generator(device=dev).manual_seed(4)
        xs = [torch.randn(clips * T, 256, h, w, device=dev, generator=g) for h, w in ((12, 20), (24, 40), (48, 80))]
        mf = torch.randn(clips * T, 256, 96, 160, device=dev, generator=g)
    else:
        from bm2f_amd.transformer_decoder import MultiScaleMaskedTransformerDecoder
        Q, K = (100, 133) if a.config == 2 else (200, 80)
        dec = MultiScaleMaskedTransformerDecoder(256, True, num_classes=K, hidden_dim=256, num_queries=Q, nheads=8,
                                                 dim_feedforward=2048, dec_layers=9, pre_norm=False, mask_dim=256,
                                                 enforce_input_project=False).to(dev)
        g = torch.Generator(device=dev).manual_seed(9)
        xs = [torch.randn(2, 256, h, h, device=dev, generator=g) for h in (32, 64, 128)]
        mf = torch.randn(2, 256, 256, 256, device=dev, generator=g)
    calls = []
    real = decoder_ops.masked_attention

    def rec(q, k, v, bits, num_heads, scale=None):
        out = real(q, k, v, bits, num_heads, scale)
        entry = {"q": q.detach().clone(), "k": k.detach().clone(), "v": v.detach().clone(), "bits": bits.clone(),
                 "h": num_heads, "scale": scale}
        calls.append(entry)
        if out.requires_grad:
            out.register_hook(lambda gr: entry.__setitem__("g", gr.detach().clone()))
        return out

    decoder_ops.masked_attention = rec
    x = [t.clone().requires_grad_() for t in xs]
    m = mf.clone().requires_grad_()
    out = dec(x, m)
    heads = [out] + out["aux_outputs"]
    loss = sum(h["pred_logits"].mean() + 0.5 * (h["pred_masks"] ** 2).mean() for h in heads)
    loss.backward()
    decoder_ops.masked_attention = real

    def err(a, b):
        return ((a - b).abs().max() / b.abs().max()).item(), ((a - b).norm() / b.norm()).item()

    for i, c in enumerate(calls):
        q, k, v, bits, H = c["q"], c["k"], c["v"], c["bits"], c["h"]
        gout = c.get("g")
        blocked = unpack_bits(bits, k.shape[1])
        res = {}
        for name, dt in (("hip", torch.float32), ("t32", torch.float32), ("f64", torch.float64)):
            qq, kk, vv = (t.detach().to(dt).clone().requires_grad_() for t in (q, k, v))
            o = real(qq, kk, vv, bits, H, c["scale"]) if name == "hip" else ref_masked_attention(qq, kk, vv, blocked, H,
                                                                                                 c["scale"])
            o.backward(gout.to(dt))
            res[name] = [t.detach().double() for t in (o, qq.grad, kk.grad, vv.grad)]
        nvis = (~blocked).sum(-1)
        line = f"call {i}: B {q.shape[0]} Lq {q.shape[1]} Lk {k.shape[1]} visible keys/row min {int(nvis.min())} " \
               f"median {int(nvis.median())}"
        for j, nm in enumerate(("out", "dq", "dk", "dv")):
            eh, et = err(res["hip"][j], res["f64"][j]), err(res["t32"][j], res["f64"][j])
            line += f" | {nm} hip {eh[0]:.1e}/{eh[1]:.1e} t32 {et[0]:.1e}/{et[1]:.1e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
