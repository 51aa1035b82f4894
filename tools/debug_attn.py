import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bm2f_amd import decoder_ops
from oracle.decoder_ref import pack_bits, ref_masked_attention
dev = torch.device("cuda")
for dt in (torch.float32, torch.bfloat16):
    for (B, Lq, Lk) in [(1, 16, 64), (1, 100, 64), (2, 100, 128), (2, 100, 1024)]:
        g = torch.Generator(device=dev).manual_seed(0)
        H = 8; C = 256
        q = torch.randn(B, Lq, C, device=dev, generator=g).to(dt)
        k = torch.randn(B, Lk, C, device=dev, generator=g).to(dt)
        v = torch.randn(B, Lk, C, device=dev, generator=g).to(dt)
        blocked = torch.rand(B, Lq, Lk, device=dev, generator=g) < 0.0
        out = decoder_ops.masked_attention(q, k, v, pack_bits(blocked), H)
        ref = ref_masked_attention(q, k, v, blocked, H)
        nan = torch.isnan(out)
        err = (out.float() - ref).abs().nan_to_num(1e9).max().item()
        rows = nan.any(-1).nonzero()[:5].tolist()
        cols = nan.any(1).nonzero()[:8].tolist()
        print(dt, B, Lq, Lk, "nan", nan.sum().item(), "err", err, "rows", rows, "cols", cols, flush=True)
