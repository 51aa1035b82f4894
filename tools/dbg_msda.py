import sys, time, torch, numpy as np
sys.path.insert(0, '.')
from bm2f_amd import msda
from oracle import msda_ref
dev = torch.device("cuda")
for N, uniform in ((1, False), (1, True)):
    shapes = [(32, 32), (64, 64), (128, 128)]
    st = torch.tensor(shapes, dtype=torch.int64)
    lsi = torch.cat((st.new_zeros(1), st.prod(1).cumsum(0)[:-1]))
    S = int(st.prod(1).sum()); M, D, L, P = 8, 32, 3, 4
    g = torch.Generator().manual_seed(0)
    v = torch.randn(N, S, M, D, generator=g)
    if uniform:
        loc = torch.rand(N, S, M, L, P, 2, generator=g)
    else:
        refs = []
        for h, w in shapes:
            ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h), torch.linspace(0.5, w - 0.5, w), indexing="ij")
            refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
        ref = torch.cat(refs, 0)
        norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)
        loc = ref[None, :, None, None, None, :] + torch.randn(N, S, M, L, P, 2, generator=g) * 2 / norm[None, None, None, :, None, :]
    a = torch.rand(N, S, M, L, P, generator=g)
    gout = torch.randn(N, S, M * D, generator=g)
    dst = msda.attach_host_shapes(st.to(dev), shapes)
    torch.cuda.synchronize(); t0 = time.time()
    gv, gl, ga = msda.ms_deform_attn_backward(v.to(dev), dst, lsi.to(dev), loc.contiguous().to(dev), a.to(dev), gout.to(dev), 64)
    torch.cuda.synchronize(); t1 = time.time()
    wv, wl, wa = msda_ref.msda_backward(v.double(), st, lsi, loc.double(), a.double(), gout.double())
    for name, got, want in (("gv", gv, wv), ("gl", gl, wl), ("ga", ga, wa)):
        got = got.cpu().double().numpy()
        err = np.abs(got - want).max() / np.abs(want).max()
        print(f"N={N} uniform={uniform} {name} err={err:.3e} nan={np.isnan(got).sum()} t={t1-t0:.3f}s", flush=True)
