"""Pins oracle/pixdec_ref.py (the functional restatement of the reference's forward_features, the checker of the
production-size pixel-decoder test on the GPU) against pixdec.npz, which the reference produced here
(tests/golden/gen_golden.py): outputs, input gradients and the fixture's parameter gradients, in fp64 on CPU
against the reference's fp32 run."""
import torch

from module_cases import PIXDEC_SHAPES, build_pixdec, rel_err
from conftest import golden


def test_pixdec_ref_matches_reference_fixture():
    from oracle import pixdec_ref
    m = build_pixdec()
    g = golden("pixdec.npz")
    feats = {k: torch.from_numpy(g[f"in_{k}"]).double().requires_grad_() for k in PIXDEC_SHAPES}
    P = pixdec_ref.params_like(m, torch.float64)
    mf, o0, ms = pixdec_ref.forward_features(m, P, feats, torch.float64)
    outs = [mf, o0] + list(ms)
    names = ["out_mask_features", "out_out0", "out_ms0", "out_ms1", "out_ms2"]
    for name, o in zip(names, outs):
        assert rel_err(o.detach(), g[name]) < 1e-5, name
    grads = [torch.from_numpy(g[f"outgrad_{i}"]).double() for i in range(len(outs))]
    torch.autograd.backward(outs, grads)
    for k, v in feats.items():
        assert rel_err(v.grad, g[f"ingrad_{k}"]) < 1e-4, k
    n = 0
    for key in g.files:
        if key.startswith("pgrad_"):
            assert rel_err(P[key[6:]].grad, g[key]) < 1e-4, key
            n += 1
    assert n > 0
