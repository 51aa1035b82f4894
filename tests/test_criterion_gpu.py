"""GPU weak-supervision path (csrc/lsap.hip, csrc/weaksup.hip via bm2f_amd/weaksup.py, criterion.py) against
the reference's outputs (tests/golden/criterion.npz, lsap.npz) and the CPU oracle (oracle/weaksup_ref.py).

Bars: matched indices bit-exact (integer work); losses rtol 1e-5 and gradients rtol 1e-4 (fp32 sums in a
different order); neighbour bits / box masks / bounds exact; Lab similarity 1e-5 (the GPU Lab conversion
and the oracle's are both fp64 then rounded to fp32)."""
import os

import numpy as np
import pytest
import torch

from bm2f_amd import weaksup
from bm2f_amd.criterion import HungarianMatcherProjPair, SetCriterionProjPair
from oracle import weaksup_ref as ref
from test_criterion_cpu import _heads, fixture_targets, prepared_lab_and_masks

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLD, "criterion.npz"))


def _scipy(c):
    from scipy.optimize import linear_sum_assignment
    return linear_sum_assignment(c)


def _solve(device, mats):
    """Batch a list of 2-D cost matrices (padded) through the GPU LSAP; -> list of (rows, cols), status."""
    B = len(mats)
    R = max(m.shape[0] for m in mats)
    C = max(m.shape[1] for m in mats)
    cost = torch.zeros(B, R, C)
    for b, m in enumerate(mats):
        cost[b, :m.shape[0], :m.shape[1]] = torch.from_numpy(m)
    rows = torch.tensor([m.shape[0] for m in mats], dtype=torch.int32, device=device)
    cols = torch.tensor([m.shape[1] for m in mats], dtype=torch.int32, device=device)
    match, status = weaksup.lsap_batched(cost.to(device), cols=cols, rows=rows)
    match = match.cpu().numpy()
    out = []
    for b, m in enumerate(mats):
        r = np.nonzero(match[b, :m.shape[0]] >= 0)[0]
        out.append((r, match[b, r].astype(np.int64)))
    return out, status.cpu().numpy()


def test_lsap_vs_reference_fixture(device):
    z = np.load(os.path.join(GOLD, "lsap.npz"))
    keys = sorted(k for k in z.files if k.startswith("c"))
    mats = [z[k] for k in keys]
    got, status = _solve(device, mats)
    assert (status == 0).all()
    for k, (i, j), m in zip(keys, got, mats):
        want = z["r" + k[1:]]
        # exact same assignment as scipy, ties included (same algorithm, same tie rule)
        assert np.array_equal(np.stack([i, j]), want), k


@pytest.mark.parametrize("shape,B", [((100, 12), 16), ((100, 100), 4), ((300, 64), 3), ((7, 40), 5),
                                     ((1000, 128), 2)])
def test_lsap_random_vs_scipy(device, shape, B):
    g = np.random.default_rng(shape[0] * 7 + shape[1])
    mats = [g.standard_normal(shape).astype(np.float32) for _ in range(B)]
    mats += [g.integers(0, 3, shape).astype(np.float32)]             # heavy ties
    got, status = _solve(device, mats)
    assert (status == 0).all()
    for (i, j), m in zip(got, mats):
        wi, wj = _scipy(m)
        assert np.array_equal(i, wi) and np.array_equal(j, wj)


def test_lsap_invalid_entries(device):
    a = np.random.default_rng(0).standard_normal((10, 4)).astype(np.float32)
    nan, ninf, allinf = a.copy(), a.copy(), np.full((6, 3), np.inf, np.float32)
    nan[3, 1] = np.nan
    ninf[0, 0] = -np.inf
    _, status = _solve(device, [a, nan, ninf, allinf])
    assert status.tolist() == [0, 3, 3, 1]
    with pytest.raises(ValueError, match="invalid numeric entries"):
        weaksup.raise_on_lsap_status(torch.tensor(status))


@pytest.mark.parametrize("N,H,W,d", [(3, 32, 32, 2), (5, 45, 70, 2), (2, 17, 130, 1), (4, 64, 64, 3)])
def test_pairwise_kernels_vs_oracle(device, N, H, W, d):
    g = torch.Generator().manual_seed(N * H + W)
    x = torch.randn(N, H, W, generator=g) * 4
    x[0, :3, :3] = 40.0                                        # saturated logits
    x[-1, -2:, :] = -35.0
    sim = torch.rand(N, 8, H, W, generator=g)
    box = (torch.rand(N, H, W, generator=g) < 0.7).float()
    s_ref = ref.pred_similarity(x.double(), d)                                          # (N, 8, H, W)
    planes = weaksup.pairwise_planes(x.to(device), d).cpu()
    torch.testing.assert_close(planes.double(), s_ref, rtol=1e-5, atol=1e-5)
    bits = weaksup.threshold_bits(sim.to(device), 0.3)
    t = (sim >= 0.3)
    want_bits = (t.to(torch.int32) << torch.arange(8)[None, :, None, None]).sum(1)
    assert torch.equal(bits.cpu().to(torch.int32), want_bits)
    rows = torch.arange(N, dtype=torch.int32, device=device)
    A = weaksup.pairwise_map(x.to(device), bits, rows, d).cpu()
    torch.testing.assert_close(A.double(), (s_ref * t).sum(1), rtol=1e-5, atol=1e-5)
    # fused loss sums + gradient vs fp64 autograd of the oracle
    xg = x.to(device).requires_grad_()
    num, den = weaksup.pairwise_sums(xg, bits, rows, box.to(device).contiguous(), rows, d)
    gscale = torch.randn(N, generator=g)
    (num * gscale.to(device)).sum().backward()
    xd = x.double().requires_grad_()
    T = t.double() * box.double()[:, None]
    num_ref = (ref.pred_similarity(xd, d) * T).sum((1, 2, 3))
    (num_ref * gscale.double()).sum().backward()
    torch.testing.assert_close(num.cpu().double(), num_ref.detach(), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(den.cpu().double(), T.sum((1, 2, 3)), rtol=0, atol=0)
    torch.testing.assert_close(xg.grad.cpu().double(), xd.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B,Q,H,W,G", [(2, 5, 32, 32, 3), (3, 7, 45, 130, 9), (1, 4, 16, 20, 0)])
def test_match_cost_kernel_vs_oracle(device, B, Q, H, W, G):
    g = torch.Generator().manual_seed(B * 100 + W)
    x = torch.randn(B, Q, H, W, generator=g) * 4
    sim = torch.rand(B, 8, H, W, generator=g)
    box = (torch.rand(B, max(G, 1), H, W, generator=g) < 0.4).float()[:, :G]
    gcount = torch.tensor([G] * (B - 1) + [max(G - 2, 0)], dtype=torch.int32)
    bits = weaksup.threshold_bits(sim.to(device), 0.3)
    num, sx, sy = weaksup.match_cost(x.to(device), bits, box.to(device).contiguous(), gcount.to(device), 2)
    assert torch.equal(sx.cpu(), x.amax(3)) and torch.equal(sy.cpu(), x.amax(2))
    s_ref = ref.pred_similarity(x.double().view(B * Q, H, W), 2).view(B, Q, 8, H, W)
    A = (s_ref * (sim >= 0.3)[:, None].double()).sum(2)                               # (B, Q, H, W)
    want = torch.einsum("bqhw,bghw->bqg", A, box.double())
    for b in range(B):
        want[b, :, int(gcount[b]):] = 0
    torch.testing.assert_close(num.cpu().double(), want, rtol=1e-5, atol=1e-4)


def test_target_prep_vs_reference(device, gold):
    z = gold
    B = len(z["heights"])
    images = [torch.from_numpy(z[f"image{b}"]).to(device) for b in range(B)]
    tg = [{"boxes": torch.from_numpy(z[f"boxes{b}"]), "labels": torch.from_numpy(z[f"labels{b}"])} for b in range(B)]
    out = weaksup.prepare_weaksup_targets(tg, images, list(z["heights"]))
    _, lab_ref, msk = prepared_lab_and_masks(z)
    pad = torch.zeros(B, 3, 128, 128)
    for b, im in enumerate(images):
        pad[b, :, :im.shape[1], :im.shape[2]] = im.float().cpu()
    lab = weaksup.images_lab(pad.to(device), 4).cpu()
    torch.testing.assert_close(lab, lab_ref, rtol=1e-6, atol=1e-5)
    for b, t in enumerate(out):
        for key in ("box_masks", "left_bounds", "right_bounds", "top_bounds", "bottom_bounds"):
            assert np.array_equal(t[key].cpu().numpy(), z[f"{key}{b}"]), key
        sim = t["images_color_similarity"]
        assert sim.shape[0] <= 1 or sim.stride(0) == 0        # zero-copy view of the image's map
        np.testing.assert_allclose(sim[0].cpu().numpy(), z[f"sim{b}"], rtol=1e-5, atol=1e-6)
        assert torch.equal(t["labels"].cpu(), torch.from_numpy(z[f"labels{b}"]))


def _to(targets, device):
    return [{k: v.to(device) for k, v in t.items()} for t in targets]


@pytest.mark.parametrize("shared", [False, True])
def test_criterion_vs_reference(device, gold, shared):
    z = gold
    w_class, w_proj, w_pair = (float(v) for v in z["weights"])
    K, warmup, n_aux = int(z["K"]), int(z["warmup"]), int(z["n_aux"])
    weights = {"loss_ce": w_class, "loss_mask_projection": w_proj, "loss_pairwise": w_pair}
    matcher = HungarianMatcherProjPair(cost_class=w_class, cost_projection=w_proj, cost_pairwise=w_pair,
                                       pairwise_size=3, pairwise_dilation=2, pairwise_color_thresh=0.3,
                                       pairwise_warmup_iters=warmup)
    crit = SetCriterionProjPair(K, matcher=matcher, weight_dict=weights, eos_coef=0.1, pairwise_size=3,
                                pairwise_dilation=2, pairwise_color_thresh=0.3, pairwise_warmup_iters=warmup,
                                losses=["labels", "projection_masks", "pairwise"], point_sample=False,
                                num_points=0, oversample_ratio=3.0, importance_sample_ratio=0.75).to(device)
    targets = _to(fixture_targets(z, shared=shared), device)
    if shared:
        targets = [dict(t, images_color_similarity=t["images_color_similarity"][:1].expand_as(
            t["images_color_similarity"])) for t in targets]
    seen = []
    orig = matcher.memory_efficient_forward

    def spy(*a, **k):
        r = orig(*a, **k)
        seen.append(r)
        return r

    matcher.memory_efficient_forward = spy
    for it in range(int(z["iters"])):
        heads = [{k: v.detach().to(device).requires_grad_() for k, v in h.items()} for h in _heads(z, it)]
        outputs = dict(heads[-1], aux_outputs=heads[:-1])
        seen.clear()
        losses = crit(outputs, targets)
        assert sorted(losses) == sorted(z["loss_keys"].tolist())
        for k, v in losses.items():
            np.testing.assert_allclose(v.item(), float(z[f"it{it}_{k}"]), rtol=1e-5, atol=1e-7, err_msg=k)
        for call, h in enumerate([n_aux] + list(range(n_aux))):
            for b, (i, j) in enumerate(seen[call]):
                assert np.array_equal(np.stack([i.cpu().numpy(), j.cpu().numpy()]), z[f"it{it}_idx{h}_{b}"])
        total = sum(v * weights[k.rsplit("_", 1)[0] if k[-1].isdigit() else k] for k, v in losses.items())
        total.backward()
        for h, hd in enumerate(heads):
            np.testing.assert_allclose(hd["pred_logits"].grad.cpu().numpy(), z[f"it{it}_glogits{h}"], rtol=1e-4,
                                       atol=1e-7)
            np.testing.assert_allclose(hd["pred_masks"].grad.cpu().numpy(), z[f"it{it}_gmasks{h}"], rtol=1e-4,
                                       atol=1e-8)
    assert float(crit._iter) == z["iters"] and float(matcher._iter) == z["iters"] * (n_aux + 1)


def test_criterion_random_vs_oracle(device):
    """Larger case, including an image without targets and more targets than queries."""
    g = torch.Generator().manual_seed(11)
    B, Q, K, H, W = 4, 30, 9, 48, 40
    G = [7, 0, 35, 12]
    targets = []
    for b in range(B):
        boxes = torch.rand(G[b], 4, generator=g) * torch.tensor([W, H, W, H]) * 4
        boxes[:, 2:] = torch.maximum(boxes[:, 2:], boxes[:, :2] + 3)
        bm = ref.box_targets(boxes, H * 4, W * 4, 4)[0]
        sim = torch.rand(8, H, W, generator=g)
        targets.append({"labels": torch.randint(0, K, (G[b],), generator=g), "box_masks": bm,
                        "images_color_similarity": sim[None].repeat(G[b], 1, 1, 1)})
    heads = [{"pred_logits": torch.randn(B, Q, K + 1, generator=g) * 2,
              "pred_masks": torch.randn(B, Q, H, W, generator=g) * 3} for _ in range(2)]
    warmup = 2
    for shared in (False, True):
        matcher = HungarianMatcherProjPair(2.0, 5.0, 5.0, pairwise_warmup_iters=warmup)
        crit = SetCriterionProjPair(K, matcher, {}, 0.1, 3, 2, 0.3, warmup, ["labels", "projection_masks", "pairwise"],
                                    False, 0, 3.0, 0.75).to(device)
        tdev = _to(targets, device)
        if shared:
            tdev = [dict(t, images_color_similarity=t["images_color_similarity"][:1].expand_as(
                t["images_color_similarity"])) if t["labels"].numel() else t for t in tdev]
        dh = [{k: v.to(device).requires_grad_() for k, v in h.items()} for h in heads]
        losses = crit(dict(dh[-1], aux_outputs=dh[:-1]), tdev)
        sum(losses.values()).backward()
        # oracle with the same warm-up schedule: matcher calls 1, 2 -> 1/2, 1; criterion iter 1 -> 1/2
        oh = [{k: v.clone().requires_grad_() for k, v in h.items()} for h in heads]
        total, want = 0.0, {}
        for call, h in enumerate([1, 0]):
            idx = ref.match(oh[h], targets, 2.0, 5.0, 5.0, 0.3, 2, min((call + 1) / warmup, 1.0))
            ls = ref.losses(oh[h], targets, idx, float(sum(G)), K, 0.1, 0.3, 2, 0.5)
            sfx = "" if h == 1 else "_0"
            want.update({k + sfx: v for k, v in ls.items()})
            total = total + sum(ls.values())
        total.backward()
        for k, v in want.items():
            np.testing.assert_allclose(losses[k].item(), v.item(), rtol=1e-5, atol=1e-7, err_msg=k)
        for a, o in zip(dh, oh):
            for k in a:
                np.testing.assert_allclose(a[k].grad.cpu().numpy(), o[k].grad.numpy(), rtol=1e-4, atol=1e-8)
