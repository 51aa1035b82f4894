"""The weak-supervision oracle (oracle/weaksup_ref.py) against the reference's own outputs
(tests/golden/criterion.npz, lsap.npz from tests/golden/gen_criterion_golden.py), plus the criterion's
device-agnostic host logic.  No GPU needed."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import weaksup_ref as ref

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLD, "criterion.npz"))


def test_rgb2lab_known_values():
    # CIE Lab (D65/2deg) of the sRGB primaries, white and black (published colour-table values)
    rgb = np.array([[255, 255, 255], [255, 0, 0], [0, 255, 0], [0, 0, 255], [0, 0, 0]], np.uint8)
    want = np.array([[100.0, 0.0, 0.0], [53.24, 80.09, 67.20], [87.73, -86.18, 83.18], [32.30, 79.19, -107.86],
                     [0.0, 0.0, 0.0]])
    np.testing.assert_allclose(ref.rgb2lab(rgb), want, atol=0.01)


def fixture_targets(z, shared=False):
    """The reference's target dicts from the fixture (similarity repeated per box, as the reference
    builds it; ``shared`` -> the zero-copy expanded form bm2f_amd.weaksup emits)."""
    out = []
    for b in range(len(z["heights"])):
        G = z[f"labels{b}"].shape[0]
        sim = torch.from_numpy(z[f"sim{b}"])
        sim = sim[None].expand(G, *sim.shape) if shared else sim[None].repeat(G, 1, 1, 1)
        out.append({"labels": torch.from_numpy(z[f"labels{b}"]), "box_masks": torch.from_numpy(z[f"box_masks{b}"]),
                    "images_color_similarity": sim})
    return out


def prepared_lab_and_masks(z, size_divisibility=32, stride=4, bottom=10):
    imgs = [torch.from_numpy(z[f"image{b}"]) for b in range(len(z["heights"]))]
    hs = max(i.shape[1] for i in imgs)
    wsz = max(i.shape[2] for i in imgs)
    Hp = (hs + size_divisibility - 1) // size_divisibility * size_divisibility
    Wp = (wsz + size_divisibility - 1) // size_divisibility * size_divisibility
    pad = torch.zeros(len(imgs), 3, Hp, Wp)
    msk = torch.zeros(len(imgs), Hp, Wp)
    for b, im in enumerate(imgs):
        pad[b, :, :im.shape[1], :im.shape[2]] = im.float()
        m = torch.ones(im.shape[1:])
        r = int(bottom * float(im.shape[1]) / float(z["heights"][b]))
        if r > 0:
            m[-r:] = 0
        msk[b, :im.shape[1], :im.shape[2]] = m
    ds = F.avg_pool2d(pad, stride, stride).byte()
    labs = [torch.as_tensor(ref.rgb2lab(ds[b].permute(1, 2, 0).numpy()), dtype=torch.float32).permute(2, 0, 1)
            for b in range(len(imgs))]
    return pad, torch.stack(labs), msk[:, stride // 2::stride, stride // 2::stride]


def test_oracle_target_prep_vs_reference(gold):
    z = gold
    pad, lab, msk = prepared_lab_and_masks(z)
    Hp, Wp = pad.shape[-2:]
    for b in range(len(z["heights"])):
        sim = ref.color_similarity(lab[b], msk[b], 2)
        np.testing.assert_allclose(sim.numpy(), z[f"sim{b}"], rtol=1e-6, atol=1e-7)
        bm, lb, rb, tb, bb = ref.box_targets(torch.from_numpy(z[f"boxes{b}"]), Hp, Wp, 4)
        for got, key in ((bm, "box_masks"), (lb, "left_bounds"), (rb, "right_bounds"), (tb, "top_bounds"),
                         (bb, "bottom_bounds")):
            assert np.array_equal(got.numpy(), z[f"{key}{b}"]), key


def _heads(z, it):
    n = int(z["n_aux"]) + 1
    return [{"pred_logits": torch.from_numpy(z[f"it{it}_logits{h}"]).requires_grad_(),
             "pred_masks": torch.from_numpy(z[f"it{it}_masks{h}"]).requires_grad_()} for h in range(n)]


def test_oracle_matcher_and_losses_vs_reference(gold):
    z = gold
    targets = fixture_targets(z)
    w_class, w_proj, w_pair = (float(v) for v in z["weights"])
    K, warmup, n_aux = int(z["K"]), int(z["warmup"]), int(z["n_aux"])
    calls = 0
    for it in range(int(z["iters"])):
        heads = _heads(z, it)
        loss_warm = min((it + 1) / warmup, 1.0)
        total = 0.0
        num_masks = float(sum(len(t["labels"]) for t in targets))
        for h in [n_aux] + list(range(n_aux)):          # the criterion's matcher call order
            calls += 1
            warm = min(calls / warmup, 1.0)
            idx = ref.match(heads[h], targets, w_class, w_proj, w_pair, 0.3, 2, warm)
            for b, (i, j) in enumerate(idx):
                assert np.array_equal(np.stack([i.numpy(), j.numpy()]), z[f"it{it}_idx{h}_{b}"]), (it, h, b)
            ls = ref.losses(heads[h], targets, idx, num_masks, K, 0.1, 0.3, 2, loss_warm)
            sfx = "" if h == n_aux else f"_{h}"
            for k, v in ls.items():
                np.testing.assert_allclose(v.item(), float(z[f"it{it}_{k}{sfx}"]), rtol=2e-6, atol=1e-7)
            total = total + w_class * ls["loss_ce"] + w_proj * ls["loss_mask_projection"] + \
                w_pair * ls["loss_pairwise"]
        total.backward()
        for h, hd in enumerate(heads):
            np.testing.assert_allclose(hd["pred_logits"].grad.numpy(), z[f"it{it}_glogits{h}"], rtol=1e-5, atol=1e-8)
            np.testing.assert_allclose(hd["pred_masks"].grad.numpy(), z[f"it{it}_gmasks{h}"], rtol=1e-4, atol=1e-9)


def test_lsap_fixture_is_scipy():
    from scipy.optimize import linear_sum_assignment
    z = np.load(os.path.join(GOLD, "lsap.npz"))
    for k in z.files:
        if k.startswith("c"):
            i, j = linear_sum_assignment(z[k])
            assert np.array_equal(np.stack([i, j]), z["r" + k[1:]])


def test_indices_from_match_host_logic():
    from bm2f_amd.weaksup import indices_from_match
    match = torch.tensor([[-1, 2, -1, 0, 1], [3, -1, -1, -1, -1], [-1] * 5, [4, 3, 2, 1, 0]], dtype=torch.int32)
    out = indices_from_match(match, [3, 1, 0, 5])
    assert [o[0].tolist() for o in out] == [[1, 3, 4], [0], [], [0, 1, 2, 3, 4]]
    assert [o[1].tolist() for o in out] == [[2, 0, 1], [3], [], [4, 3, 2, 1, 0]]


def test_criterion_requires_cuda():
    from bm2f_amd import weaksup
    with pytest.raises(RuntimeError, match="CUDA"):
        weaksup.threshold_bits(torch.zeros(1, 8, 4, 4), 0.3)
