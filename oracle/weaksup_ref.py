"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's box-supervised (weak-supervision)
criterion, matcher and target preparation (SUP_TYPE "mask_projection_and_pairwise").

Checker for bm2f_amd/criterion.py and bm2f_amd/weaksup.py in tests/ and for the golden generator's
skimage stand-in; never imported by the product path.  Pinned by tests/golden/criterion.npz, which the
reference itself produced in this container (tests/golden/gen_criterion_golden.py).

Restated (per image, plain torch on CPU, scipy for the assignment exactly as the reference calls it):
* matcher costs        mask2former/modeling/matcher.py:23-35 (pairwise cost), :42-46 (axis projection),
                       :48-83 (similarity cost), :103-121 (dice), :259-313 (HungarianMatcherProjPair)
* losses               mask2former/modeling/criterion.py:25-77 (pairwise / projection dice), :156-181
                       (predicted similarities), :239-369 (SetCriterionProjPair.loss_*), :392-429 (forward)
* target preparation   mask2former/maskformer_model.py:399-507, weaksup_utils.py:7-57
* rgb2lab              scikit-image's ``skimage.color.rgb2lab`` (the reference's ``from skimage import
                       color``, requirements.txt:7, version unpinned there; not installed here), restated
                       from its published algorithm: img_as_float, sRGB companding, xyz_from_rgb, D65/2deg
                       white (0.95047, 1, 1.08883), CIE f(t).  Parity vs skimage itself is UNPINNED (no
                       skimage here); it is checked against published Lab values of the sRGB primaries.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from scipy.optimize import linear_sum_assignment

_XYZ_FROM_RGB = np.array([[0.412453, 0.357580, 0.180423],
                          [0.212671, 0.715160, 0.072169],
                          [0.019334, 0.119193, 0.950227]])
_D65 = np.array([0.95047, 1.0, 1.08883])


def rgb2lab(img_u8: np.ndarray) -> np.ndarray:
    """(..., 3) uint8 sRGB -> (..., 3) float64 CIE Lab (skimage.color.rgb2lab semantics)."""
    a = img_u8.astype(np.float64) / 255.0
    a = np.where(a > 0.04045, ((a + 0.055) / 1.055) ** 2.4, a / 12.92)
    xyz = a @ _XYZ_FROM_RGB.T
    t = xyz / _D65
    f = np.where(t > 0.008856, np.cbrt(t), 7.787 * t + 16.0 / 116.0)
    L = 116.0 * f[..., 1] - 16.0
    A = 500.0 * (f[..., 0] - f[..., 1])
    B = 200.0 * (f[..., 1] - f[..., 2])
    return np.stack([L, A, B], -1)


def neighbours(x: torch.Tensor, dilation: int) -> torch.Tensor:
    """(N, C, H, W) -> (N, C, 8, H, W): the 3x3 dilated taps minus the centre, zero outside (unfold)."""
    N, C, H, W = x.shape
    d = dilation
    xp = F.pad(x, (d, d, d, d))
    taps = []
    for ky in range(3):
        for kx in range(3):
            if ky == 1 and kx == 1:
                continue
            taps.append(xp[:, :, ky * d:ky * d + H, kx * d:kx * d + W])
    return torch.stack(taps, 2)


def pred_similarity(logits: torch.Tensor, dilation: int) -> torch.Tensor:
    """(N, H, W) mask logits -> (N, 8, H, W) -log P(same label) for each neighbour pair."""
    lf = F.logsigmoid(logits)[:, None]
    lb = F.logsigmoid(-logits)[:, None]
    u = lf[:, :, None] + neighbours(lf, dilation)
    v = lb[:, :, None] + neighbours(lb, dilation)
    m = torch.maximum(u, v)
    return -(torch.log(torch.exp(u - m) + torch.exp(v - m)) + m)[:, 0]


def color_similarity(lab: torch.Tensor, mask: torch.Tensor, dilation: int) -> torch.Tensor:
    """lab (3, h, w), mask (h, w) -> (8, h, w) exp(-||lab_p - lab_q|| / 2) * mask_q."""
    nb = neighbours(lab[None], dilation)[0]                       # (3, 8, h, w)
    diff = lab[:, None] - nb
    sim = torch.exp(-torch.norm(diff, dim=0) * 0.5)
    w = neighbours(mask[None, None], dilation)[0, 0]
    return sim * w


def _dice_cost(src, tgt):
    s = src.sigmoid()
    num = 2 * s @ tgt.t()
    den = s.sum(-1)[:, None] + tgt.sum(-1)[None, :]
    return 1 - (num + 1) / (den + 1)


def match_costs(logits, masks, labels, box, sim, w_class, w_proj, w_pair, thr, dilation, warm):
    """One image: logits (Q, K+1), masks (Q, H, W), labels (G,), box (G, H, W), sim (G, 8, H, W)."""
    prob = logits.softmax(-1)
    c_class = -prob[:, labels]
    c_proj = _dice_cost(masks.amax(2), box.amax(2)) + _dice_cost(masks.amax(1), box.amax(1))
    t = (sim >= thr).float() * box[:, None]
    s = pred_similarity(masks, dilation)
    c_pair = (s.flatten(1) @ t.flatten(1).t()) / t.flatten(1).sum(1)[None].clamp(min=1.0)
    return w_class * c_class + w_proj * c_proj + w_pair * (c_pair * warm)


def match(outputs, targets, w_class, w_proj, w_pair, thr, dilation, warm):
    """-> list of (query idx, target idx) int64 tensors, sorted by query (scipy's order)."""
    out = []
    for b, t in enumerate(targets):
        C = match_costs(outputs["pred_logits"][b].float(), outputs["pred_masks"][b].float(), t["labels"],
                        t["box_masks"].float(), t["images_color_similarity"].float(), w_class, w_proj, w_pair,
                        thr, dilation, warm)
        i, j = linear_sum_assignment(C.detach().cpu().numpy())
        out.append((torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)))
    return out


def losses(outputs, targets, indices, num_masks, num_classes, eos_coef, thr, dilation, warm):
    """loss_ce, loss_mask_projection, loss_pairwise of one decoder head, differentiable w.r.t. outputs."""
    logits = outputs["pred_logits"].float()
    B, Q = logits.shape[:2]
    bi = torch.cat([torch.full_like(s, b) for b, (s, _) in enumerate(indices)])
    si = torch.cat([s for s, _ in indices])
    cls = torch.full((B, Q), num_classes, dtype=torch.int64)
    cls[bi, si] = torch.cat([t["labels"][j] for t, (_, j) in zip(targets, indices)])
    wt = torch.ones(num_classes + 1)
    wt[-1] = eos_coef
    l_ce = F.cross_entropy(logits.transpose(1, 2), cls, wt)

    src = outputs["pred_masks"][bi, si].float()                    # (N, H, W)
    box = torch.cat([t["box_masks"][j] for t, (_, j) in zip(targets, indices)]).float()
    sim = torch.cat([t["images_color_similarity"][j] for t, (_, j) in zip(targets, indices)]).float()

    def proj_dice(x, y):
        x = x.sigmoid()
        return 1.0 - 2 * (x * y).sum(1) / ((x ** 2.0).sum(1) + (y ** 2.0).sum(1) + 1e-3)

    l_proj = (proj_dice(src.amax(2), box.amax(2)) + proj_dice(src.amax(1), box.amax(1))).sum() / num_masks
    t = (sim >= thr).float() * box[:, None]
    s = pred_similarity(src, dilation)
    l_pair = (s * t).sum() / t.sum().clamp(min=1.0) / num_masks * warm
    return {"loss_ce": l_ce, "loss_mask_projection": l_proj, "loss_pairwise": l_pair}


def box_targets(boxes: torch.Tensor, h_pad: int, w_pad: int, stride: int):
    """Full-resolution box rasters sampled at the stride grid plus the projection bounds
    (maskformer_model.py:451-491); boxes (G, 4) x0, y0, x1, y1 in pixels."""
    G = boxes.shape[0]
    start = stride // 2
    full = torch.zeros(G, h_pad, w_pad)
    lb = torch.zeros(G, h_pad)
    rb = torch.zeros(G, h_pad)
    tb = torch.zeros(G, w_pad)
    bb = torch.zeros(G, w_pad)
    for g in range(G):
        x0, y0, x1, y1 = (int(v) for v in boxes[g].tolist())
        full[g, y0:y1 + 1, x0:x1 + 1] = 1.0
        m = full[g].int()
        lb[g] = torch.argmax(m, 1)
        rb[g] = w_pad - torch.argmax(m.flip(1), 1)
        tb[g] = torch.argmax(m, 0)
        bb[g] = h_pad - torch.argmax(m.flip(0), 0)
    return (full[:, start::stride, start::stride], lb[:, start::stride] / stride, rb[:, start::stride] / stride,
            tb[:, start::stride] / stride, bb[:, start::stride] / stride)
