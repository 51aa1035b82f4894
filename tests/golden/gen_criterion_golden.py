"""Generate tests/golden/criterion.npz and lsap.npz by running the REFERENCE weak-supervision code in
this container (never on the GPU box; nothing under /root/reference is copied).

    python tests/golden/gen_criterion_golden.py [--ref /root/reference]

Imported in place, with test-only stand-ins for absent third-party packages (gen_golden.install_stubs
plus cv2, torchvision._is_tracing, detectron2 comm/point_features/structures/data/modeling bits, and
``skimage.color`` whose ``rgb2lab`` is oracle/weaksup_ref.rgb2lab -- skimage is not installed, so the
Lab conversion itself is the one unpinned piece):
  * MaskFormer.prepare_weaksup_targets (maskformer_model.py:399-507) called unbound on uint8 images and
    boxes -> box_masks, colour similarities, projection bounds;
  * HungarianMatcherProjPair (matcher.py:213-337) and SetCriterionProjPair (criterion.py:184-429) with
    3 decoder heads (2 aux), run for several iterations (pairwise warm-up 3 iters) -> matched indices per
    head, every loss, and the gradients of the weighted loss sum w.r.t. pred_logits / pred_masks;
  * scipy.optimize.linear_sum_assignment (the reference's LSAP, matcher.py:311) on random, integer-valued
    (tie-heavy) and rectangular cost matrices -> lsap.npz.
"""
from __future__ import annotations

import argparse
import importlib
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from gen_golden import install_stubs  # noqa: E402
from oracle.weaksup_ref import rgb2lab  # noqa: E402


def install_weaksup_stubs():
    install_stubs()
    mods = {}
    for name in ["cv2", "torchvision", "torchvision.ops", "torchvision.ops.boxes", "detectron2.utils.comm",
                 "detectron2.projects", "detectron2.projects.point_rend",
                 "detectron2.projects.point_rend.point_features", "detectron2.structures",
                 "detectron2.structures.masks", "detectron2.data", "detectron2.modeling.backbone",
                 "detectron2.modeling.postprocessing", "detectron2.utils.memory", "skimage", "skimage.color"]:
        mods[name] = types.ModuleType(name)

    def unavailable(*a, **k):
        raise RuntimeError("stand-in: not used by the weak-supervision path")

    class ImageList:
        def __init__(self, tensor):
            self.tensor = tensor

        @staticmethod
        def from_tensors(tensors, size_divisibility=0, pad_value=0.0):
            # detectron2 ImageList.from_tensors: pad every image bottom/right to the max size rounded up to
            # size_divisibility, stack
            hs = max(t.shape[-2] for t in tensors)
            ws = max(t.shape[-1] for t in tensors)
            if size_divisibility > 1:
                s = size_divisibility
                hs, ws = (hs + s - 1) // s * s, (ws + s - 1) // s * s
            out = tensors[0].new_full((len(tensors),) + tuple(tensors[0].shape[:-2]) + (hs, ws), pad_value)
            for i, t in enumerate(tensors):
                out[i, ..., :t.shape[-2], :t.shape[-1]].copy_(t)
            return ImageList(out)

    mods["torchvision"]._is_tracing = lambda: False
    mods["torchvision"].ops = mods["torchvision.ops"]
    mods["torchvision.ops"].boxes = mods["torchvision.ops.boxes"]
    mods["torchvision.ops.boxes"].box_area = unavailable
    mods["detectron2.utils.comm"].get_world_size = lambda: 1
    pf = mods["detectron2.projects.point_rend.point_features"]
    pf.point_sample = unavailable
    pf.get_uncertain_point_coords_with_randomness = unavailable
    for n in ("Boxes", "Instances", "BitMasks"):
        setattr(mods["detectron2.structures"], n, type(n, (), {}))
    mods["detectron2.structures"].ImageList = ImageList
    mods["detectron2.structures.masks"].BitMasks = mods["detectron2.structures"].BitMasks
    mods["detectron2.data"].MetadataCatalog = types.SimpleNamespace(get=unavailable)
    d2m = sys.modules["detectron2.modeling"]
    d2m.META_ARCH_REGISTRY = d2m.SEM_SEG_HEADS_REGISTRY
    d2m.build_backbone = unavailable
    d2m.build_sem_seg_head = unavailable
    mods["detectron2.modeling.backbone"].Backbone = torch.nn.Module
    mods["detectron2.modeling.postprocessing"].sem_seg_postprocess = unavailable
    mods["detectron2.utils.memory"].retry_if_cuda_oom = lambda f: f
    sys.modules["detectron2.layers"].cat = torch.cat
    mods["skimage.color"].rgb2lab = rgb2lab
    mods["skimage"].color = mods["skimage.color"]
    sys.modules.update(mods)


def import_reference(ref_root):
    install_weaksup_stubs()
    sys.path.insert(0, ref_root)
    for pkg in ("mask2former", "mask2former.modeling", "mask2former.utils"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(ref_root, *pkg.split("."))]
        sys.modules[pkg] = m
    return types.SimpleNamespace(
        matcher=importlib.import_module("mask2former.modeling.matcher"),
        criterion=importlib.import_module("mask2former.modeling.criterion"),
        model=importlib.import_module("mask2former.maskformer_model"),
        wsu=importlib.import_module("mask2former.utils.weaksup_utils"))


class _Boxes:
    def __init__(self, t):
        self.tensor = t


class _Inst:
    def __init__(self, boxes, classes):
        self.gt_boxes = _Boxes(boxes)
        self.gt_classes = classes

    def __len__(self):
        return self.gt_classes.shape[0]


# image sizes (unpadded) and box counts (the reference cannot prepare an image without boxes:
# torch.cat of an empty list, maskformer_model.py:498); padding to /32 makes 128 x 128
SIZES = [(128, 120), (100, 128), (112, 96)]
COUNTS = [3, 1, 5]
HEIGHTS = [256, 200, 224]   # "height" of the original annotation (bottom-pixel removal scales with it)
Q, K = 20, 6                # queries, classes (K+1 logits)
N_AUX = 2
ITERS = 4
WARMUP = 3
WEIGHTS = {"loss_ce": 2.0, "loss_mask_projection": 5.0, "loss_pairwise": 5.0}


def make_inputs(gen):
    images, insts = [], []
    for (h, w), g in zip(SIZES, COUNTS):
        # smooth-ish colour field + noise so that some neighbour similarities pass the 0.3 threshold
        yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
        base = torch.stack([(xx * 2) % 256, (yy * 2) % 256, ((xx + yy) * 1) % 256]).float()
        blocks = (torch.rand(3, h // 16 + 1, w // 16 + 1, generator=gen) * 255).repeat_interleave(16, 1) \
            .repeat_interleave(16, 2)[:, :h, :w]
        region = (torch.rand(1, h // 32 + 1, w // 32 + 1, generator=gen) < 0.5).repeat_interleave(32, 1) \
            .repeat_interleave(32, 2)[:, :h, :w]
        img = torch.where(region, base * 0.25, blocks)
        img = (img + torch.randint(-3, 4, (3, h, w), generator=gen)).clamp(0, 255).to(torch.uint8)
        images.append(img)
        x0 = torch.randint(0, w - 8, (g,), generator=gen).float() + torch.rand(g, generator=gen)
        y0 = torch.randint(0, h - 8, (g,), generator=gen).float() + torch.rand(g, generator=gen)
        x1 = torch.minimum(x0 + 4 + torch.rand(g, generator=gen) * 60, torch.tensor(float(w - 1)))
        y1 = torch.minimum(y0 + 4 + torch.rand(g, generator=gen) * 60, torch.tensor(float(h - 1)))
        insts.append(_Inst(torch.stack([x0, y0, x1, y1], 1), torch.randint(0, K, (g,), generator=gen)))
    return images, insts


def gen_criterion(ref, out):
    gen = torch.Generator().manual_seed(123)
    images, insts = make_inputs(gen)
    fake = types.SimpleNamespace(bottom_pixels_removed=10, size_divisibility=32, mask_out_stride=4,
                                 pairwise_size=3, pairwise_dilation=2, device=torch.device("cpu"))
    targets = ref.model.MaskFormer.prepare_weaksup_targets(fake, insts, images, HEIGHTS)
    res = {"Q": Q, "K": K, "n_aux": N_AUX, "iters": ITERS, "warmup": WARMUP, "heights": np.array(HEIGHTS),
           "weights": np.array([WEIGHTS[k] for k in ("loss_ce", "loss_mask_projection", "loss_pairwise")])}
    for b, (img, inst, t) in enumerate(zip(images, insts, targets)):
        res[f"image{b}"] = img.numpy()
        res[f"boxes{b}"] = inst.gt_boxes.tensor.numpy()
        res[f"labels{b}"] = inst.gt_classes.numpy()
        res[f"box_masks{b}"] = t["box_masks"].numpy()
        for k in ("left_bounds", "right_bounds", "top_bounds", "bottom_bounds"):
            res[f"{k}{b}"] = t[k].numpy()
        sim = t["images_color_similarity"]
        if sim.shape[0]:
            assert all(torch.equal(sim[0], s) for s in sim)
            res[f"sim{b}"] = sim[0].numpy()
    h, w = targets[0]["box_masks"].shape[-2:]
    matcher = ref.matcher.HungarianMatcherProjPair(
        cost_class=WEIGHTS["loss_ce"], cost_projection=WEIGHTS["loss_mask_projection"],
        cost_pairwise=WEIGHTS["loss_pairwise"], pairwise_size=3, pairwise_dilation=2, pairwise_color_thresh=0.3,
        pairwise_warmup_iters=WARMUP)
    crit = ref.criterion.SetCriterionProjPair(
        K, matcher=matcher, weight_dict=WEIGHTS, eos_coef=0.1, pairwise_size=3, pairwise_dilation=2,
        pairwise_color_thresh=0.3, pairwise_warmup_iters=WARMUP, losses=["labels", "projection_masks", "pairwise"],
        point_sample=False, num_points=0, oversample_ratio=3.0, importance_sample_ratio=0.75)
    B = len(images)
    idx_calls = []
    orig = matcher.memory_efficient_forward

    def spy(outputs, tg):
        r = orig(outputs, tg)
        idx_calls.append(r)
        return r

    matcher.memory_efficient_forward = spy
    for it in range(ITERS):
        heads = []
        for hd in range(N_AUX + 1):
            lg = (torch.randn(B, Q, K + 1, generator=gen) * 2).requires_grad_()
            # masks: a blend of box-like blobs and noise so matching is informative but not trivial
            mk = (torch.randn(B, Q, h, w, generator=gen) * 3).requires_grad_()
            heads.append({"pred_logits": lg, "pred_masks": mk})
        outputs = dict(heads[-1])
        outputs["aux_outputs"] = heads[:-1]
        idx_calls.clear()
        losses = crit(outputs, targets)
        total = sum(losses[k] * WEIGHTS[k.rsplit("_", 1)[0] if k[-1].isdigit() else k] for k in losses)
        total.backward()
        for hd, hdict in enumerate(heads):
            res[f"it{it}_logits{hd}"] = hdict["pred_logits"].detach().numpy()
            res[f"it{it}_masks{hd}"] = hdict["pred_masks"].detach().numpy()
            res[f"it{it}_glogits{hd}"] = hdict["pred_logits"].grad.numpy()
            res[f"it{it}_gmasks{hd}"] = hdict["pred_masks"].grad.numpy()
        # matcher call order: final head first, then aux 0..n-1 (criterion.py:406, :420-421)
        order = [N_AUX] + list(range(N_AUX))
        for call, hd in enumerate(order):
            for b, (i, j) in enumerate(idx_calls[call]):
                res[f"it{it}_idx{hd}_{b}"] = np.stack([i.numpy(), j.numpy()]).astype(np.int64)
        for k, v in losses.items():
            res[f"it{it}_{k}"] = np.float64(v.item())
    res["loss_keys"] = np.array(sorted(losses.keys()))
    np.savez_compressed(os.path.join(out, "criterion.npz"), **res)


def gen_lsap(out):
    from scipy.optimize import linear_sum_assignment
    gen = np.random.default_rng(7)
    res = {}
    cases = []
    for shape in [(1, 1), (5, 5), (20, 3), (3, 20), (100, 15), (100, 100), (64, 64), (200, 7), (7, 200),
                  (1000, 50), (37, 128)]:
        cases.append(("rand", gen.standard_normal(shape).astype(np.float32)))
    for shape in [(10, 10), (30, 6), (6, 30), (100, 20), (50, 50)]:
        cases.append(("int", gen.integers(0, 4, shape).astype(np.float32)))
    cases.append(("const", np.ones((12, 5), np.float32)))
    cases.append(("inf", np.where(gen.random((16, 6)) < 0.3, np.inf, gen.random((16, 6))).astype(np.float32)))
    for n, (kind, c) in enumerate(cases):
        i, j = linear_sum_assignment(c)
        res[f"c{n}_{kind}"] = c
        res[f"r{n}_{kind}"] = np.stack([i, j]).astype(np.int64)
    np.savez_compressed(os.path.join(out, "lsap.npz"), **res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    a = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref = import_reference(a.ref)
    gen_criterion(ref, a.out)
    print("wrote criterion.npz")
    gen_lsap(a.out)
    print("wrote lsap.npz")


if __name__ == "__main__":
    main()
