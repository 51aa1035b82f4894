"""Box-supervised Hungarian matcher and set criterion on the GPU.

Drop-ins for the reference's ``HungarianMatcherProjPair`` (mask2former/modeling/matcher.py:213-337) and
``SetCriterionProjPair`` (mask2former/modeling/criterion.py:184-442): same constructor arguments, buffers
(``_iter``, ``empty_weight``: checkpoints load), ``forward(outputs, targets)`` contracts and loss keys
(``loss_ce``, ``loss_mask_projection``, ``loss_pairwise`` and the ``_i`` aux copies).

What changes is where the work runs.  The reference loops over images, builds each (Q, G) cost on the
device, copies it to the host and calls scipy per image per decoder head (matcher.py:309-311: 10 x batch
host round trips per step), and reads ``_iter`` / ``num_masks`` back with ``.item()``.  Here

* the three costs are computed for the whole batch at once: class cost by one gather; projection dice
  by batched GEMMs over the row / column maxima; the pairwise-affinity cost by one kernel pass over all
  B*Q masks (``m2f_pairwise_rows`` mode 0: sum_k bit_k s_k per pixel, s = -log P(same label) of the 8
  dilated neighbours, bit_k = colour similarity >= thresh) followed by a (Q x HW) x (HW x G) GEMM against
  the box masks -- exact because the reference's per-target similarity is the image's one map repeated
  G times (maskformer_model.py:498-500); a per-target similarity falls back to the general form
  s (Q, 8HW) x T (8HW, G);
* all B assignments are solved in one launch of the GPU LSAP (``m2f_lsap_batched``: scipy's algorithm
  and tie rule in fp64) and turned into index tensors without a host sync;
* the pairwise loss is one fused forward / backward kernel pair over the matched masks (no (N, 8, H, W)
  intermediates);
* ``_iter`` is mirrored on the host, ``num_masks`` stays a device scalar under torch.distributed, and
  LSAP failures (NaN / -inf / infeasible costs, which scipy raises for) are checked once per criterion call
  (``check_matching = False`` on the criterion skips that one sync).

Matched indices are returned as int64 tensors on the masks' device (the reference returns CPU tensors;
both index the same way).
"""
from __future__ import annotations


import numpy as np
import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.utils.rnn import pad_sequence

from . import weaksup as ws


def _dist_world():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_world_size()
    return 0


class _IterMirror:
    """Host copy of a float32 ``_iter`` buffer so the warm-up factor needs no ``.item()`` per call."""

    def __init__(self, module):
        self.value = None
        module._register_load_state_dict_pre_hook(self._invalidate)

    def _invalidate(self, *args, **kwargs):
        self.value = None

    def step(self, buf):
        buf += 1
        if self.value is None:
            self.value = float(buf.item())       # once after construction / load_state_dict
        else:
            self.value = float(np.float32(self.value) + np.float32(1.0))
        return self.value


def _dice_cost(src, tgt):
    """Batched batch_dice_loss (matcher.py:103-121): src (B, Q, L) logits, tgt (B, G, L)."""
    s = src.sigmoid()
    num = 2 * torch.bmm(s, tgt.transpose(1, 2))
    den = s.sum(-1)[:, :, None] + tgt.sum(-1)[:, None, :]
    return 1 - (num + 1) / (den + 1)


class WeakTargets:
    """Per-call device-side target tensors shared by the matcher and every loss of all decoder heads."""

    def __init__(self, targets, device, thresh):
        self.G = [int(t["labels"].shape[0]) for t in targets]
        self.B = len(targets)
        self.Gm = max(self.G) if self.G else 0
        self.offsets = np.concatenate([[0], np.cumsum(self.G)]).astype(np.int64).tolist()
        self.labels = [t["labels"].to(device) for t in targets]
        self.box_list = [t["box_masks"].to(device=device, dtype=torch.float32) for t in targets]
        H, W = self.box_list[0].shape[-2:] if self.box_list else (0, 0)
        self.H, self.W = int(H), int(W)
        self.box_all = torch.cat(self.box_list).contiguous() if self.box_list else None      # (T, H, W)
        sims = [t["images_color_similarity"] for t in targets]
        self.shared = all(s.shape[0] <= 1 or s.stride(0) == 0 for s in sims)
        if self.shared:
            img = [s[0] if s.shape[0] else torch.zeros(8, self.H, self.W, device=device) for s in sims]
            img = torch.stack([s.to(device=device, dtype=torch.float32) for s in img])        # (B, 8, H, W)
            self.bits = ws.threshold_bits(img, thresh)                                          # (B, H, W)
        else:
            self.sim_list = [s.to(device=device, dtype=torch.float32) for s in sims]
            sim_all = torch.cat(self.sim_list)
            self.bits = ws.threshold_bits(sim_all, thresh) if sim_all.shape[0] else None       # (T, H, W)
        self.thresh = thresh
        self.device = device
        self._padded = None
        self._match_aux = None

    def padded(self):
        if self._padded is None:
            labels = pad_sequence([l.long() for l in self.labels], batch_first=True)                # (B, Gm)
            box = pad_sequence(self.box_list, batch_first=True).contiguous()                     # (B, Gm, H, W)
            self._padded = (labels, box)
        return self._padded

    def match_aux(self):
        """Matcher-side constants of the targets: box axis projections, the pairwise normaliser
        sum_p box_g(p) popcount(bits(p)) (shared similarity) and the per-image target counts."""
        if self._match_aux is None:
            _, box = self.padded()
            B, Gm = box.shape[:2]
            aux = {"box_x": box.amax(3), "box_y": box.amax(2), "gcount": ws.h2d(self.G, self.device),
                   "extents": ws.box_extents(box)}
            if self.shared:
                k = torch.arange(8, device=box.device, dtype=torch.uint8)
                tsum = ((self.bits.view(B, -1, 1) >> k) & 1).sum(-1, dtype=torch.float32)       # (B, HW)
                aux["pair_den"] = (box.view(B, Gm, -1) * tsum[:, None]).sum(-1).clamp(min=1.0)  # (B, Gm)
            self._match_aux = aux
        return self._match_aux


class HungarianMatcherProjPair(nn.Module):
    """Reference: mask2former/modeling/matcher.py:213-337 (same arguments and ``_iter`` buffer)."""

    def __init__(self, cost_class: float = 1, cost_projection: float = 1, cost_pairwise: float = 1,
                 pairwise_size: int = 3, pairwise_dilation: int = 2, pairwise_color_thresh: float = 0.3,
                 pairwise_warmup_iters: int = 10000, point_sample: bool = False, num_points: int = 12544):
        super().__init__()
        self.cost_class = cost_class
        self.cost_projection = cost_projection
        self.cost_pairwise = cost_pairwise
        self.pairwise_size = pairwise_size
        self.pairwise_dilation = pairwise_dilation
        self.pairwise_color_thresh = pairwise_color_thresh
        self.pairwise_warmup_iters = pairwise_warmup_iters
        self.point_sample = point_sample
        self.num_points = num_points
        assert cost_class != 0 or cost_projection != 0 or cost_pairwise != 0, "all costs cant be 0"
        if pairwise_size != 3:
            raise ValueError("only pairwise_size 3 is implemented")
        self.register_buffer("_iter", torch.zeros([1]))
        self._iter_host = _IterMirror(self)
        self.last_status = None

    @torch.no_grad()
    def cost_matrix(self, outputs, tg: WeakTargets, warm: float) -> torch.Tensor:
        """(B, Q, Gm) fp32 matching cost of every image (columns >= G_b are padding)."""
        logits, masks = outputs["pred_logits"], outputs["pred_masks"]
        B, Q = logits.shape[:2]
        H, W = masks.shape[-2:]
        labels, box = tg.padded()
        aux = tg.match_aux()
        Gm = tg.Gm
        prob = logits.float().softmax(-1)
        c_class = -torch.gather(prob, 2, labels[:, None, :].expand(B, Q, Gm))
        x = masks.float().contiguous()
        pair = None
        if tg.shared:
            # one pass over the masks: pairwise numerators and both axis projections
            num, sx, sy = ws.match_cost(x, tg.bits, box, aux["gcount"], self.pairwise_dilation, aux["extents"])
            pair = num / aux["pair_den"][:, None, :]
        else:
            sx, sy = x.amax(3), x.amax(2)
        c_proj = _dice_cost(sx, aux["box_x"]) + _dice_cost(sy, aux["box_y"])
        C = self.cost_class * c_class + self.cost_projection * c_proj
        if self.cost_pairwise != 0 and warm != 0:
            if pair is None:
                pair = self._pairwise_cost_general(x, tg)
            C = C + self.cost_pairwise * (pair * warm)
        return C

    def _pairwise_cost_general(self, x, tg):
        """Per-target similarity maps: s (Q, 8HW) x T (8HW, G) per image (matcher.py:23-35, :48-83)."""
        B, Q, H, W = x.shape
        d = self.pairwise_dilation
        out = x.new_zeros((B, Q, tg.Gm))
        for b in range(B):
            G = tg.G[b]
            if G == 0:
                continue
            s = ws.pairwise_planes(x[b].contiguous(), d).view(Q, -1)                          # (Q, 8HW)
            t = ((tg.sim_list[b] >= tg.thresh).float() * tg.box_list[b][:, None]).view(G, -1)
            out[b, :, :G] = (s @ t.t()) / t.sum(1)[None].clamp(min=1.0)
        return out

    @torch.no_grad()
    def memory_efficient_forward(self, outputs, targets, prepared: WeakTargets | None = None):
        masks = outputs["pred_masks"]
        tg = prepared or WeakTargets(targets, masks.device, self.pairwise_color_thresh)
        B, Q = outputs["pred_logits"].shape[:2]
        if tg.Gm == 0:
            e = torch.empty(0, dtype=torch.int64, device=masks.device)
            return [(e, e) for _ in range(B)]
        warm = min(self._iter_host.value / float(self.pairwise_warmup_iters), 1.0)
        C = self.cost_matrix(outputs, tg, warm)
        match, status = ws.lsap_batched(C, cols=ws.h2d(tg.G, masks.device))
        self.last_status = status
        return ws.indices_from_match(match, [min(Q, g) for g in tg.G])

    @torch.no_grad()
    def forward(self, outputs, targets, prepared: WeakTargets | None = None):
        self._iter_host.step(self._iter)
        return self.memory_efficient_forward(outputs, targets, prepared)

    def __repr__(self, _repr_indent=4):
        head = "Matcher " + self.__class__.__name__
        body = [f"cost_class: {self.cost_class}", f"cost_projection: {self.cost_projection}",
                f"cost_pairwise: {self.cost_pairwise}"]
        return "\n".join([head] + [" " * _repr_indent + line for line in body])


class SetCriterionProjPair(nn.Module):
    """Reference: mask2former/modeling/criterion.py:184-442 (losses "labels", "projection_masks",
    "pairwise"; point sampling is not used by this criterion in the reference either)."""

    def __init__(self, num_classes, matcher, weight_dict, eos_coef, pairwise_size, pairwise_dilation,
                 pairwise_color_thresh, pairwise_warmup_iters, losses, point_sample, num_points, oversample_ratio,
                 importance_sample_ratio):
        super().__init__()
        self.num_classes = num_classes
        self.matcher = matcher
        self.weight_dict = weight_dict
        self.eos_coef = eos_coef
        self.pairwise_size = pairwise_size
        self.pairwise_dilation = pairwise_dilation
        self.pairwise_color_thresh = pairwise_color_thresh
        self.pairwise_warmup_iters = pairwise_warmup_iters
        self.losses = losses
        self.point_sample = point_sample
        if point_sample:
            self.num_points = num_points
            self.oversample_ratio = oversample_ratio
            self.importance_sample_ratio = importance_sample_ratio
        if pairwise_size != 3:
            raise ValueError("only pairwise_size 3 is implemented")
        empty_weight = torch.ones(self.num_classes + 1)
        empty_weight[-1] = self.eos_coef
        self.register_buffer("empty_weight", empty_weight)
        self.register_buffer("_iter", torch.zeros([1]))
        self._iter_host = _IterMirror(self)
        self.check_matching = True   # one host sync per call for scipy's ValueErrors; False skips it
        self._tg = self._tg_key = None
        self._status = []
        self._gathered = {}

    # -- losses --------------------------------------------------------------------------------------
    def loss_labels(self, outputs, targets, indices, num_masks):
        src_logits = outputs["pred_logits"].float()
        idx = self._get_src_permutation_idx(indices)
        target_classes_o = torch.cat([t["labels"].to(src_logits.device)[J] for t, (_, J) in zip(targets, indices)])
        target_classes = torch.full(src_logits.shape[:2], self.num_classes, dtype=torch.int64,
                                    device=src_logits.device)
        target_classes[idx] = target_classes_o
        return {"loss_ce": F.cross_entropy(src_logits.transpose(1, 2), target_classes, self.empty_weight)}

    def _matched(self, outputs, targets, indices):
        """Matched masks (N, H, W) and flat target rows, gathered once per head for both mask losses
        (one IndexBackward, so one full-size gradient buffer per head)."""
        tg = self._targets(targets, outputs["pred_masks"].device)
        key = (id(outputs["pred_masks"]), id(indices))
        hit = self._gathered.get(key)
        if hit is not None and hit[0] is outputs["pred_masks"] and hit[1] is indices:
            return tg, hit[2], hit[3]
        src = outputs["pred_masks"][self._get_src_permutation_idx(indices)].float().contiguous()   # (N, H, W)
        flat = torch.cat([j + tg.offsets[b] for b, (_, j) in enumerate(indices)])                # target rows
        self._gathered[key] = (outputs["pred_masks"], indices, src, flat)
        return tg, src, flat

    def loss_projection_masks(self, outputs, targets, indices, num_masks):
        tg, src, flat = self._matched(outputs, targets, indices)
        box = tg.box_all[flat]
        x = src.max(dim=2)[0].sigmoid()          # projection on the H axis (max over W), criterion.py:353
        y = src.max(dim=1)[0].sigmoid()
        with torch.no_grad():
            bx = box.max(dim=2)[0]
            by = box.max(dim=1)[0]

        def dice(p, t):
            inter = (p * t).sum(dim=1)
            union = (p ** 2.0).sum(dim=1) + (t ** 2.0).sum(dim=1) + 1e-3
            return 1. - (2 * inter / union)

        return {"loss_mask_projection": (dice(x, bx) + dice(y, by)).sum() / num_masks}

    def loss_pairwise(self, outputs, targets, indices, num_masks):
        tg, src, flat = self._matched(outputs, targets, indices)
        box_row = flat.to(torch.int32)
        if tg.shared:
            t_row = self._get_src_permutation_idx(indices)[0].to(torch.int32)
        else:
            t_row = box_row
        bits = tg.bits if tg.bits is not None else torch.zeros((1, tg.H, tg.W), dtype=torch.uint8,
                                                                 device=src.device)
        num, den = ws.pairwise_sums(src, bits, t_row.contiguous(), tg.box_all, box_row.contiguous(),
                                    self.pairwise_dilation)
        warm = min(self._iter_host.value / float(self.pairwise_warmup_iters), 1.0)
        return {"loss_pairwise": num.sum() / den.sum().clamp(min=1.0) / num_masks * warm}

    def _get_src_permutation_idx(self, indices):
        batch_idx = torch.cat([torch.full_like(src, i) for i, (src, _) in enumerate(indices)])
        src_idx = torch.cat([src for (src, _) in indices])
        return batch_idx, src_idx

    def _get_tgt_permutation_idx(self, indices):
        batch_idx = torch.cat([torch.full_like(tgt, i) for i, (_, tgt) in enumerate(indices)])
        tgt_idx = torch.cat([tgt for (_, tgt) in indices])
        return batch_idx, tgt_idx

    def get_loss(self, loss, outputs, targets, indices, num_masks):
        loss_map = {"labels": self.loss_labels, "projection_masks": self.loss_projection_masks,
                    "pairwise": self.loss_pairwise}
        assert loss in loss_map, f"do you really want to compute {loss} loss?"
        return loss_map[loss](outputs, targets, indices, num_masks)

    # -- driver --------------------------------------------------------------------------------------
    def _targets(self, targets, device):
        # built once per forward() for all heads; a direct get_loss() call outside forward builds its own
        if self._tg is None or self._tg_key is not targets:
            self._tg = WeakTargets(targets, device, self.pairwise_color_thresh)
            self._tg_key = targets
        return self._tg

    def _match(self, outputs, targets):
        if isinstance(self.matcher, HungarianMatcherProjPair):
            idx = self.matcher(outputs, targets, prepared=self._targets(targets, outputs["pred_masks"].device))
            if self.matcher.last_status is not None:
                self._status.append(self.matcher.last_status)
            return idx
        return self.matcher(outputs, targets)

    def forward(self, outputs, targets):
        self._iter_host.step(self._iter)
        self._tg = self._tg_key = None
        self._status = []
        self._gathered = {}
        try:
            outputs_without_aux = {k: v for k, v in outputs.items() if k != "aux_outputs"}
            indices = self._match(outputs_without_aux, targets)
            dev = next(iter(outputs.values())).device
            n = sum(len(t["labels"]) for t in targets)
            world = _dist_world()
            if world:
                nm = torch.as_tensor([n], dtype=torch.float, device=dev)
                torch.distributed.all_reduce(nm)
                num_masks = torch.clamp(nm / world, min=1)[0]      # stays on the device (no .item())
            else:
                num_masks = max(float(np.float32(n)), 1.0)
            losses = {}
            for loss in self.losses:
                losses.update(self.get_loss(loss, outputs, targets, indices, num_masks))
            for i, aux_outputs in enumerate(outputs.get("aux_outputs", [])):
                indices = self._match(aux_outputs, targets)
                for loss in self.losses:
                    l_dict = self.get_loss(loss, aux_outputs, targets, indices, num_masks)
                    losses.update({k + f"_{i}": v for k, v in l_dict.items()})
            if self.check_matching and self._status:
                ws.raise_on_lsap_status(torch.stack(self._status))
            return losses
        finally:
            self._tg = self._tg_key = None
            self._status = []
            self._gathered = {}

    def __repr__(self):
        head = "Criterion " + self.__class__.__name__
        body = [f"matcher: {self.matcher.__repr__(_repr_indent=8)}", f"losses: {self.losses}",
                f"weight_dict: {self.weight_dict}", f"num_classes: {self.num_classes}", f"eos_coef: {self.eos_coef}"]
        return "\n".join([head] + [" " * 4 + line for line in body])
