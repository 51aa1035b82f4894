"""The training step the benchmark times: R50 backbone -> MSDeformAttn pixel decoder -> masked decoder.

Mirrors the reference's training forward (maskformer_model.py:258-320, mask_former_head.py:115-132)
with the criterion replaced by the sum of means of every head's outputs (the
Hungarian matcher / weak-supervision losses are outside the hot path).  The backbone is
detectron2's R50 as configured by the reference (Base-COCO-*.yaml: depth 50, STRIDE_IN_1X1 False,
FrozenBN, FREEZE_AT 0, res2..res5), written here in plain PyTorch (MIOpen convs) since detectron2 / torchvision
are absent.  It runs NCHW or channels-last (``ResNet50(channels_last=True)``: MIOpen's NHWC kernels, no layout
transposes); bench.py picks channels-last under fp16 autocast, whose NHWC kernels the shipped MIOpen find-db covers
(without find-db entries MIOpen's FAST find mode picks NHWC kernels ~10x slower, so NCHW elsewhere).  FrozenBN is
folded into the conv weights on the fly (same function, one op fewer per conv).  Optimizer: AdamW + full-model grad-norm clipping
(train_net.py:185-263, SOLVER: BASE_LR 1e-4, WEIGHT_DECAY 0.05, CLIP_VALUE 0.01).
"""
from __future__ import annotations

import ctypes
import os
import types

import torch
import torch.nn.functional as F
from torch import nn

from .pixel_decoder import MSDeformAttnPixelDecoder
from .registry import ShapeSpec
from .transformer_decoder import MultiScaleMaskedTransformerDecoder

PIXEL_MEAN = (123.675, 116.280, 103.530)
PIXEL_STD = (58.395, 57.120, 57.375)
_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}   # M2F_F32 / M2F_F16 / M2F_BF16


class FrozenBNConv(nn.Module):
    """conv (no bias) + FrozenBatchNorm2d: the BN scale is folded into the conv weights on the fly, the BN
    shift is returned for the fused bias(+shortcut)+ReLU that follows (:func:`bias_act`)."""

    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride=stride, padding=padding, bias=False)
        nn.init.kaiming_normal_(self.conv.weight, mode="fan_out", nonlinearity="relu")
        self.register_buffer("weight", torch.ones(cout))
        self.register_buffer("bias", torch.zeros(cout))
        self.register_buffer("running_mean", torch.zeros(cout))
        self.register_buffer("running_var", torch.ones(cout))
        self.eps = 1e-5

    def _consts(self):
        """(scale, shift) of the frozen BN, fp32; computed once per device (the buffers never change)."""
        c = getattr(self, "_bn_consts", None)
        if c is None or c[0].device != self.weight.device:
            scale = self.weight * (self.running_var + self.eps).rsqrt()
            c = (scale.contiguous(), (self.bias - self.running_mean * scale).contiguous())
            self._bn_consts = c
        return c

    def conv_shift(self, x):
        """(conv(x) with the BN scale folded into the weights, per-channel BN shift)."""
        scale, shift = self._consts()
        # a channels-last input gets a channels-last weight copy: MIOpen then runs its NHWC kernels on the tensors
        # as they are, with no NCHW <-> NHWC transposes around each convolution
        cl = x.dim() == 4 and x.shape[1] > 1 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)
        w = _ScaledWeight.apply(self.conv.weight, scale, x.dtype,
                                torch.channels_last if cl else torch.contiguous_format)
        return F.conv2d(x, w, None, self.conv.stride, self.conv.padding), shift

    def forward(self, x):
        y, shift = self.conv_shift(x)
        return y + shift.view(1, -1, 1, 1).to(y.dtype)


class _ScaledWeight(torch.autograd.Function):
    """w * scale[co] in the conv's input dtype in one pass (autocast would multiply, then cast), and the
    weight gradient back in fp32 in one pass."""

    @staticmethod
    def forward(ctx, w, scale, dtype, fmt=torch.contiguous_format):
        out = torch.empty(w.shape, dtype=dtype, device=w.device, memory_format=fmt)
        torch.mul(w, scale.view(-1, 1, 1, 1), out=out)
        ctx.save_for_backward(scale)
        return out

    @staticmethod
    def backward(ctx, grad):
        (scale,) = ctx.saved_tensors
        gw = torch.empty(grad.shape, dtype=torch.float32, device=grad.device)   # the parameter's own layout
        torch.mul(grad, scale.view(-1, 1, 1, 1), out=gw)
        return gw, None, None, None


class _BiasAct(torch.autograd.Function):
    """y = relu(x + r + bias[c]) in place on x (bias: frozen BN shift, no gradient).

    ``nout`` > 1 returns y plus nout - 1 aliases of it, one per consumer (a block output feeds the next
    block's first conv, its shortcut / identity path and, at a stage end, the pixel decoder): the backward
    then receives each consumer's gradient separately and forms sum * (y > 0) in one pass
    (m2f_relu_bwd_sum) instead of the engine's accumulating adds followed by threshold_backward."""

    @staticmethod
    def forward(ctx, x, r, bias, nout):
        from . import _native
        code = _CODE[x.dtype]
        cl = 0 if x.is_contiguous() else 1
        _native.call("m2f_bias_act_nchw", x.data_ptr(), r.data_ptr() if r is not None else None,
                     bias.data_ptr(), x.shape[0], x.shape[1], x.shape[2] * x.shape[3], code, cl,
                     torch.cuda.current_stream(x.device).cuda_stream)
        ctx.mark_dirty(x)
        ctx.save_for_backward(x)
        ctx.has_r = r is not None
        if nout == 1:
            return x
        return (x,) + tuple(x.view(x.shape) for _ in range(nout - 1))

    @staticmethod
    def backward(ctx, *grads):
        from . import _native
        (y,) = ctx.saved_tensors
        gs = [g for g in grads if g is not None]
        if len(gs) == 1:
            g = torch.ops.aten.threshold_backward(gs[0], y, 0)  # ReLU's own backward: one pass
        elif (len(gs) <= 4 and y.numel() % 8 == 0 and y.data_ptr() % 16 == 0 and _dense(y)
              and all(t.dtype == y.dtype and t.stride() == y.stride() and t.data_ptr() % 16 == 0 for t in gs)):
            g = torch.empty_like(y, memory_format=torch.preserve_format)   # elementwise: any dense layout
            ptrs = (ctypes.c_void_p * len(gs))(*[t.data_ptr() for t in gs])
            _native.call("m2f_relu_bwd_sum", ptrs, len(gs), y.data_ptr(), g.data_ptr(), y.numel(),
                         _CODE[y.dtype], torch.cuda.current_stream(y.device).cuda_stream)
        else:
            g = torch.ops.aten.threshold_backward(sum(gs), y, 0)
        return g, (g if ctx.has_r else None), None, None


def _dense(t):
    return t.is_contiguous() or t.is_contiguous(memory_format=torch.channels_last)


def bias_act(x, bias, residual=None, nout=1):
    """relu(x + residual + bias[c]) (NCHW); one fused pass on a HIP device.  nout > 1: a tuple of nout
    handles of the result, one per consumer (see _BiasAct)."""
    hw = x.shape[2] * x.shape[3]
    cl = torch.channels_last
    ok = ((x.is_contiguous() and hw % 8 == 0 and (residual is None or residual.is_contiguous()))
          or (x.is_contiguous(memory_format=cl) and x.shape[1] % 8 == 0
              and (residual is None or residual.is_contiguous(memory_format=cl))))
    if (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and ok
            and (residual is None or residual.dtype == x.dtype)):
        return _BiasAct.apply(x, residual, bias.float().contiguous(), nout)
    y = x + bias.view(1, -1, 1, 1).to(x.dtype)
    if residual is not None:
        y = y + residual
    y = F.relu(y)
    return y if nout == 1 else (y,) * nout


class _MaxPool3s2(torch.autograd.Function):
    """``F.max_pool2d(x, 3, 2, 1)`` (NCHW) with a 1-byte winner position per window (csrc/eltwise.hip)."""

    @staticmethod
    def forward(ctx, x):
        from . import _native
        N, C, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty(N, C, OH, OW, device=x.device, dtype=x.dtype)
        win = torch.empty(N, C, OH, OW, device=x.device, dtype=torch.uint8)
        _native.call("m2f_maxpool3s2_fwd", x.data_ptr(), y.data_ptr(), win.data_ptr(), N * C, H, W,
                     _CODE[x.dtype], torch.cuda.current_stream(x.device).cuda_stream)
        ctx.save_for_backward(win)
        ctx.in_shape = x.shape
        return y

    @staticmethod
    def backward(ctx, grad):
        from . import _native
        (win,) = ctx.saved_tensors
        g = grad.contiguous()
        N, C, H, W = ctx.in_shape
        gx = torch.empty(ctx.in_shape, device=g.device, dtype=g.dtype)
        _native.call("m2f_maxpool3s2_bwd", g.data_ptr(), win.data_ptr(), gx.data_ptr(), N * C, H, W,
                     _CODE[g.dtype], torch.cuda.current_stream(g.device).cuda_stream)
        return gx


class _MaxPool3s2NHWC(torch.autograd.Function):
    """The same pool on a channels-last 16-bit x (csrc/eltwise.hip ``m2f_maxpool3s2_nhwc``), y channels-last."""

    @staticmethod
    def forward(ctx, x):
        from . import _native
        N, C, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty(N, OH, OW, C, device=x.device, dtype=x.dtype).permute(0, 3, 1, 2)
        win = torch.empty(N, OH, OW, C, device=x.device, dtype=torch.uint8)
        _native.call("m2f_maxpool3s2_nhwc", 0, x.data_ptr(), y.data_ptr(), win.data_ptr(), N, H, W, C,
                     _CODE[x.dtype], torch.cuda.current_stream(x.device).cuda_stream)
        ctx.save_for_backward(win)
        ctx.in_shape = x.shape
        return y

    @staticmethod
    def backward(ctx, grad):
        from . import _native
        (win,) = ctx.saved_tensors
        N, C, H, W = ctx.in_shape
        g = grad.contiguous(memory_format=torch.channels_last)
        gx = torch.empty(N, H, W, C, device=g.device, dtype=g.dtype).permute(0, 3, 1, 2)
        _native.call("m2f_maxpool3s2_nhwc", 1, g.data_ptr(), gx.data_ptr(), win.data_ptr(), N, H, W, C,
                     _CODE[g.dtype], torch.cuda.current_stream(g.device).cuda_stream)
        return gx


def max_pool_stem(x):
    """detectron2 BasicStem's ``F.max_pool2d(x, kernel_size=3, stride=2, padding=1)``."""
    if (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.dim() == 4 and x.shape[1] % 8 == 0
            and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)):
        return _MaxPool3s2NHWC.apply(x)
    if x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and x.dim() == 4 and x.is_contiguous():
        return _MaxPool3s2.apply(x)
    return F.max_pool2d(x, kernel_size=3, stride=2, padding=1)


class Bottleneck(nn.Module):
    def __init__(self, cin, cb, cout, stride):
        super().__init__()
        self.shortcut = FrozenBNConv(cin, cout, 1, stride) if (cin != cout or stride != 1) else None
        self.conv1 = FrozenBNConv(cin, cb, 1, 1)             # STRIDE_IN_1X1: False
        self.conv2 = FrozenBNConv(cb, cb, 3, stride, 1)
        self.conv3 = FrozenBNConv(cb, cout, 1, 1)

    def forward(self, x, nout=1):
        """x: the input, or handles of it (conv, residual path[, others]); nout handles of the output."""
        xc, xr = (x[0], x[1]) if isinstance(x, tuple) else (x, x)
        out = bias_act(*self.conv1.conv_shift(xc))
        out = bias_act(*self.conv2.conv_shift(out))
        out, shift = self.conv3.conv_shift(out)
        if self.shortcut is not None:
            sc, sc_shift = self.shortcut.conv_shift(xr)
            shift = shift + sc_shift
        else:
            sc = xr
        return bias_act(out, shift, sc, nout)


class ResNet50(nn.Module):
    def __init__(self, channels_last=False):
        super().__init__()
        self.channels_last = channels_last   # NHWC activations end to end (MIOpen's NHWC kernels, no transposes)
        self.stem = FrozenBNConv(3, 64, 7, 2, 3)
        cfg = [("res2", 3, 64, 256, 1), ("res3", 4, 128, 512, 2), ("res4", 6, 256, 1024, 2),
               ("res5", 3, 512, 2048, 2)]
        cin = 64
        self.stage_names = []
        for name, n, cb, cout, stride in cfg:
            blocks = [Bottleneck(cin if i == 0 else cout, cb, cout, stride if i == 0 else 1) for i in range(n)]
            self.add_module(name, nn.Sequential(*blocks))
            self.stage_names.append(name)
            cin = cout

    def output_shape(self):
        ch = {"res2": 256, "res3": 512, "res4": 1024, "res5": 2048}
        st = {"res2": 4, "res3": 8, "res4": 16, "res5": 32}
        return {k: ShapeSpec(channels=ch[k], stride=st[k]) for k in self.stage_names}

    def forward(self, x):
        if self.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        x = bias_act(*self.stem.conv_shift(x))
        x = max_pool_stem(x)
        out = {}
        # each block output is handed on as one handle per consumer (conv, residual path, and at a stage
        # end the pixel decoder) so its ReLU backward sums their gradients in one pass
        for si, name in enumerate(self.stage_names):
            blocks = list(getattr(self, name))
            for bi, blk in enumerate(blocks):
                last = bi == len(blocks) - 1
                nout = (1 if si == len(self.stage_names) - 1 else 3) if last else 2
                x = blk(x, nout)
            out[name] = x[-1] if isinstance(x, tuple) else x
        return out


def default_cfg(num_queries=100, num_classes=133):
    """The model-shape keys of configs/coco/panoptic-segmentation/maskformer2_R50_bs16_50ep.yaml."""
    n = types.SimpleNamespace
    return n(MODEL=n(
        SEM_SEG_HEAD=n(IN_FEATURES=["res2", "res3", "res4", "res5"], CONVS_DIM=256, MASK_DIM=256, NORM="GN",
                       TRANSFORMER_ENC_LAYERS=6, DEFORMABLE_TRANSFORMER_ENCODER_IN_FEATURES=["res3", "res4", "res5"],
                       COMMON_STRIDE=4, NUM_CLASSES=num_classes, PIXEL_DECODER_NAME="MSDeformAttnPixelDecoder"),
        MASK_FORMER=n(DROPOUT=0.0, NHEADS=8, HIDDEN_DIM=256, NUM_OBJECT_QUERIES=num_queries, DIM_FEEDFORWARD=2048,
                      DEC_LAYERS=10, PRE_NORM=False, ENFORCE_INPUT_PROJ=False,
                      TRANSFORMER_DECODER_NAME="MultiScaleMaskedTransformerDecoder")))


class MaskFormerHead(nn.Module):
    """The reference's head glue (meta_arch/mask_former_head.py:115-132) for the
    "multi_scale_pixel_decoder" configuration: pixel decoder -> masked-attention decoder."""

    def __init__(self, cfg, input_shape):
        super().__init__()
        self.pixel_decoder = MSDeformAttnPixelDecoder(cfg, input_shape)
        self.predictor = MultiScaleMaskedTransformerDecoder(cfg, cfg.MODEL.SEM_SEG_HEAD.CONVS_DIM, True)

    def forward(self, features, mask=None):
        mask_features, _, multi_scale = self.pixel_decoder.forward_features(features)
        return self.predictor(multi_scale, mask_features, mask)


class MaskFormerR50(nn.Module):
    def __init__(self, cfg=None, channels_last=False):
        super().__init__()
        cfg = cfg or default_cfg()
        self.backbone = ResNet50(channels_last)
        self.sem_seg_head = MaskFormerHead(cfg, self.backbone.output_shape())
        self.register_buffer("pixel_mean", torch.tensor(PIXEL_MEAN).view(-1, 1, 1), False)
        self.register_buffer("pixel_std", torch.tensor(PIXEL_STD).view(-1, 1, 1), False)

    @property
    def pixel_decoder(self):
        return self.sem_seg_head.pixel_decoder

    @property
    def predictor(self):
        return self.sem_seg_head.predictor

    def forward(self, images):
        x = (images - self.pixel_mean) / self.pixel_std
        return self.sem_seg_head(self.backbone(x))


# backbone output channels of the Swin variants in BASELINE configs 4 and 5 (EMBED_DIM 192 / 96, x2 per stage)
SWIN_CHANNELS = {"swin_l": {"res2": 192, "res3": 384, "res4": 768, "res5": 1536},
                 "swin_t": {"res2": 96, "res3": 192, "res4": 384, "res5": 768}}
STRIDES = {"res2": 4, "res3": 8, "res4": 16, "res5": 32}


class HeadBench(nn.Module):
    """The per-rank slice of BASELINE configs 4 and 5 without the backbone (the Swin is outside the hot path):
    backbone-shaped features -> MSDeformAttnPixelDecoder -> (video) masked-attention decoder, as
    MaskFormerHead.layers (mask_former_head.py:118-121).  Config 4: Swin-L channels, Q = 200, K = 80
    (configs/coco/instance-segmentation/swin/maskformer2_swin_large_IN21k_384_bs16_100ep.yaml); config 5:
    Swin-T channels, the video decoder with Q = 100, K = 40 and T frames per clip
    (configs/youtubevis_2019/video_maskformer2_R50_bs16_8ep.yaml)."""

    def __init__(self, swin, num_queries, num_classes, frames=None):
        super().__init__()
        from .video_decoder import VideoMultiScaleMaskedTransformerDecoder
        shape = {k: ShapeSpec(channels=c, stride=STRIDES[k]) for k, c in SWIN_CHANNELS[swin].items()}
        self.pixel_decoder = MSDeformAttnPixelDecoder(
            shape, transformer_dropout=0.0, transformer_nheads=8, transformer_dim_feedforward=1024,
            transformer_enc_layers=6, conv_dim=256, mask_dim=256, norm="GN",
            transformer_in_features=["res3", "res4", "res5"], common_stride=4)
        kw = dict(num_classes=num_classes, hidden_dim=256, num_queries=num_queries, nheads=8, dim_feedforward=2048,
                  dec_layers=9, pre_norm=False, mask_dim=256, enforce_input_project=False)
        if frames:
            self.predictor = VideoMultiScaleMaskedTransformerDecoder(256, True, num_frames=frames, **kw)
        else:
            self.predictor = MultiScaleMaskedTransformerDecoder(256, True, **kw)

    def forward(self, features):
        mask_features, _, multi_scale = self.pixel_decoder.forward_features(features)
        return self.predictor(multi_scale, mask_features)


def head_features(swin, n, h, w, device, seed=0):
    """Backbone-shaped random features (requires_grad: their gradient is what the backbone would receive)."""
    g = torch.Generator(device=device).manual_seed(seed)
    return {k: torch.randn(n, c, h // STRIDES[k], w // STRIDES[k], device=device, generator=g).requires_grad_()
            for k, c in SWIN_CHANNELS[swin].items()}


def wrap_ddp(model, device=None):
    """Data parallel over the image batch: DDP's bucketed gradient all-reduce (RCCL on ROCm, gloo on
    CPU) overlapped with the backward -- the path's only cross-GPU exchange."""
    kw = dict(broadcast_buffers=False, gradient_as_bucket_view=True, bucket_cap_mb=64)
    if device is not None and device.type == "cuda":
        kw["device_ids"] = [device.index]
    return torch.nn.parallel.DistributedDataParallel(model, **kw)


def param_digest(model):
    """Per-parameter bit checksums, int64 (n_params,): the sum of each parameter's raw 32-bit words (16-bit
    parameters are widened first).  Two replicas hold bitwise-equal parameters only if these agree, so comparing
    them across ranks checks that data parallelism kept every replica in step (train_net.py:328 launches one
    replica per GPU; DDP's all-reduce must leave them identical)."""
    out = []
    for p in model.parameters():
        t = p.detach()
        if t.element_size() != 4:
            t = t.float()
        out.append(t.contiguous().view(torch.int32).to(torch.int64).sum())
    return torch.stack(out) if out else torch.zeros(0, dtype=torch.int64)


def rank_consistency(model, elapsed=None):
    """All-gather :func:`param_digest` (and each rank's timed-loop seconds) over the default process group.
    Returns {"world_seen", "ranks_agree", "mismatched_params", "step_s_min", "step_s_max"}; at world size 1 (no
    process group) the trivially consistent record of this process alone."""
    import torch.distributed as dist
    dig = param_digest(model)
    if not (dist.is_available() and dist.is_initialized()):
        rec = {"world_seen": 1, "ranks_agree": True, "mismatched_params": 0}
        if elapsed is not None:
            rec.update(step_s_min=elapsed, step_s_max=elapsed)
        return rec
    world = dist.get_world_size()
    dev = dig.device if dist.get_backend() == "gloo" else next(model.parameters()).device
    dig = dig.to(dev)
    allg = [torch.empty_like(dig) for _ in range(world)]
    dist.all_gather(allg, dig)
    bad = torch.zeros(dig.numel(), dtype=torch.bool, device=dev)
    for d in allg[1:]:
        bad |= d != allg[0]
    rec = {"world_seen": world, "ranks_agree": not bool(bad.any()), "mismatched_params": int(bad.sum())}
    if elapsed is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        ts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(ts, t)
        vals = [float(x) for x in ts]
        rec.update(step_s_min=min(vals), step_s_max=max(vals))
    return rec


def graph_safe_sum(x):
    """``x.sum(dtype=float32)`` as dim-wise reductions over rows of at most 1024 elements, repeated until one
    remains: torch's single-output reduction of a large tensor zeroes its cross-block semaphores with a memset, and
    on this ROCm a memset captured in a HIP graph is not re-run correctly on replay (tools/graph_memset_check.py),
    which :class:`GraphStep` relies on.  Eager and replayed steps sum in the same order."""
    v = x.reshape(-1)
    first = True
    while first or v.numel() > 1:
        n = v.numel()
        rows = (n + 1023) // 1024
        if rows * 1024 != n:
            v = torch.cat([v, v.new_zeros(rows * 1024 - n)])
        v = v.view(rows, 1024).sum(1, dtype=torch.float32)
        first = False
    return v.view(())


class _MeanF32(torch.autograd.Function):
    """``x.float().mean()`` without the fp32 copy: the mean accumulates in fp32 straight from the bf16
    masks, and the gradient is the same bf16(g / numel) the cast's backward would produce, written as one
    fill (no fp32 (B, Q, H, W) intermediate in either pass)."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape, ctx.dtype, ctx.n = x.shape, x.dtype, x.numel()
        return graph_safe_sum(x) / x.numel()

    @staticmethod
    def backward(ctx, g):
        v = (g.float() / ctx.n).to(ctx.dtype)
        return torch.empty(ctx.shape, dtype=ctx.dtype, device=g.device).fill_(v)


def _mean_f32(x):
    return _MeanF32.apply(x) if x.requires_grad else graph_safe_sum(x) / x.numel()


def surrogate_loss(out):
    """Sum over the 10 heads of mean(pred_logits) + mean(pred_masks), in fp32."""
    heads = [out] + list(out["aux_outputs"])
    return sum(_mean_f32(h["pred_logits"]) + _mean_f32(h["pred_masks"]) for h in heads)


def make_optimizer(model, capturable=False):
    """AdamW (lr 1e-4, weight decay 0.05; train_net.py:185-263).  On a GPU the fused single-kernel form: with
    it GradScaler.step hands found_inf to the kernel instead of reading it on the host (torch's non-fused path
    syncs on found_inf.item() every fp16 step).  Same update arithmetic.  ``capturable``: the step counter on the
    device, so the step can be captured in a graph (:class:`GraphStep`)."""
    params = list(model.parameters())
    if params and params[0].is_cuda:
        return torch.optim.AdamW(params, lr=1e-4, weight_decay=0.05, fused=True, capturable=capturable)
    return torch.optim.AdamW(params, lr=1e-4, weight_decay=0.05, foreach=True)


def make_scaler(amp_dtype):
    """detectron2's AMPTrainer scales the loss under fp16 autocast (GradScaler); bf16 and fp32 need none."""
    if amp_dtype is torch.float16:
        return torch.amp.GradScaler("cuda")
    return None


def train_step(model, opt, images, amp_dtype=torch.bfloat16, clip=0.01, scaler=None):
    """One step: forward under autocast, the surrogate loss, backward (scaled under fp16), full-model grad-norm
    clipping, AdamW.  ``images``: the image batch, or a feature dict for :class:`HeadBench`."""
    opt.zero_grad(set_to_none=True)
    dev = images.device if torch.is_tensor(images) else next(iter(images.values())).device
    if not torch.is_tensor(images):
        for t in images.values():
            t.grad = None
    with torch.autocast(device_type=dev.type, dtype=amp_dtype, enabled=amp_dtype is not None):
        out = model(images)
        loss = surrogate_loss(out)
    if scaler is not None:
        scaler.scale(loss).backward()
        scaler.unscale_(opt)
        torch.nn.utils.clip_grad_norm_(model.parameters(), clip, foreach=True)
        scaler.step(opt)
        scaler.update()
        return loss.detach()
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), clip, foreach=True)
    opt.step()
    return loss.detach()


_NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
               7: "event_record", 10: "mem_alloc", 11: "mem_free"}


def graph_node_counts(graph):
    """Node kinds of a captured torch.cuda.CUDAGraph (kept with keep_graph=True), through the HIP runtime's
    hipGraphGetNodes / hipGraphNodeGetType."""
    hip = ctypes.CDLL("libamdhip64.so")
    g = ctypes.c_void_p(graph.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    if hip.hipGraphGetNodes(g, None, ctypes.byref(n)) != 0:
        raise RuntimeError("hipGraphGetNodes failed")
    nodes = (ctypes.c_void_p * n.value)()
    if hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) != 0:
        raise RuntimeError("hipGraphGetNodes failed")
    counts = {}
    t = ctypes.c_int(0)
    for i in range(n.value):
        if hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t)) != 0:
            raise RuntimeError("hipGraphNodeGetType failed")
        k = _NODE_TYPES.get(t.value, str(t.value))
        counts[k] = counts.get(k, 0) + 1
    return counts


class GraphMemsetError(RuntimeError):
    """A captured step holds memset nodes while graph packet capture is on (see :class:`GraphStep`)."""

    def __init__(self, msg, nodes):
        super().__init__(msg)
        self.nodes = nodes


class GraphStep:
    """The whole training step -- forward, loss, backward, GradScaler unscale / inf check, gradient clipping and
    the fused AdamW (capturable: its step counter lives on the device) -- captured once as a HIP graph
    (torch.cuda.CUDAGraph) and replayed.  The per-rank slices of configs 4 and 5 launch a few thousand small
    kernels per step for two images, more than the host issues in the time the GPU runs them; a replay issues them
    all at once.  Every input is static (the same feature / image tensors each step), the library's launches go to
    torch's current stream (the capture stream), and nothing in the step reads a device value on the host (host
    spatial shapes are tagged up front, GradScaler hands found_inf to the fused optimizer).  Warm-up steps run
    eagerly on a side stream first (lazy state, MIOpen find-db, workspaces), as torch's whole-network capture
    recipe prescribes.

    Replay correctness: with the ROCm runtime's graph packet capture on (its default, unless
    ``DEBUG_CLR_GRAPH_PACKET_CAPTURE=0`` was set before HIP started) a captured memset is not re-run correctly on
    later replays.  The constructor counts the captured node kinds (``nodes``) and raises
    :class:`GraphMemsetError` instead of returning a graph that would replay wrong sums."""

    def __init__(self, model, opt, images, amp_dtype, scaler=None, warmup=3, debug_dump=None, sdpa_math=False):
        from torch.nn.attention import SDPBackend, sdpa_kernel
        import contextlib
        self.model, self.opt, self.images, self.amp, self.scaler = model, opt, images, amp_dtype, scaler
        # sdpa_math: the decoder's self-attention on the math backend (bitwise-repeatable; tests)
        ctx = sdpa_kernel([SDPBackend.MATH]) if sdpa_math else contextlib.nullcontext()
        with ctx:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    train_step(model, opt, images, amp_dtype, scaler=scaler)
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            self.graph = torch.cuda.CUDAGraph(keep_graph=True)
            if debug_dump:
                self.graph.enable_debug_mode()
            with torch.cuda.graph(self.graph):
                self.loss = train_step(model, opt, images, amp_dtype, scaler=scaler)
        if debug_dump:   # the captured graph as a dot file (node types and kernel names; diagnostics)
            self.graph.debug_dump(debug_dump)
        # node kinds (kernel / memcpy / memset ...): a memset node replays wrongly under the runtime's packet capture
        self.nodes = graph_node_counts(self.graph)
        if self.nodes.get("memset") and os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") != "0":
            raise GraphMemsetError(
                f"the captured step holds {self.nodes['memset']} memset node(s), which the ROCm runtime's graph packet "
                "capture replays wrongly (tools/graph_memset_check.py): set DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 before HIP "
                "starts, or run the step eagerly", self.nodes)
        self.graph.instantiate()

    def __call__(self):
        self.graph.replay()
        return self.loss
