"""TEST INFRASTRUCTURE ONLY — the reference's CPU path for bench.py's cpu_baseline leg.

The benchmark's model (bm2f_amd.bench_model.MaskFormerR50) run on host cores with every HIP op
replaced by the oracle's CPU restatement of the reference algorithm: MSDA through
``ms_deform_attn_core_pytorch`` (oracle.msda_ref.core_pytorch; the reference's own CPU fallback,
ops/modules/ms_deform_attn.py:116-121), and the decoder's mask/attention ops through
oracle.decoder_ref (F.interpolate + sigmoid threshold, MultiheadAttention math with a bool mask).
This is the reference's CPU forward/backward, fp32, as SURVEY §6 timed it in the survey container.

Sampling follows BASELINE.md §3: config 1 (1 x 512^2) and one 1024^2 image, warm-up 1, median of 3.
"""
from __future__ import annotations

import contextlib
import os
import statistics
import time

import torch


@contextlib.contextmanager
def reference_cpu_ops():
    from bm2f_amd import decoder_ops, msda

    from .decoder_ref import pack_bits, ref_attn_bool, ref_masked_attention, unpack_bits
    from .msda_ref import core_pytorch

    saved = (msda.MSDeformAttnFunction.apply, decoder_ops.attn_mask_bits, decoder_ops.masked_attention)

    def msda_apply(value, shapes, lsi, loc, attn, step):
        return core_pytorch(value, shapes.cpu(), loc, attn)

    def bits_fn(logits, size, row_fix=True):
        return pack_bits(ref_attn_bool(logits.detach(), size, row_fix))

    def attn_fn(q, k, v, bits, num_heads, scale=None):
        return ref_masked_attention(q, k, v, unpack_bits(bits, k.shape[1]), num_heads, scale).to(q.dtype)

    msda.MSDeformAttnFunction.apply = staticmethod(msda_apply)
    decoder_ops.attn_mask_bits, decoder_ops.masked_attention = bits_fn, attn_fn
    try:
        yield
    finally:
        msda.MSDeformAttnFunction.apply, decoder_ops.attn_mask_bits, decoder_ops.masked_attention = saved


def cpu_threads():
    """Threads for the CPU leg: os.cpu_count(), capped by the CPU share this process may use (its affinity
    mask and OMP_NUM_THREADS: a GPU box exposes the whole machine's CPUs but grants one GPU's share)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def time_cpu_step(res=1024, images=1, steps=3, warmup=1, threads=None, seed=0):
    """Median seconds per fwd+bwd step of `images` images at res x res on the host (fp32, reference CPU
    path), after `warmup` untimed steps.  Returns (median_s, threads, all_times)."""
    from bm2f_amd.bench_model import MaskFormerR50, surrogate_loss

    threads = threads or cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(seed)
        model = MaskFormerR50().train()
        x = torch.randn(images, 3, res, res) * 57.0 + 117.0
        times = []
        with reference_cpu_ops():
            for i in range(warmup + steps):
                t0 = time.perf_counter()
                model.zero_grad(set_to_none=True)
                loss = surrogate_loss(model(x))
                loss.backward()
                if i >= warmup:
                    times.append(time.perf_counter() - t0)
        return statistics.median(times), threads, times
    finally:
        torch.set_num_threads(prev)
