#!/usr/bin/env python
"""Benchmark: images/sec of the Mask2Former R50 training step (fwd + bwd + AdamW) on synthetic
1024x1024 batches, 16 images per GPU (BASELINE.json config 2; config 3 at --gpus 8).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 16] [--res 1024] [--amp fp16|bf16|none]

One process per GPU.  ``--gpus N`` with N > 1 outside torch.distributed.run starts
``python -m torch.distributed.run --nproc-per-node N`` itself (before touching the GPU) and exits with its
status; under torchrun (WORLD_SIZE set) N must equal WORLD_SIZE.  Gradients are all-reduced by DDP over
RCCL (backend "nccl"), the only exchange on this path.  Rank 0 prints ONE JSON line.
Besides the contract fields it reports:
  roofline      the MSDA backward kernel (the hot path's dominant hand-written kernel): algorithmic bytes
                per launch (115.60 MB per 1024^2 image) / its mean duration, measured with HIP
                events on the launch stream, vs the 8 TB/s HBM peak; traffic = PMC-measured HBM bytes per
                launch (profiles/msda_bwd_traffic.json).
  roofline_all  the same for every hand-written kernel family (HBM- or MFMA-bound as DESIGN.md §3 says),
                from extra instrumented steps after the timed region (the timed steps carry no events).
  The headline runs under AMP fp16 with a GradScaler, the reference's training precision
  (Base-COCO-PanopticSegmentation.yaml SOLVER.AMP.ENABLED; detectron2's AMPTrainer).
  modes         N=1 only: the same step under AMP bf16 (no scaler) and with no autocast at all (fp32 parity
                mode), fewer steps.
  achievable    N=1 only: measured ceilings on this box -- a float4 stream copy (m2f_stream_copy,
                2 x 2 GiB per launch) and an 8192^3 bf16 GEMM (hipBLASLt via torch.matmul) -- so each roofline
                entry carries its fraction of the spec peak (frac) and of the measured one (frac_achievable).
  cpu_baseline  the reference's CPU path (oracle/cpu_path.py) on config 1 (1 x 512^2) and one 1024^2 image,
                warm-up 1, median of 3, rank 0, N=1; value = the 1024^2 img/s.
  world_seen / ranks_agree / rank_check
                the process group's size as RCCL saw it (dist.get_world_size()), and whether every replica holds
                bitwise-equal parameters after the timed steps (per-parameter checksums of the raw words,
                all-gathered: bench_model.rank_consistency), with each rank's ms/step and their min / max -- so
                a config-3 run (--gpus 8) carries its own evidence that DDP kept the ranks in step.
  env           every M2F_* variable in the environment.  The bench refuses to run with any set (they select
                non-default engines or geometries); --allow-knobs permits them for experiments.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec fwd+bwd, R50 100-query 1024² bs16, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TF = 2500.0      # dense bf16/f16 MFMA
F32_PEAK_TF = 157.3        # f32 MFMA (= f32 vector)
LDS_B128_PEAK_GBS = 150000.0   # ds_read_b64/b128 with every CU streaming at 2.4 GHz (MI355X_MICROARCH.md §LDS)


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=[2, 4, 5],
                    help="BASELINE.json config: 2/3 = the R50 step (default; 3 is --gpus 8), 4 / 5 = the per-rank "
                         "pixel-decoder + decoder slice of the Swin-L Q=200 / video T=5 configs (backbone excluded)")
    ap.add_argument("--frames", type=int, default=5, help="config 5: frames per clip")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="images (config 5: clips) per GPU; default 16 / 2 / 2")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--queries", type=int, default=None, help="default 100 (configs 2, 5) / 200 (config 4)")
    ap.add_argument("--amp", default="fp16", choices=["fp16", "bf16", "none"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-modes", action="store_true", help="skip the bf16 / fp32 mode lines")
    ap.add_argument("--no-peaks", action="store_true", help="skip the achievable-peak probes")
    ap.add_argument("--no-dropin", action="store_true", help="skip the op-level MSDeformAttnFunction timing")
    ap.add_argument("--mode-steps", type=int, default=10)
    ap.add_argument("--mode-warmup", type=int, default=3)
    ap.add_argument("--kernel-steps", type=int, default=2, help="instrumented steps for roofline_all")
    ap.add_argument("--graph", type=int, default=None, choices=[0, 1],
                    help="capture the step in a HIP graph and replay it (default: on for the per-rank configs 4 / 5 "
                         "at one rank, whose small steps are host-launch bound; off for config 2)")
    ap.add_argument("--channels-last", type=int, default=None, choices=[0, 1],
                    help="config 2: run the R50 backbone channels-last (MIOpen NHWC kernels, no layout transposes; 156.8 vs "
                         "158.4 ms per step NCHW on one box, profiles/r05_g_bench_cl*.json).  Default: on for fp16 autocast, "
                         "whose NHWC kernels the shipped MIOpen find-db covers; off otherwise (without find-db entries "
                         "MIOpen's fast find picks NHWC kernels that run the step ~10x slower)")
    ap.add_argument("--allow-knobs", action="store_true")
    ap.add_argument("--master-port", type=int, default=29531)
    a = ap.parse_args(argv)
    if a.batch is None:
        a.batch = 16 if a.config == 2 else 2
    if a.queries is None:
        a.queries = 200 if a.config == 4 else 100
    if a.graph is None:
        a.graph = 1 if a.config in (4, 5) and a.gpus == 1 else 0
    return a


def knob_env():
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("M2F_")}


def maybe_launch(args):
    """--gpus N > 1 without torchrun: run torch.distributed.run as a child (no GPU touched here)."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        return
    if args.gpus <= 1:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={args.master_port}", os.path.abspath(__file__)] + sys.argv[1:]
    log("launching " + " ".join(cmd[2:]))
    raise SystemExit(subprocess.call(cmd))


# ----------------------------------------------------------------------------------------------------
# per-kernel timing: HIP events around libbm2f entry points, on torch's current stream (the stream the
# C ABI launches on), with each call's algorithmic work computed from its arguments
# ----------------------------------------------------------------------------------------------------
def _attn_bytes(a, fwd):
    # m2f_masked_attn_{fwd,bwd}(dtype, q, k, v, bits, [out, gout, lse,] B, Lq, Lk, H, hd, ...)
    o = 5 if fwd else 8
    dt, B, Lq, Lk, H, hd = a[0], a[o], a[o + 1], a[o + 2], a[o + 3], a[o + 4]
    el = 4 if dt == 0 else 2
    kv = 2 * B * Lk * H * hd * el
    q = B * Lq * H * hd * el
    bits = B * Lq * ((Lk + 31) // 32) * 4
    flops = 4 * B * H * Lq * Lk * hd
    if fwd:
        return kv + 2 * q + bits + B * H * Lq * 4, flops
    return 2 * kv + 4 * q + bits + B * H * Lq * 4, flops * 5 // 2


def _msda_bytes(a, fused, bwd):
    if fused:  # (value, proj, ld, ref, rbs, hs, [gout,] N, S, M, D, L, Lq, P, ...)
        o = 7 if bwd else 6
        N, S, M, D, L, Lq, P = a[o:o + 7]
    else:      # (value, shapes, lsi, loc, attn, [gout,] N, S, M, D, L, Lq, P, ...)
        o = 6 if bwd else 5
        N, S, M, D, L, Lq, P = a[o:o + 7]
    value = N * S * M * D * 4
    loc = N * Lq * M * L * P * 2 * 4
    attn = N * Lq * M * L * P * 4
    out = N * Lq * M * D * 4
    fwd_b = value + loc + attn + out
    gather = N * Lq * M * L * P * 4 * D * 4       # four corner rows of D fp32 per sample, through L1 / L2
    return (fwd_b + value + loc + attn if bwd else fwd_b), 0, gather


def _x3(M, N, K):
    return 0, 2 * M * N * K


ENTRIES = {
    # name: (family, bound, work(args) -> (bytes, flops))
    "m2f_msda_fused_bwd_f32": ("msda_bwd", "hbm", lambda a: _msda_bytes(a, True, True)),
    "m2f_msda_fused_bwd_hm_f32": ("msda_bwd", "hbm", lambda a: _msda_bytes(a, True, True)),
    "m2f_msda_bwd_f32": ("msda_bwd", "hbm", lambda a: _msda_bytes(a, False, True)),
    "m2f_msda_fused_fwd_f32": ("msda_fwd", "hbm", lambda a: _msda_bytes(a, True, False)),
    "m2f_msda_fused_fwd_hm_f32": ("msda_fwd", "hbm", lambda a: _msda_bytes(a, True, False)),
    "m2f_msda_fwd_f32": ("msda_fwd", "hbm", lambda a: _msda_bytes(a, False, False)),
    "m2f_attn_mask_bits": ("attn_mask_bits", "hbm", lambda a: (
        a[2] * a[3] * a[4] * a[5] * a[6] * (4 if a[1] == 0 else 2) + a[2] * a[3] * a[11] * 4, 0)),
    "m2f_masked_attn_fwd": ("masked_attn_fwd", "hbm", lambda a: _attn_bytes(a, True)),
    "m2f_masked_attn_bwd": ("masked_attn_bwd", "hbm", lambda a: _attn_bytes(a, False)),
    # (dtype, embed, feats, B, Q, C, T, H, W, th, tw, masks, bits, nwords): feats read + masks written
    "m2f_mask_heads_fwd": ("mask_heads_fwd", "hbm", lambda a: (
        2 * a[3] * a[6] * a[7] * a[8] * (a[5] + a[4]) + 2 * a[3] * a[4] * a[5] + 4 * a[3] * a[4] * a[13],
        2 * a[3] * a[4] * a[5] * a[6] * a[7] * a[8])),
    # (dtype, g, f, B, Q, C, n, de, ws, wsb, stream): G and F read once
    "m2f_mask_heads_bwd_embed": ("mask_heads_bwd_embed", "hbm", lambda a: (
        2 * a[3] * a[6].value * (a[4] + a[5]) + 2 * a[3] * a[4] * a[5], 2 * a[3] * a[4] * a[5] * a[6].value)),
    # (dtype, ptrs, H, et, B, Q, QP, C, n, out_dtype, df, stream): the heads' G read once, df written once
    "m2f_mask_heads_bwd_feats": ("mask_heads_bwd_feats", "hbm", lambda a: (
        2 * a[2] * a[4] * a[5] * a[8].value + (4 if a[9] == 0 else 2) * a[4] * a[7] * a[8].value,
        2 * a[2] * a[4] * a[5] * a[7] * a[8].value)),
    "m2f_gemm_f32x3_nt": ("x3_gemm_nt", "mfma", lambda a: _x3(a[11], a[12], a[13])),
    "m2f_gemm_f32x3_nt_add": ("x3_gemm_nt", "mfma", lambda a: _x3(a[14], a[15], a[16])),
    "m2f_gemm_f32x3_tn": ("x3_gemm_tn", "mfma", lambda a: _x3(a[7], a[8], a[9])),
    "m2f_conv_f32x3": ("x3_conv", "mfma", lambda a: _x3(a[4] * a[7] * a[8], a[6] if a[10] == 0 else a[5],
                                                      (a[5] if a[10] == 0 else a[6]) * a[9] * a[9])),
    "m2f_conv_f32x3_wgrad": ("x3_conv_wgrad", "mfma", lambda a: _x3(a[5] * a[9] * a[9], a[6], a[4] * a[7] * a[8])),
}

MFMA_NOTE = {
    "x3_gemm_nt": "fp32 GEMM as 6 bf16 MFMA products (split operands): mfma work = 6 x 2MNK vs the 2.5 PF bf16 peak",
    "x3_gemm_tn": "as x3_gemm_nt (weight gradients, split over rows, fixed-order slab sums)",
    "x3_conv": "as x3_gemm_nt (implicit-GEMM conv, 1x1 and 3x3)",
    "x3_conv_wgrad": "as x3_gemm_nt (1x1 conv weight gradients)",
    "mask_heads_fwd": "bqc,bchw->bqhw on bf16/f16 MFMA with the fused bitmask epilogue (HBM-bound: mfma_tflops)",
    "mask_heads_bwd_embed": "d embed = G F^T on bf16/f16 MFMA, split over HW (HBM-bound: mfma_tflops)",
    "mask_heads_bwd_feats": "d features = sum_h E_h^T G_h on bf16/f16 MFMA over the heads in place (HBM-bound)",
    "masked_attn_fwd": "flash-style masked attention on 16x16x16 bf16/f16 MFMA: 4 B H Lq Lk hd flops (HBM-bound: "
                       "mfma_tflops)",
    "masked_attn_bwd": "its backward (P recomputed from the saved LSE): 10 B H Lq Lk hd flops (HBM-bound: mfma_tflops)",
}


class KernelTimer:
    def __init__(self):
        self.enabled = False
        self.events = {}

    def install(self, native):
        fn = native.call
        timer = self

        def wrapped(name, *args):
            ent = ENTRIES.get(name)
            if not timer.enabled or ent is None:
                return fn(name, *args)
            import torch
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            out = fn(name, *args)
            e.record()
            work = ent[2](args)
            nbytes, flops = work[0], work[1]
            gather = work[2] if len(work) > 2 else 0
            timer.events.setdefault(ent[0], []).append((s, e, nbytes, flops, gather))
            return out

        native.call = wrapped

    def summary(self, steps):
        import torch
        torch.cuda.synchronize()
        res = {}
        for fam, evs in self.events.items():
            ms = [ev[0].elapsed_time(ev[1]) for ev in evs]
            nb = sum(ev[2] for ev in evs)
            fl = sum(ev[3] for ev in evs)
            ga = sum(ev[4] for ev in evs)
            tot = sum(ms)
            res[fam] = {"calls_per_step": len(ms) / steps, "mean_ms": tot / len(ms), "ms_per_step": tot / steps,
                        "bytes": nb, "flops": fl, "gather_bytes": ga, "total_ms": tot}
        return res


def roofline_entry(fam, k, bound):
    t = k["total_ms"] * 1e-3
    if bound == "hbm":
        ach = k["bytes"] / t / 1e9
        ent = {"kernel": fam, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(ach / HBM_PEAK_GBS, 4), "mean_launch_ms": round(k["mean_ms"], 4),
               "ms_per_step": round(k["ms_per_step"], 3)}
        if k["flops"] and fam in MFMA_NOTE:
            ent["mfma_tflops"] = round(k["flops"] / t / 1e12, 1)
            ent["note"] = MFMA_NOTE[fam]
        if k.get("gather_bytes"):
            rate = round(k["gather_bytes"] / t / 1e9, 1)
            if fam == "msda_fwd":   # the LDS-window forward reads its corner rows from LDS (ds_read_b128)
                ent["lds_gather_gbs"] = rate
                ent["lds_peak_gbs"] = LDS_B128_PEAK_GBS
                ent["frac_lds"] = round(rate / LDS_B128_PEAK_GBS, 4)
                ent["gather_note"] = ("corner rows (4 x 128 B per sample) read from the LDS windows by ds_read_b128, "
                                      "vs the chip's ds_read_b128 rate (MI355X_MICROARCH.md §LDS); not the binding "
                                      "limit: the kernel is VALU-issue bound (profiles/r04_pmc_fl1_*)")
            else:                   # the backward's phase 2 gathers corner rows through L1 / L2
                ent["gather_gbs"] = rate
                ent["gather_note"] = ("phase-2 corner-row gathers (4 x 128 B per sample) through L1 / L2, vs the "
                                      "measured gather probe (achievable.l2_gather_gbs); one of the units the "
                                      "kernel's phases use in turn, not the single binding limit")
        return ent
    if fam.startswith("x3"):
        ach = 6 * k["flops"] / t / 1e12
        return {"kernel": fam, "bound": "mfma", "achieved": round(ach, 1), "peak": BF16_PEAK_TF, "unit": "TFLOP/s",
                "frac": round(ach / BF16_PEAK_TF, 4), "fp32_equiv_tflops": round(k["flops"] / t / 1e12, 1),
                "mean_launch_ms": round(k["mean_ms"], 4), "ms_per_step": round(k["ms_per_step"], 3),
                "note": MFMA_NOTE.get(fam)}
    ach = k["flops"] / t / 1e12
    return {"kernel": fam, "bound": "mfma", "achieved": round(ach, 1), "peak": BF16_PEAK_TF, "unit": "TFLOP/s",
            "frac": round(ach / BF16_PEAK_TF, 4), "mean_launch_ms": round(k["mean_ms"], 4),
            "ms_per_step": round(k["ms_per_step"], 3), "note": MFMA_NOTE.get(fam)}


def measure_peaks(device):
    """Achievable ceilings on this box: HBM by a nontemporal stream copy, MFMA by a large bf16 GEMM."""
    import torch
    from bm2f_amd import _native
    st = torch.cuda.current_stream(device)
    nbytes = 2 << 30
    a = torch.empty(nbytes, dtype=torch.uint8, device=device).fill_(1)
    b = torch.empty_like(a)

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps * 1e-3

    t_copy = {mode: timed(lambda: _native.call("m2f_stream_copy", a.data_ptr(), b.data_ptr(), nbytes, mode,
                                               st.cuda_stream), 20) for mode in (0, 1)}
    del a, b
    n = 8192
    x = torch.randn(n, n, device=device, dtype=torch.bfloat16)
    y = torch.randn(n, n, device=device, dtype=torch.bfloat16)
    out = torch.empty(n, n, device=device, dtype=torch.bfloat16)
    t_mm = timed(lambda: torch.matmul(x, y, out=out), 20)
    del x, y, out
    torch.cuda.empty_cache()
    rates = {mode: 2 * nbytes / t / 1e9 for mode, t in t_copy.items()}
    # L2-resident gather of 128-byte rows from one head's value rows of one 1024^2 image (2.75 MB)
    rows, ng = 21504, 1 << 26
    table = torch.randn(rows, 32, device=device)
    sink = torch.empty(2048 * 256, device=device)
    t_g = timed(lambda: _native.call("m2f_gather_probe", table.data_ptr(), rows, ng, sink.data_ptr(), sink.numel(),
                                     st.cuda_stream), 10)
    del table, sink
    return {"hbm_gbs": round(max(rates.values()), 1), "bf16_gemm_tflops": round(2 * n ** 3 / t_mm / 1e12, 1),
            "l2_gather_gbs": round(128 * ng / t_g / 1e9, 1),
            "gather_probe": "m2f_gather_probe: 2^26 pseudo-random 128-B rows of a 2.75 MB table (one head's value rows "
                            "of a 1024^2 image, L2-resident), 8 lanes x float4 per row, 4 rows in flight, mean of 10",
            "hbm_probe": "m2f_stream_copy, 2 GiB in + 2 GiB out per launch, mean of 20, the faster of a one-pass "
                         f"float4 copy ({rates[0]:.0f} GB/s) and a strided nontemporal one ({rates[1]:.0f} GB/s)",
            "mfma_probe": f"torch.matmul bf16 {n}x{n}x{n} (hipBLASLt), mean of 20"}


def add_achievable(ent, peaks):
    if not peaks or not ent:
        return ent
    key = "hbm_gbs" if ent.get("unit") == "GB/s" else "bf16_gemm_tflops"
    ent["achievable_peak"] = peaks[key]
    ent["frac_achievable"] = round(ent["achieved"] / peaks[key], 4)
    if "gather_gbs" in ent and peaks.get("l2_gather_gbs"):
        ent["frac_gather"] = round(ent["gather_gbs"] / peaks["l2_gather_gbs"], 4)
    return ent


def head_config_line(args, world, value, knobs):
    """Metric / config fields of the per-rank config 4 / 5 lines (the backbone is excluded: not on the path)."""
    amp = args.amp + (" with GradScaler" if args.amp == "fp16" else "")
    if args.config == 4:
        return {"metric": "images/sec fwd+bwd per rank, Swin-L COCO-instance 200-query 1024^2, pixel decoder + "
                          "decoder (BASELINE config 4 slice, backbone excluded)",
                "unit": "images/s", "cpu_baseline": None,
                "data": "synthetic (Swin-L-shaped randn features, random-init weights)",
                "config": {"workload": f"config 4 per rank: {args.batch} images/GPU at {args.res}^2, Swin-L feature "
                                       f"channels 192/384/768/1536, MSDA pixel decoder (fp32) + {args.queries}-query "
                                       f"decoder, K=80, fwd+bwd+AdamW under AMP {amp}; the Swin-L backbone is not "
                                       "on the hot path and not timed",
                           "model": "maskformer2_swin_large head", "global_batch": world * args.batch,
                           "seq_len": sum((args.res // s) ** 2 for s in (32, 16, 8)), "queries": args.queries,
                           "parallelism": f"dp{world}", "env": knobs}}
    frames = args.frames
    return {"metric": "clips/sec fwd+bwd per rank, Video Mask2Former T=5 384x640, pixel decoder + video decoder "
                      "(BASELINE config 5 slice, backbone excluded)",
            "unit": "clips/s", "frames_per_s": round(value * frames, 3), "cpu_baseline": None,
            "data": "synthetic (Swin-T-shaped randn features, random-init weights)",
            "config": {"workload": f"config 5 per rank: {args.batch} clips x T={frames} frames at 360x640 padded to "
                                   f"384x640, Swin-T feature channels 96/192/384/768, MSDA pixel decoder per frame "
                                   f"(N={args.batch * frames}, S=5040, fp32) + video decoder ({args.queries} queries, "
                                   f"K=40, memory T*HW tokens, einsum bqc,btchw), fwd+bwd+AdamW under AMP {amp}; "
                                   "the backbone is not on the hot path and not timed",
                       "model": "video_maskformer2_swin_tiny head", "global_batch": world * args.batch,
                       "frames": frames, "seq_len": 5040, "queries": args.queries, "parallelism": f"dp{world}",
                       "env": knobs}}


def _msda_layer_case(device, n, res, noise, seed=7):
    """Config-2 layer-shaped MSDA inputs: reference-init rays (ms_deform_attn.py:66-80, 1..P px per level) plus
    N(0, noise px) offsets around each query's reference point, random logits, value and grad_output."""
    import math
    import torch
    shapes = [(res // s, res // s) for s in (32, 16, 8)]
    M, D, L, P = 8, 32, 3, 4
    S = sum(h * w for h, w in shapes)
    g = torch.Generator(device=device).manual_seed(seed)
    refs = []
    for h, w in shapes:
        ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h, device=device),
                                torch.linspace(0.5, w - 0.5, w, device=device), indexing="ij")
        refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
    ref = torch.cat(refs, 0)
    th = torch.arange(M, device=device) * (2 * math.pi / M)
    grid = torch.stack([th.cos(), th.sin()], -1)
    grid = grid / grid.abs().max(-1, keepdim=True)[0]
    off = (grid.view(M, 1, 1, 2) * torch.arange(1, P + 1, device=device).view(1, 1, P, 1)).expand(M, L, P, 2)
    off = off[None, None] + noise * torch.randn(n, S, M, L, P, 2, device=device, generator=g)
    logits = torch.randn(n, S, M, L * P, device=device, generator=g)
    value = torch.randn(n, S, M, D, device=device, generator=g)
    gout = torch.randn(n, S, M * D, device=device, generator=g)
    proj = torch.cat([off.reshape(n, S, -1), logits.reshape(n, S, -1)], -1).contiguous()
    rf = ref[None, :, None, :].expand(n, S, L, 2).contiguous()
    return shapes, value, proj, rf, gout


def measure_spread(device, n, res, timer, noise=4.0, iters=5):
    """The fused MSDA kernels (what the step runs) at the config-2 layer shape in the sampling regime of a trained
    model: reference-init rays plus N(0, 4 px) offsets (the step's own encoder sees near-init offsets).  The
    backward's windows then spill samples to the direct path and flush more rows."""
    import torch
    from bm2f_amd.msda import MSDeformAttnFusedFunction
    shapes, value, proj, rf, gout = _msda_layer_case(device, n, res, noise, seed=11)
    v, pj = value.requires_grad_(), proj.requires_grad_()

    def step():
        MSDeformAttnFusedFunction.apply(v, pj, rf, tuple(shapes), 4).backward(gout)
    step()
    torch.cuda.synchronize()
    saved, timer.events, timer.enabled = timer.events, {}, True
    for _ in range(iters):
        step()
    res_k = timer.summary(iters)
    timer.events, timer.enabled = saved, False
    out = []
    for fam in ("msda_fwd", "msda_bwd"):
        if res_k.get(fam):
            ent = roofline_entry(fam, res_k[fam], "hbm")
            ent["kernel"] = f"{fam}_spread{noise:g}"
            ent["note"] = (f"fused kernels, config-2 layer shape, reference-init rays + N(0, {noise:g} px) offsets "
                           f"(a trained model's spread), mean of {iters} launches")
            out.append(ent)
    del v, pj, value, proj, rf, gout
    torch.cuda.empty_cache()
    return out


def measure_dropin(device, n, res, timer, kern, iters=5):
    """The reference's unchanged op-level call (ops/modules/ms_deform_attn.py:116-117 ->
    MSDeformAttnFunction.apply, ops/functions/ms_deform_attn_func.py:32-49): a device spatial_shapes with no host
    tag, materialised sampling_locations / attention_weights, at the config-2 layer shape (reference-init rays
    + N(0, 1 px) noise).  Kernel time per launch (HIP events) against the fused kernels the step
    runs."""
    import math
    import torch
    from bm2f_amd.msda import MSDeformAttnFunction
    shapes = [(res // s, res // s) for s in (32, 16, 8)]
    M, D, L, P = 8, 32, 3, 4
    S = sum(h * w for h, w in shapes)
    g = torch.Generator(device=device).manual_seed(7)
    refs = []
    for h, w in shapes:
        ys, xs = torch.meshgrid(torch.linspace(0.5, h - 0.5, h, device=device),
                                torch.linspace(0.5, w - 0.5, w, device=device), indexing="ij")
        refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
    ref = torch.cat(refs, 0)
    th = torch.arange(M, device=device) * (2 * math.pi / M)
    grid = torch.stack([th.cos(), th.sin()], -1)
    grid = grid / grid.abs().max(-1, keepdim=True)[0]
    off = (grid.view(M, 1, 1, 2) * torch.arange(1, P + 1, device=device).view(1, 1, P, 1)).expand(M, L, P, 2)
    off = off[None, None] + torch.randn(n, S, M, L, P, 2, device=device, generator=g)
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32, device=device)
    loc = (ref[None, :, None, None, None, :] + off / norm[None, None, None, :, None, :]).contiguous()
    attn = torch.randn(n, S, M, L * P, device=device, generator=g).softmax(-1).view(n, S, M, L, P).contiguous()
    value = torch.randn(n, S, M, D, device=device, generator=g)
    gout = torch.randn(n, S, M * D, device=device, generator=g)
    lsi = torch.tensor([0, shapes[0][0] * shapes[0][1], shapes[0][0] * shapes[0][1] + shapes[1][0] * shapes[1][1]],
                       device=device)
    v, lc, a = (t.requires_grad_() for t in (value, loc, attn))

    def step():
        st = torch.tensor(shapes, dtype=torch.int64, device=device)   # fresh and untagged, as the encoder's
        MSDeformAttnFunction.apply(v, st, lsi, lc, a, 64).backward(gout)

    # the fused kernels on the SAME samples (offsets in pixels from the reference points, logits whose softmax
    # is attn): the step's own fused launches see the encoder's activations, a different sample spread
    from bm2f_amd.msda import MSDeformAttnFusedFunction
    proj = torch.cat([off.reshape(n, S, -1), attn.detach().log().reshape(n, S, -1)], -1).detach().contiguous()
    rf = ref[None, :, None, :].expand(n, S, L, 2).contiguous()
    vf, pf = value.detach().clone().requires_grad_(), proj.requires_grad_()

    def step_fused():
        MSDeformAttnFusedFunction.apply(vf, pf, rf, tuple(shapes), P).backward(gout)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        saved, timer.events, timer.enabled = timer.events, {}, True
        for _ in range(iters):
            fn()
        res_k = timer.summary(iters)
        timer.events, timer.enabled = saved, False
        return res_k
    def faster(a, b):   # per kernel family, the round with the lower mean
        return {f: min((r[f] for r in (a, b) if f in r), key=lambda e: e["mean_ms"]) for f in set(a) | set(b)}
    # two alternating rounds: the side timed first otherwise pays the clock ramp after the step's idle gap
    res_k, res_f = timed(step), timed(step_fused)
    res_k, res_f = faster(res_k, timed(step)), faster(res_f, timed(step_fused))
    out = {}
    for fam in ("msda_fwd", "msda_bwd"):
        k = res_k.get(fam)
        if not k:
            continue
        ent = roofline_entry(fam, k, "hbm")
        ent["kernel"] = f"{fam} via MSDeformAttnFunction (m2f_msda_{fam[5:]}_f32, untagged device spatial_shapes)"
        if res_f.get(fam):
            ent["fused_same_inputs_ms"] = round(res_f[fam]["mean_ms"], 4)
            ent["vs_fused_same_inputs"] = round(k["mean_ms"] / res_f[fam]["mean_ms"], 3)
        if kern.get(fam):
            ent["vs_fused_step_kernel"] = round(k["mean_ms"] / kern[fam]["mean_ms"], 3)
        out[fam] = ent
    del v, lc, a, value, loc, attn, gout, vf, pf, proj, rf
    torch.cuda.empty_cache()
    return out


def load_traffic():
    path = os.path.join(ROOT, "profiles", "msda_bwd_traffic.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def main():
    args = parse_args()
    # before any HIP call (bm2f_amd/__init__.py): the runtime's graph packet capture replays captured memsets
    # wrongly on this ROCm.  A graph-replayed run keeps it (faster replays) and checks after the capture that the
    # step holds no memset node (GraphStep.nodes), falling back to eager steps if it does; others turn it off.
    graph_run = bool(args.graph) and int(os.environ.get("WORLD_SIZE", "1")) == 1
    os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "1" if graph_run else "0")
    maybe_launch(args)
    knobs = knob_env()
    if knobs and not args.allow_knobs:
        raise SystemExit(f"bench.py: M2F_* variables set ({', '.join(knobs)}); they select non-default engines or "
                         "geometries. Unset them, or pass --allow-knobs for an experiment (they are recorded).")

    from bm2f_amd.miopen_tuning import use_shipped_find_db
    use_shipped_find_db()  # FAST find mode + the shipped NORMAL-mode find-db (no search on a fresh box)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)

    from bm2f_amd import _native
    from bm2f_amd.bench_model import (GraphMemsetError, GraphStep, HeadBench, MaskFormerR50, default_cfg, head_features, make_optimizer,
                                      make_scaler, rank_consistency, train_step, wrap_ddp)

    timer = KernelTimer()
    timer.install(_native)

    torch.manual_seed(0)
    if args.config == 2:
        if args.channels_last is None:
            args.channels_last = int(args.amp == "fp16")
        model = MaskFormerR50(default_cfg(num_queries=args.queries), channels_last=bool(args.channels_last)).to(device)
        g = torch.Generator(device=device).manual_seed(1000 + rank)
        images = torch.randn(args.batch, 3, args.res, args.res, device=device, generator=g) * 57.0 + 117.0
    elif args.config == 4:   # 2 images per GPU at 1024^2, Swin-L features
        model = HeadBench("swin_l", args.queries, 80).to(device)
        images = head_features("swin_l", args.batch, args.res, args.res, device, seed=1000 + rank)
    else:                    # 2 clips x T frames at 360x640 padded to 384x640, Swin-T features
        model = HeadBench("swin_t", args.queries, 40, frames=args.frames).to(device)
        images = head_features("swin_t", args.batch * args.frames, 384, 640, device, seed=1000 + rank)
    use_graph = bool(args.graph) and world == 1
    if world > 1:
        model = wrap_ddp(model, device)
    opt = make_optimizer(model, capturable=use_graph)
    dtypes = {"bf16": torch.bfloat16, "fp16": torch.float16, "none": None}

    def barrier():
        if world > 1:
            dist.barrier()

    def run(amp_name, steps, warmup, tag, graph=False):
        amp = dtypes[amp_name]
        scaler = make_scaler(amp)
        t0 = time.perf_counter()
        if graph:   # warm-up steps run eagerly inside the capture helper, then the captured step is replayed
            try:
                step_fn = GraphStep(model, opt, images, amp, scaler=scaler, warmup=max(warmup, 2))
                graph_info["nodes"] = step_fn.nodes
                log(f"{tag} warmup {warmup} + capture done ({time.perf_counter() - t0:.1f}s), nodes {step_fn.nodes}")
            except GraphMemsetError as e:   # memset nodes replay wrongly under packet capture
                log(f"{tag}: {e}: eager steps")
                graph_info.update(nodes=e.nodes, fallback="memset nodes under packet capture: eager steps")
                graph = False
        if not graph:
            def step_fn():
                return train_step(model, opt, images, amp, scaler=scaler)
            for i in range(warmup):
                step_fn()
                torch.cuda.synchronize()
                log(f"{tag} warmup {i + 1}/{warmup} done ({time.perf_counter() - t0:.1f}s)")
        barrier()
        torch.cuda.synchronize()
        start = last = time.perf_counter()
        for i in range(steps):
            step_fn()
            if time.perf_counter() - last > 30:
                log(f"{tag} step {i + 1}/{steps}")
                last = time.perf_counter()
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - start
        if world > 1:
            ts = [torch.zeros(1, device=device, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(ts, torch.tensor([elapsed], device=device, dtype=torch.float64))
            per_rank = [float(t) for t in ts]
            elapsed = max(per_rank)     # the job's time: the slowest rank
        else:
            per_rank = [elapsed]
        rank_times[tag] = per_rank
        log(f"{tag}: {steps} steps in {elapsed:.3f}s")
        return elapsed

    graph_info = {}
    rank_times = {}
    elapsed = run(args.amp, args.steps, args.warmup, "timed", graph=use_graph)
    # config 3 checks itself: after the timed steps every replica must hold bitwise-equal parameters (a parameter
    # DDP failed to reduce, or a rank that fell out of step, shows here), and the process group must be the size
    # the launcher asked for
    consistency = rank_consistency(model)
    consistency["rank_ms_per_step"] = [round(t / args.steps * 1e3, 3) for t in rank_times["timed"]]
    consistency["step_ms_min"] = min(consistency["rank_ms_per_step"])
    consistency["step_ms_max"] = max(consistency["rank_ms_per_step"])
    consistency["backend"] = dist.get_backend() if world > 1 else None
    if not consistency["ranks_agree"]:
        log(f"ranks disagree after the timed steps: {consistency['mismatched_params']} parameters differ")
    use_graph = use_graph and "fallback" not in graph_info
    peaks = None
    if world == 1 and not args.no_peaks:
        peaks = measure_peaks(device)
        log(f"achievable peaks: {peaks}")

    # instrumented steps (after the timed region): per-kernel-family durations and algorithmic work
    kern = {}
    if args.kernel_steps > 0:
        timer.enabled = True
        for _ in range(args.kernel_steps):
            train_step(model, opt, images, dtypes[args.amp], scaler=make_scaler(dtypes[args.amp]))
        kern = timer.summary(args.kernel_steps)
        timer.enabled = False

    dropin = None
    spread = []
    if world == 1 and args.config == 2 and not args.no_dropin:
        dropin = measure_dropin(device, args.batch, args.res, timer, kern)
        spread = measure_spread(device, args.batch, args.res, timer)
    modes = None
    if world == 1 and args.config == 2 and not args.no_modes:
        modes = {}
        for name in ("fp16", "bf16", "none"):
            if name == args.amp:
                continue
            torch.cuda.empty_cache()
            # the channels-last backbone only under fp16 autocast (the shipped NHWC find-db entries are fp16)
            cl_mode = bool(args.channels_last) and name == "fp16"
            model.backbone.channels_last = cl_mode
            el = run(name, args.mode_steps, args.mode_warmup, f"mode {name}")
            key = {"fp16": "amp_fp16", "bf16": "amp_bf16", "none": "fp32_parity"}[name]
            modes[key] = {"value": round(world * args.batch * args.mode_steps / el, 3), "unit": "images/s",
                          "ms_per_step": round(el / args.mode_steps * 1e3, 3), "steps": args.mode_steps, "warmup": args.mode_warmup,
                          "autocast": None if name == "none" else name,
                          "grad_scaler": name == "fp16", "backbone_layout": "channels_last" if cl_mode else "nchw"}
        model.backbone.channels_last = bool(args.channels_last)

    if rank == 0:
        value = world * args.batch * args.steps / elapsed
        roof = None
        bwd = kern.get("msda_bwd")
        if bwd:
            nbytes = bwd["bytes"] // int(round(bwd["calls_per_step"] * args.kernel_steps))   # per launch
            achieved = nbytes / (bwd["mean_ms"] * 1e-3) / 1e9
            tr = load_traffic()
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": (tr or {}).get("hbm_bytes_per_launch") if tr else None,
                    "kernel": "MSDA backward (m2f_msda_fused_bwd_hm_f32: the fused backward on the module's "
                              "head-major projection)",
                    "algorithmic_bytes_per_launch": nbytes, "mean_launch_ms": round(bwd["mean_ms"], 4)}
            if bwd.get("gather_bytes"):
                roof["gather_gbs"] = round(bwd["gather_bytes"] / (bwd["total_ms"] * 1e-3) / 1e9, 1)
            add_achievable(roof, peaks)
        bounds = {v[0]: v[1] for v in ENTRIES.values()}
        roof_all = [add_achievable(roofline_entry(fam, k, bounds[fam]), peaks)
                    for fam, k in sorted(kern.items(), key=lambda x: -x[1]["total_ms"])]
        roof_all += [add_achievable(ent, peaks) for ent in spread]
        cpu = None
        if world == 1 and args.config == 2 and not args.no_cpu_baseline:
            from oracle.cpu_path import cpu_model, time_cpu_step
            log("cpu baseline ...")
            s512, threads, t512 = time_cpu_step(res=512, images=1, steps=3, warmup=1)
            s1k, _, t1k = time_cpu_step(res=args.res, images=1, steps=3, warmup=1)
            cpu = {"value": round(1.0 / s1k, 4), "unit": "images/s", "cores": threads, "kind": "port",
                   "os_cpu_count": os.cpu_count(), "cpu_model": cpu_model(),
                   "config1_512_images_per_s": round(1.0 / s512, 4),
                   "sample": f"reference CPU path (oracle/cpu_path.py: the same model with the reference's "
                             f"ms_deform_attn_core_pytorch and MultiheadAttention math), fp32 fwd+bwd, 1 image, "
                             f"warm-up 1 + median of 3 at {args.res}^2 (value; s/step {[round(t, 3) for t in t1k]}) "
                             f"and at 512^2 (config 1; s/step {[round(t, 3) for t in t512]}); {threads} threads = "
                             f"os.cpu_count() capped by this process's CPU share"}
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.amp if args.amp != "none" else "fp32",
            "data": "synthetic (randn images, random-init weights)",
            "config": {"workload": "config 2: Mask2Former R50 COCO-panoptic, 100 queries, 1024x1024, "
                                   f"{args.batch} images/GPU, fwd+bwd+AdamW; pixel decoder + MSDA in fp32 "
                                   f"(as the reference forces), backbone/decoder under AMP {args.amp}"
                                   + (" with GradScaler" if args.amp == "fp16" else ""),
                       "model": "maskformer2_R50", "global_batch": world * args.batch,
                       "seq_len": sum((args.res // s) ** 2 for s in (32, 16, 8)), "queries": args.queries,
                       "parallelism": f"dp{world}", "env": knobs,
                       "backbone_layout": "channels_last" if args.channels_last else "nchw"},
            "roofline": roof, "roofline_all": roof_all, "achievable": peaks, "modes": modes, "cpu_baseline": cpu,
            "msda_op_dropin": dropin,
            "world_seen": consistency["world_seen"], "ranks_agree": consistency["ranks_agree"],
            "rank_check": consistency,
        }
        if args.config in (4, 5):
            line.update(head_config_line(args, world, value, knobs))
        line["config"]["graph_replay"] = use_graph
        if graph_info:
            line["config"]["graph"] = dict(graph_info, packet_capture=os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE"))
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
