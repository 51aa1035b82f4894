"""Teacher-forced decoder parity at full per-rank size (tests/test_scale_gpu.py; the harness itself is exercised on CPU
by tests/test_decoder_parity_cpu.py).

Three runs of one decoder module on the same inputs and loss (sum over the heads of mean(pred_logits) +
0.5 mean(pred_masks^2)):

1. the reference semantics in fp64 on the CPU: the module cast to fp64, the decoder ops routed through their torch
   restatements (oracle/decoder_ref.py: interpolate + sigmoid + threshold + row fix, MultiheadAttention math), i.e.
   mask2former_transformer_decoder.py:363-452 (and the video decoder's :365-474) evaluated in fp64.  Every attention
   mask it hands a cross-attention layer (and the logits it came from) is recorded;
2. the same reference semantics in fp32 on the GPU, every layer given run 1's masks: the reference's own fp32
   arithmetic, whose distance from run 1 is the noise floor the bars below scale with.  Run twice, with the
   self-attention's SDPA on torch's default backend and on its MATH backend: two equally valid fp32 evaluations of the
   reference, and the floor is the larger of their distances.  (Why two: at config 5 a layer-0 FFN pre-activation
   sits within fp32 rounding of 0, so some fp32 evaluations flip its ReLU against fp64 -- the MATH-backend reference
   and the HIP path do, the default-backend reference happens not to -- and the flip moves one hidden unit's row of
   linear1's weight gradient and, through it, the query embeddings' gradients by up to 4.5e-3 of their max: the same
   discrete event as a mask bit at the sigmoid threshold, tools/decoder_parity_diag.py,
   profiles/r06_g_decoder_parity_diag.txt.)
3. the HIP path (masked-attention kernels, the attention-mask kernel, the fp32 GEMM / einsum paths) in fp32, every
   layer given run 1's masks (teacher forcing: free-running, a logit within fp32 rounding of the sigmoid threshold
   flips a mask bit and that query's row then follows a different mask through the later layers -- a divergence that
   says nothing about the kernels).  The attention-mask kernel still runs on the HIP path's own logits at every
   layer: its bits are compared with run 1's, and every bit that differs must lie within fp32 rounding of the
   threshold (|fp64 resized logit| below 1e-5 of its row's largest).

Bars (the pixel decoder's rule, tests/test_scale_gpu.py::test_pixdec_config2_full_size_vs_reference_math): every
tensor -- outputs, input gradients and every parameter gradient -- within max(1e-3, 2 x run 2's larger distance from
run 1) of run 1, in both metrics (max |a - b| / max |b| and ||a - b|| / ||b||); outputs within 1e-3 outright
(north_star's fp32 bar)."""
import contextlib
import copy

import torch
import torch.nn.functional as F

from oracle.decoder_ref import torch_decoder_ops, unpack_bits


def _loss(out):
    heads = [out] + list(out["aux_outputs"])
    return sum(h["pred_logits"].mean() + 0.5 * (h["pred_masks"] ** 2).mean() for h in heads)


@contextlib.contextmanager
def _mask_hook(fn):
    """Wrap decoder_ops.attn_mask_bits (whatever it currently is): fn(inner, logits, size, row_fix) -> bits."""
    from bm2f_amd import decoder_ops
    inner = decoder_ops.attn_mask_bits

    def hooked(logits, size, row_fix=True):
        return fn(inner, logits, size, row_fix)

    decoder_ops.attn_mask_bits = hooked
    try:
        yield
    finally:
        decoder_ops.attn_mask_bits = inner


def _run(dec, xs, mf, ref_ops, hook):
    x = [t.clone().requires_grad_() for t in xs]
    m = mf.clone().requires_grad_()
    dec.zero_grad(set_to_none=True)
    with (torch_decoder_ops() if ref_ops else contextlib.nullcontext()), _mask_hook(hook):
        out = dec(x, m)
        _loss(out).backward()
    res = {"out_pred_masks": out["pred_masks"], "out_pred_logits": out["pred_logits"]}
    for i, h in enumerate(out["aux_outputs"]):
        res[f"out_aux{i}_pred_logits"] = h["pred_logits"]
    res.update({f"ingrad_x{i}": t.grad for i, t in enumerate(x)})
    res["ingrad_mask_features"] = m.grad
    res.update({f"pgrad_{n}": p.grad for n, p in dec.named_parameters() if p.grad is not None})
    return {k: v.detach().to("cpu", torch.float64) for k, v in res.items()}


def _resize(logits, size):
    """The reference's resize before the threshold (ref_attn_bool without the threshold): (B, Q, T*h*w) values."""
    if logits.dim() == 4:
        return F.interpolate(logits, size=size, mode="bilinear", align_corners=False).flatten(2)
    b, q, t = logits.shape[:3]
    m = F.interpolate(logits.flatten(0, 1), size=size, mode="bilinear", align_corners=False)
    return m.view(b, q, t * size[0] * size[1])


def _errs(a, b):
    return (((a - b).abs().max() / b.abs().max().clamp_min(1e-300)).item(),
            ((a - b).norm() / b.norm().clamp_min(1e-300)).item())


def decoder_parity(dec, xs, mf, device, hip=True, log=None, bit_tol=1e-5):
    """Runs 1-3 above for ``dec`` (on ``device``, fp32) with level inputs ``xs`` and mask features ``mf`` (fp32, on
    ``device``).  ``hip`` False makes run 3 another run of the restatements (the CPU harness check).  Returns
    (report lines, failing tensor names, bits checked, bits differing)."""
    # 1. fp64 reference on the CPU, recording every mask it hands a cross-attention layer
    records = []

    def record(inner, logits, size, row_fix):
        bits = inner(logits, size, row_fix)
        records.append((logits.detach().to("cpu", torch.float64).clone(), tuple(size), row_fix, bits.detach().cpu()))
        return bits

    dec64 = copy.deepcopy(dec).to("cpu", torch.float64)
    want = _run(dec64, [t.to("cpu", torch.float64) for t in xs], mf.to("cpu", torch.float64), True, record)
    del dec64

    # 2. / 3. fp32, teacher-forced with run 1's masks
    def forced_hook(check):
        it = iter(range(len(records)))

        def hook(inner, logits, size, row_fix):
            i = next(it)
            _, rsize, rfix, bits = records[i]
            assert tuple(size) == rsize and row_fix == rfix, f"mask call {i}: {size} vs {rsize}"
            if check is not None:
                check.append((i, inner(logits, size, row_fix).detach().cpu()))
            return bits.to(logits.device)
        return hook

    from torch.nn.attention import SDPBackend, sdpa_kernel
    ref32 = _run(dec, xs, mf, True, forced_hook(None))
    with sdpa_kernel([SDPBackend.MATH]):
        ref32m = _run(dec, xs, mf, True, forced_hook(None))
    own = []
    got = _run(dec, xs, mf, not hip, forced_hook(own))
    assert set(got) == set(want) == set(ref32), (set(want) ^ set(got))

    lines, bad = [], []
    n_bits = n_diff = 0
    for i, bits in own:
        logits64, size, _, forced = records[i]
        n = size[0] * size[1] * (logits64.shape[2] if logits64.dim() == 5 else 1)   # keys: T * h * w
        a, b = unpack_bits(bits, n), unpack_bits(forced, n)
        n_bits += a.numel()
        diff = a != b
        nd = int(diff.sum())
        n_diff += nd
        if nd:
            v = _resize(logits64, size)
            rowmax = v.abs().amax(-1, keepdim=True).expand_as(v)
            worst = (v[diff].abs() / rowmax[diff]).max().item()
            lines.append(f"mask call {i}: {nd} of {a.numel()} bits differ; largest |fp64 logit| / row max among them "
                         f"{worst:.2e} (bar {bit_tol:.0e})")
            if worst > bit_tol:
                bad.append(f"mask{i}")
    lines.append(f"attention-mask bits: {n_diff} of {n_bits} differ from the fp64 reference's")
    for k in sorted(want):
        assert got[k].shape == want[k].shape, k
        e_max, e_norm = _errs(got[k], want[k])
        (d_max, d_norm), (m_max, m_norm) = _errs(ref32[k], want[k]), _errs(ref32m[k], want[k])
        r_max, r_norm = max(d_max, m_max), max(d_norm, m_norm)
        bar, bar_n = max(1e-3, 2 * r_max), max(1e-3, 2 * r_norm)
        ok = e_max <= bar and e_norm <= bar_n and (not k.startswith("out_") or e_max < 1e-3)
        lines.append(f"{k:64s} hip max {e_max:.2e} norm {e_norm:.2e} | ref-fp32 max {d_max:.2e} / {m_max:.2e} norm "
                     f"{d_norm:.2e} / {m_norm:.2e} | bars {bar:.1e} / {bar_n:.1e} {'ok' if ok else 'FAIL'}")
        if not ok:
            bad.append(k)
    n_tight = sum(1 for k in want if _errs(got[k], want[k])[0] < 1e-3)
    lines.append(f"{len(want)} tensors ({sum(1 for k in want if k.startswith('pgrad_'))} parameter gradients); "
                 f"{n_tight} within 1e-3 of their max; failures: {bad}")
    if log:
        with open(log, "w") as fh:
            fh.write("\n".join(lines) + "\n")
    return lines, bad, n_bits, n_diff
