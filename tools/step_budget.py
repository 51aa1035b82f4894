"""Per-step time budget of the config-2 training step (bench.py's step: AMP fp16 + GradScaler, fwd + bwd + clip +
fused AdamW), in three views:

  phases    HIP events at the phase boundaries (backbone / pixel decoder / decoder fwd, loss, decoder / pixel decoder /
            backbone bwd, clip, optimizer), mean over --steps steps;
  families  every GPU kernel of --prof-steps profiled steps (torch.profiler), grouped into the hand-written SURVEY §8
            kernels (MSDA, masked attention, mask heads), the x3 fp32 engine, the other libbm2f kernels, hipBLASLt,
            MIOpen, RCCL and torch's own elementwise / reduction / copy kernels ("glue");
  glue      the torch kernels by the aten op that launched them, its input shapes and dtypes, and the Python call
            site behind it (forward: the frame; backward: the forward call that built the autograd node, from a
            separate anomaly-mode step).

    python tools/step_budget.py [--out gpurun_out/budget] [--steps 3] [--prof-steps 2] [--amp fp16]

Writes <out>.json and <out>.md."""
import argparse
import collections
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bm2f_amd.miopen_tuning import use_shipped_find_db  # noqa: E402

use_shipped_find_db()
import torch  # noqa: E402

from bm2f_amd.bench_model import (MaskFormerR50, default_cfg, make_optimizer, make_scaler,  # noqa: E402
                                  surrogate_loss, train_step)

HOT = (("msda", "§8 MSDA (fwd + bwd)"), ("mattn", "§8 masked attention"), ("mask_heads", "§8 mask heads"),
       ("mask_de", "§8 mask heads"), ("mask_df", "§8 mask heads"), ("mask_row_fix", "§8 mask heads"),
       ("attn_mask_bits", "§8 mask heads"))


def family(name):
    n = name
    for key, fam in HOT:
        if key in n:
            return fam
    if "x3_" in n:
        return "x3 fp32 engine (encoder linears, pixel-decoder convs)"
    if n.startswith("Cijk_") or "hipblaslt" in n.lower():
        return "hipBLASLt GEMMs"
    if n.startswith(("igemm_", "batched_transpose", "SubTensorOp", "MIOpen", "naive_conv", "Op2d", "Op1d",
                     "gridwise", "transpose_NCHW", "transpose_NHWC")) or "miopen" in n.lower():
        return "MIOpen (backbone convs + layout transposes)"
    if "nccl" in n.lower() or "rccl" in n.lower():
        return "RCCL"
    if n.startswith("__amd_rocclr"):
        return "runtime copies / fills"
    if "at::native" in n or n.startswith(("void at::", "at::")) or "elementwise_kernel" in n or "reduce_kernel" in n:
        return "torch glue (elementwise / reductions / copies)"
    if "(anonymous namespace)" in n or n.startswith("_ZN12_GLOBAL__N_1"):
        return "other libbm2f kernels (add+LN, GN, FPN, transposes, backbone epilogues)"
    return "other"


def short(name, n=110):
    return name if len(name) <= n else name[:n] + "..."


def phases(model, opt, images, amp, scaler, steps):
    names = ["start", "backbone_fwd", "pixdec_fwd", "decoder_fwd", "loss", "decoder_bwd", "pixdec_bwd",
             "backbone_bwd", "unscale+clip", "opt+scaler"]
    tot = {n: 0.0 for n in names[1:]}
    for it in range(steps + 1):
        ev = {}

        def mark(name):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev[name] = e
        opt.zero_grad(set_to_none=True)
        mark("start")
        with torch.autocast("cuda", dtype=amp):
            x = (images - model.pixel_mean) / model.pixel_std
            feats = model.backbone(x)
            mark("backbone_fwd")
            mf, _, ms = model.pixel_decoder.forward_features(feats)
            mark("pixdec_fwd")
            out = model.predictor(ms, mf)
            mark("decoder_fwd")
            loss = surrogate_loss(out)
            mark("loss")
        mf.register_hook(lambda g: mark("decoder_bwd"))
        feats["res5"].register_hook(lambda g: mark("pixdec_bwd"))
        scaler.scale(loss).backward()
        mark("backbone_bwd")
        scaler.unscale_(opt)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.01, foreach=True)
        mark("unscale+clip")
        scaler.step(opt)
        scaler.update()
        mark("opt+scaler")
        torch.cuda.synchronize()
        if it == 0:
            continue
        for i in range(1, len(names)):
            tot[names[i]] += ev[names[i - 1]].elapsed_time(ev[names[i]]) / steps
    return tot


MARK = "FillFunctor<short>"   # phase-boundary marker kernels (an int16 fill): nothing else in the step fills int16


def marked_step(model, opt, images, amp, scaler, marker):
    """train_step with an int16 fill launched at each phase boundary (forward: in program order; backward: from
    tensor hooks, which run as autograd reaches them), so the kernel timeline splits into the phases."""
    opt.zero_grad(set_to_none=True)
    marker()
    with torch.autocast("cuda", dtype=amp):
        x = (images - model.pixel_mean) / model.pixel_std
        feats = model.backbone(x)
        marker()
        mf, _, ms = model.pixel_decoder.forward_features(feats)
        marker()
        out = model.predictor(ms, mf)
        marker()
        loss = surrogate_loss(out)
        marker()
    def hook(g):
        marker()   # returns None: the gradient is left as it is
    mf.register_hook(hook)
    feats["res5"].register_hook(hook)
    scaler.scale(loss).backward()
    marker()
    scaler.unscale_(opt)
    torch.nn.utils.clip_grad_norm_(model.parameters(), 0.01, foreach=True)
    marker()
    scaler.step(opt)
    scaler.update()
    marker()


PHASES = ["backbone_fwd", "pixdec_fwd", "decoder_fwd", "loss", "decoder_bwd", "pixdec_bwd", "backbone_bwd",
          "unscale+clip", "opt+scaler"]


def profile(model, opt, images, amp, scaler, steps):
    from torch.profiler import ProfilerActivity, profile as tprof
    buf = torch.zeros(1, dtype=torch.int16, device=images.device)
    with tprof(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(steps):
            marked_step(model, opt, images, amp, scaler, lambda: buf.fill_(1) and None)
        torch.cuda.synchronize()
    kern = collections.defaultdict(lambda: [0.0, 0])
    glue = collections.defaultdict(lambda: [0.0, 0, "", collections.Counter()])
    from torch.autograd import DeviceType
    evs = prof.profiler.kineto_results.events()
    ops = {}   # correlation id -> (cpu op name, input shapes)
    for e in evs:
        if e.device_type() == DeviceType.CPU and e.linked_correlation_id() == 0:
            ops[e.correlation_id()] = (e.name(), tuple(tuple(x) for x in (e.shapes() or []) if x))
    launches = []   # (gpu start, name, ms, cpu op, shapes)
    for e in evs:
        if e.device_type() == DeviceType.CUDA and e.duration_ns() > 0:
            op, shp = ops.get(e.linked_correlation_id(), ("?", ()))
            launches.append((e.start_ns(), e.name(), e.duration_ns() / 1e6, op, shp))
    launches.sort(key=lambda t: t[0])
    grid = collections.defaultdict(float)   # (phase, family) -> ms per step
    phase = -1
    for _, name, ms, op, shp in launches:
        if MARK in name:
            phase = (phase + 1) % (len(PHASES) + 1)
            continue
        if phase < 0 or phase >= len(PHASES):
            continue
        ph = PHASES[phase]
        fam = family(name)
        grid[(ph, fam)] += ms / steps
        kern[name][0] += ms / steps
        kern[name][1] += 1
        if fam.startswith("torch glue") or fam.startswith("runtime"):
            key = (op, shp)
            glue[key][0] += ms / steps
            glue[key][1] += 1
            glue[key][2] = short(name, 80)
            glue[key][3][ph] += 1
    return kern, glue, grid


def scan_sites(model, opt, images, amp, scaler):
    """(aten op, input shapes) -> Python call sites, from one eager step under a dispatch mode (anomaly mode
    keeps each autograd node's forward traceback)."""
    from torch.utils._python_dispatch import TorchDispatchMode
    sites = collections.defaultdict(collections.Counter)

    class Scan(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            shp = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor) and a.dim() > 0)
            name = "aten::" + func.__name__.split(".")[0]
            node = torch._C._current_autograd_node()
            if node is not None:
                tb = node.metadata.get("traceback_", [])
                lines = [ln.strip().splitlines()[0] for ln in tb if "bm2f_amd" in ln or "tools/" in ln]
                site = f"bwd of {node.name()} <- " + " <- ".join(
                    ln.split("File ")[-1].replace('"', "").replace(ROOT + "/", "") for ln in reversed(lines[-2:]))
            else:
                frames = [f for f in traceback.extract_stack() if "torch/" not in f.filename
                          and "step_budget" not in f.filename][-2:]
                site = " <- ".join(f"{os.path.relpath(f.filename, ROOT)}:{f.lineno}" for f in reversed(frames))
            sites[(name, shp)][site] += 1
            return out

    with torch.autograd.detect_anomaly(check_nan=False), Scan():
        train_step(model, opt, images, amp, scaler=scaler)
    torch.cuda.synchronize()
    return sites


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/budget")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--prof-steps", type=int, default=2)
    ap.add_argument("--amp", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--no-sites", action="store_true")
    ap.add_argument("--channels-last", type=int, default=1, choices=[0, 1], help="backbone layout (as bench.py)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = MaskFormerR50(default_cfg(), channels_last=bool(a.channels_last)).to(dev)
    opt = make_optimizer(model)
    amp = torch.float16 if a.amp == "fp16" else torch.bfloat16
    scaler = make_scaler(amp) or torch.amp.GradScaler("cuda", enabled=False)
    g = torch.Generator(device=dev).manual_seed(1000)
    images = torch.randn(16, 3, 1024, 1024, device=dev, generator=g) * 57.0 + 117.0
    for _ in range(3):
        train_step(model, opt, images, amp, scaler=scaler)
    torch.cuda.synchronize()
    ph = phases(model, opt, images, amp, scaler, a.steps)
    print("phases", json.dumps({k: round(v, 2) for k, v in ph.items()}), flush=True)
    kern, glue, grid = profile(model, opt, images, amp, scaler, a.prof_steps)
    sites = {} if a.no_sites else scan_sites(model, opt, images, amp, scaler)
    fams = collections.defaultdict(float)
    for n, (ms, _) in kern.items():
        fams[family(n)] += ms
    step_ms = sum(ph.values())
    kern_ms = sum(fams.values())
    res = {"step_ms_events": round(step_ms, 2), "kernel_ms_per_step": round(kern_ms, 2),
           "phases_ms": {k: round(v, 2) for k, v in ph.items()},
           "families_ms": {k: round(v, 2) for k, v in sorted(fams.items(), key=lambda x: -x[1])},
           "phase_family_ms": {ph: {f: round(v, 3) for (p2, f), v in sorted(grid.items()) if p2 == ph}
                               for ph in PHASES},
           "kernels": [{"name": short(n, 160), "family": family(n), "ms_per_step": round(ms, 3),
                        "calls_per_step": c / a.prof_steps}
                       for n, (ms, c) in sorted(kern.items(), key=lambda x: -x[1][0])[:80]],
           "glue": []}
    for (op, shp), (ms, c, kn, phs) in sorted(glue.items(), key=lambda x: -x[1][0])[:60]:
        st = sites.get((op, shp)) or collections.Counter()
        res["glue"].append({"op": op, "shapes": [list(s) for s in shp], "ms_per_step": round(ms, 3),
                            "calls_per_step": c / a.prof_steps, "kernel": kn, "phases": dict(phs),
                            "sites": [f"{n}x {s}" for s, n in st.most_common(4)]})
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out + ".json", "w") as f:
        json.dump(res, f, indent=1)
    lines = [f"# Config-2 step budget ({a.amp}, bs16 1024², 1x MI355X)", "",
             f"Step by HIP events: **{step_ms:.1f} ms**; GPU kernel time in the profiled steps: **{kern_ms:.1f} ms**.",
             "", "## Phases (HIP events)", "", "| phase | ms |", "|---|---|"]
    lines += [f"| {k} | {v:.2f} |" for k, v in ph.items()]
    lines += ["", "## Kernel families (torch.profiler, ms per step)", "", "| family | ms | share |", "|---|---|---|"]
    lines += [f"| {k} | {v:.2f} | {100 * v / kern_ms:.1f} % |" for k, v in res["families_ms"].items()]
    fl = list(res["families_ms"])
    abbrev = {f: f.split(" (")[0] for f in fl}
    lines += ["", "## Phase x family (kernel ms per step)", "",
              "| phase | " + " | ".join(abbrev[f] for f in fl) + " | total |", "|---" * (len(fl) + 2) + "|"]
    for ph in PHASES:
        row = [grid.get((ph, f), 0.0) for f in fl]
        lines.append(f"| {ph} | " + " | ".join(f"{v:.2f}" for v in row) + f" | {sum(row):.2f} |")
    lines += ["", "## Torch glue by call site (ms per step)", "", "| ms | calls | phase | op | shapes | site |",
              "|---|---|---|---|---|---|"]
    for gl in res["glue"][:40]:
        lines.append(f"| {gl['ms_per_step']:.3f} | {gl['calls_per_step']:g} | {','.join(gl['phases'])} | {gl['op']} | "
                     f"{' '.join('x'.join(map(str, s)) for s in gl['shapes'][:3])} | {'; '.join(gl['sites'][:2])} |")
    lines += ["", "## Top kernels (ms per step)", "", "| ms | calls | family | kernel |", "|---|---|---|---|"]
    lines += [f"| {k['ms_per_step']:.3f} | {k['calls_per_step']:g} | {k['family'].split(' (')[0]} | "
              f"`{short(k['name'], 90)}` |" for k in res["kernels"][:50]]
    with open(a.out + ".md", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]), flush=True)


if __name__ == "__main__":
    main()
