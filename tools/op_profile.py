"""torch.profiler op-level table of one training step (device time per aten op).
python tools/op_profile.py [--batch 16] [--part pixdec|all] [--rows 40] [--attribute]

--attribute  also maps every GPU kernel to the innermost aten op that launched it and the autograd
             node around it (from the profiler's chrome trace), and prints device time per
             (autograd node, aten op, kernel) -- e.g. which convolution_backward owns Col2Im."""
import argparse
import collections
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bm2f_amd.miopen_tuning import use_shipped_find_db  # noqa: E402

use_shipped_find_db()
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bm2f_amd.bench_model import MaskFormerR50, make_optimizer, make_scaler, train_step  # noqa: E402


def attribute(trace_path, rows):
    with open(trace_path) as f:
        ev = json.load(f)["traceEvents"]
    ops = collections.defaultdict(list)        # tid -> [(ts, end, name)]
    launches = {}                              # correlation -> (tid, ts)
    kernels = []
    for e in ev:
        if e.get("ph") != "X":
            continue
        cat = e.get("cat", "")
        if cat == "cpu_op" or cat == "user_annotation":
            ops[e["tid"]].append((e["ts"], e["ts"] + e.get("dur", 0), e["name"]))
        elif cat == "cuda_runtime":
            c = e.get("args", {}).get("correlation")
            if c is not None:
                launches[c] = (e["tid"], e["ts"])
        elif cat == "kernel":
            kernels.append(e)
    for v in ops.values():
        v.sort()
    agg = collections.defaultdict(float)
    cnt = collections.Counter()
    for k in kernels:
        c = k.get("args", {}).get("correlation")
        tid, ts = launches.get(c, (None, None))
        inner, node = "?", "-"
        if tid is not None:
            best = None
            for s, t, n in ops[tid]:
                if s > ts:
                    break
                if t >= ts:
                    if n.startswith("autograd::engine::evaluate_function"):
                        node = n.split(": ", 1)[-1]
                    elif best is None or s >= best[0]:
                        best = (s, n)
            inner = best[1] if best else "?"
        key = (node, inner, k["name"][:70])
        agg[key] += k.get("dur", 0)
        cnt[key] += 1
    total = sum(agg.values())
    print(f"\n== kernel attribution: {total / 1e3:.1f} ms device time ==")
    for key, us in sorted(agg.items(), key=lambda x: -x[1])[:rows]:
        print(f"{us / 1e3:8.2f} ms {cnt[key]:5d}  {key[0][:34]:34s} {key[1][:34]:34s} {key[2]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=45)
    ap.add_argument("--part", default="all")
    ap.add_argument("--amp", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--attribute", action="store_true")
    ap.add_argument("--shapes", default="", help="print input shapes of aten ops whose name contains this")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = MaskFormerR50().to(dev)
    opt = make_optimizer(model)
    x = torch.randn(a.batch, 3, a.res, a.res, device=dev) * 57 + 117
    if a.part == "pixdec":
        feats = {k: torch.randn(a.batch, c, a.res // s, a.res // s, device=dev, requires_grad=True)
                 for k, (c, s) in {"res2": (256, 4), "res3": (512, 8), "res4": (1024, 16), "res5": (2048, 32)}.items()}

        def step():
            mf, o0, ms = model.pixel_decoder.forward_features(feats)
            (mf.mean() + sum(t.mean() for t in ms)).backward()
    else:
        amp = torch.float16 if a.amp == "fp16" else torch.bfloat16
        scaler = make_scaler(amp)

        def step():
            train_step(model, opt, x, amp, scaler=scaler)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=bool(a.shapes)) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=60))
    if a.shapes:
        rows = [e for e in prof.key_averages(group_by_input_shape=True) if a.shapes in e.key]
        rows.sort(key=lambda e: -e.self_device_time_total)
        for e in rows[:30]:
            print(f"{e.self_device_time_total / 1e3:8.2f} ms {e.count:4d}  {e.key[:40]:40s} {str(e.input_shapes)[:160]}")
    if a.attribute:
        path = os.path.join(tempfile.gettempdir(), f"op_profile_{os.getpid()}.json")
        prof.export_chrome_trace(path)
        attribute(path, a.rows * 2)
        os.unlink(path)


if __name__ == "__main__":
    main()
