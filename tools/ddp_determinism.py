"""Which forward op makes two identical MaskFormerR50 copies disagree at step 0 (the DDP test's 1e-3 loss gap)?

    python tools/ddp_determinism.py

Runs identical copies (same weights, same 256^2 inputs, AMP bf16) in sequence and prints the loss and gradient
differences: (a) cold, as the DDP test ran them (the first copy meets every convolution shape first); (b) after a
warm-up step on a scratch copy; (c) warm and deterministic (torch.use_deterministic_algorithms + MSDA
deterministic mode).  Diagnostic only."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bm2f_amd import _native  # noqa: E402
from bm2f_amd.bench_model import MaskFormerR50, default_cfg, make_optimizer, train_step  # noqa: E402


def run(models, images):
    losses, grads = [], []
    for m in models:
        opt = make_optimizer(m)
        losses.append(train_step(m, opt, images, torch.bfloat16).item())
        grads.append({n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None})
    return losses, grads


def report(tag, losses, grads):
    l0 = losses[0]
    print(f"[{tag}] losses {losses}  rel diffs {[abs(l - l0) / abs(l0) for l in losses[1:]]}", flush=True)
    worst = []
    for i in range(1, len(grads)):
        w = (0.0, "")
        nbit = 0
        for n, g in grads[0].items():
            d = (grads[i][n] - g).norm().item() / max(g.norm().item(), 1e-20)
            nbit += int(not torch.equal(grads[i][n], g))
            w = max(w, (d, n))
        worst.append((w, nbit, len(grads[0])))
    print(f"[{tag}] worst relative L2 grad diff vs copy 0, params not bitwise equal: {worst}", flush=True)


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    base = MaskFormerR50(default_cfg()).to(dev)
    images = torch.randn(2, 3, 256, 256, device=dev) * 57.0 + 117.0
    copies = [copy.deepcopy(base) for _ in range(3)]
    report("cold", *run(copies, images))
    copies = [copy.deepcopy(base) for _ in range(3)]
    report("warm", *run(copies, images))
    torch.backends.cudnn.deterministic = True
    copies = [copy.deepcopy(base) for _ in range(3)]
    report("warm + cudnn.deterministic only", *run(copies, images))
    torch.backends.cudnn.deterministic = False
    torch.use_deterministic_algorithms(True, warn_only=True)
    copies = [copy.deepcopy(base) for _ in range(3)]
    report("warm + use_deterministic_algorithms only", *run(copies, images))
    torch.backends.cudnn.deterministic = True
    with _native.options(msda_bwd_det=1):
        copies = [copy.deepcopy(base) for _ in range(3)]
        report("warm+det", *run(copies, images))
        copies = [copy.deepcopy(base) for _ in range(3)]
        report("warm+det again", *run(copies, images))


if __name__ == "__main__":
    main()
