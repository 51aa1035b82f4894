"""The N>1 path on CPU: two ranks over gloo, DDP-wrapped exactly as bench.py wraps the model
(bench_model.wrap_ddp), HIP ops replaced by the oracle's CPU restatements.

- one step of the head: every rank holds the same gradients, equal to the average of the per-rank gradients;
- two full training steps of the benchmark model (MaskFormerR50 at 64^2: backbone, pixel decoder, decoder,
  surrogate loss, grad-norm clipping, AdamW) through ``bench_model.train_step``, as bench.py runs config 3: the
  ranks' parameters agree bitwise after step 2 (``rank_consistency``, the check bench.py reports as
  ``ranks_agree``), and equal a single-process emulation that averages the two ranks' gradients by hand.
  A parameter DDP leaves unreduced, or a bucket error DDP raises only on its second iteration, fails here."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)


def _worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from bm2f_amd.bench_model import MaskFormerHead, default_cfg, surrogate_loss, wrap_ddp
    from bm2f_amd.registry import ShapeSpec
    from oracle.cpu_path import reference_cpu_ops

    shapes = {"res2": ShapeSpec(channels=256, stride=4), "res3": ShapeSpec(channels=512, stride=8),
              "res4": ShapeSpec(channels=1024, stride=16), "res5": ShapeSpec(channels=2048, stride=32)}
    torch.manual_seed(0)
    head = MaskFormerHead(default_cfg(num_queries=20, num_classes=10), shapes)
    g = torch.Generator().manual_seed(100 + rank)
    feats = {k: torch.randn(1, s.channels, 64 // s.stride, 64 // s.stride, generator=g) for k, s in shapes.items()}
    with reference_cpu_ops():
        # local gradients without DDP
        surrogate_loss(head(feats)).backward()
        local = torch.cat([p.grad.flatten() for p in head.parameters()])
        head.zero_grad(set_to_none=True)
        ddp = wrap_ddp(head)
        surrogate_loss(ddp(feats)).backward()
    synced = torch.cat([p.grad.flatten() for p in head.parameters()])
    avg = local.clone()
    dist.all_reduce(avg)
    avg /= world
    others = [torch.empty_like(synced) for _ in range(world)]
    dist.all_gather(others, synced)
    torch.save({"synced": synced, "avg": avg, "same": all(torch.equal(o, synced) for o in others)},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_two_ranks_gloo(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(tmp_path / f"rank{r}.pt", weights_only=True)
        assert res["same"], "ranks disagree after the DDP all-reduce"
        torch.testing.assert_close(res["synced"], res["avg"], rtol=1e-5, atol=1e-7)


RES, STEPS = 64, 2


def _images(rank):
    g = torch.Generator().manual_seed(1000 + rank)     # bench.py's per-rank image seed
    return torch.randn(1, 3, RES, RES, generator=g) * 57.0 + 117.0


def _model():
    from bm2f_amd.bench_model import MaskFormerR50, default_cfg
    torch.manual_seed(0)
    return MaskFormerR50(default_cfg(num_queries=20, num_classes=10))


def _emulate(world, steps):
    """Single process: per step, each rank's gradients on its own images, averaged by hand, then the same
    clipping and AdamW as train_step."""
    from bm2f_amd.bench_model import make_optimizer, surrogate_loss
    model = _model()
    opt = make_optimizer(model)
    params = list(model.parameters())
    for _ in range(steps):
        acc = [torch.zeros_like(p) for p in params]
        for r in range(world):
            opt.zero_grad(set_to_none=True)
            surrogate_loss(model(_images(r))).backward()
            for a, p in zip(acc, params):
                if p.grad is not None:
                    a += p.grad / world
        for a, p in zip(acc, params):
            p.grad = a
        torch.nn.utils.clip_grad_norm_(params, 0.01, foreach=True)
        opt.step()
    return torch.cat([p.detach().flatten() for p in params])


def _worker_steps(rank, world, port, out_dir):
    _init(rank, world, port)
    from bm2f_amd.bench_model import make_optimizer, param_digest, rank_consistency, train_step, wrap_ddp
    from oracle.cpu_path import reference_cpu_ops

    model = _model()
    start = param_digest(model)
    ddp = wrap_ddp(model)
    opt = make_optimizer(ddp)
    images = _images(rank)
    with reference_cpu_ops():
        losses = [float(train_step(ddp, opt, images, amp_dtype=None)) for _ in range(STEPS)]
        rec = rank_consistency(ddp, elapsed=float(rank))
        emu = _emulate(world, STEPS) if rank == 0 else None
    params = torch.cat([p.detach().flatten() for p in model.parameters()])
    torch.save({"rec": rec, "losses": losses, "params": params, "emu": emu,
                "moved": bool((param_digest(model) != start).any())}, os.path.join(out_dir, f"steps{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_two_ranks_two_train_steps_gloo(tmp_path):
    port = _free_port()
    mp.spawn(_worker_steps, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = [torch.load(tmp_path / f"steps{r}.pt", weights_only=True) for r in range(2)]
    for r in res:
        assert r["rec"]["world_seen"] == 2
        assert r["rec"]["ranks_agree"], f"{r['rec']['mismatched_params']} parameters differ across ranks"
        assert r["rec"]["step_s_min"] == 0.0 and r["rec"]["step_s_max"] == 1.0
        assert r["moved"], "the optimizer did not change the parameters"
    assert torch.equal(res[0]["params"], res[1]["params"])
    assert res[0]["losses"] != res[1]["losses"], "ranks saw the same images"
    torch.testing.assert_close(res[0]["params"], res[0]["emu"], rtol=1e-6, atol=1e-7)


def test_rank_consistency_single_process():
    from bm2f_amd.bench_model import rank_consistency
    rec = rank_consistency(torch.nn.Linear(4, 3), elapsed=2.5)
    assert rec == {"world_seen": 1, "ranks_agree": True, "mismatched_params": 0, "step_s_min": 2.5,
                   "step_s_max": 2.5}
