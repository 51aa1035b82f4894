"""The N>1 path on CPU: two ranks over gloo, DDP-wrapped head (pixel decoder + masked decoder) exactly as
bench.py wraps the model (bench_model.wrap_ddp), HIP ops replaced by the oracle's CPU restatements.
After one step every rank must hold the same gradients, equal to the average of the per-rank gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
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
