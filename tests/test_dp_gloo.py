"""Data-parallel fast_st on CPU with the gloo backend (world_size 2): the
flat-gradient SUM all-reduce with the mean/W + sum scaling of train.py gives the
single-device full-batch gradient (SURVEY.md §8e TV-sum trap).  The loss here is
a CPU stand-in with the same structure (batch-mean terms + a batch-sum term);
the HIP kernels themselves are covered by tests/test_parity_gpu.py."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _loss(params, batch, world):
    w, b = params
    y = torch.tanh(batch @ w + b)               # "transform net"
    mean_terms = 1e5 * (y ** 2).mean() + (y - batch[:, :3]).pow(2).mean()
    tv_sum = 1e-6 * (y[:, 1:] - y[:, :-1]).abs().sum()
    return mean_terms / world + tv_sum


def _flat_grad(params):
    return torch.cat([p.grad.reshape(-1) for p in params])


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(0)
    w = torch.randn(8, 3, generator=g).requires_grad_()
    b = torch.randn(3, generator=g).requires_grad_()
    batch = torch.randn(16, 8, generator=g)
    shard = batch.chunk(world)[rank]
    _loss((w, b), shard, world).backward()
    flat = _flat_grad((w, b))
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    if rank == 0:
        w2, b2 = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
        _loss((w2, b2), batch, 1).backward()
        q.put(float((flat - _flat_grad((w2, b2))).norm() / _flat_grad((w2, b2)).norm()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_allreduce_scaling_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    err = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert err < 1e-6
