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


# ------------------------------------------------------------ static_train's sharding
def test_sharded_batch_sampler_partitions_global_batches():
    from styletransfer_amd.distributed import ShardedBatchSampler
    n, B, world = 23, 8, 4
    ref = ShardedBatchSampler(n, B, 0, 1, shuffle=True, seed=3, drop_last=True)
    shards = [ShardedBatchSampler(n, B, r, world, shuffle=True, seed=3) for r in range(world)]
    for epoch in (0, 1):
        for s in shards + [ref]:
            s.set_epoch(epoch)
        glob = list(ref)
        per = [list(s) for s in shards]
        assert len(glob) == n // B and all(len(p) == len(glob) for p in per)
        for k, g in enumerate(glob):
            assert sum((p[k] for p in per), []) == g  # rank slices tile the global batch
    e0 = list(ShardedBatchSampler(n, B, 0, 1, seed=3))
    s1 = ShardedBatchSampler(n, B, 0, 1, seed=3)
    s1.set_epoch(1)
    assert e0 != list(s1)                          # reshuffled per epoch
    # world 1 keeps the partial tail batch (the reference DataLoader does)
    assert [len(b) for b in ShardedBatchSampler(n, B, shuffle=False)] == [8, 8, 7]
    import pytest
    with pytest.raises(ValueError):
        ShardedBatchSampler(n, 6, 0, 4)


def _loader_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from styletransfer_amd import dataset
    from styletransfer_amd import distributed as D
    shard = D.from_env()                          # no GPU here: gloo
    assert (shard.rank, shard.world) == (rank, world)
    _, train = dataset.get_synthetic_loader(4, n_train=10, size=8, shard=shard)
    mine = torch.cat([b for b in train])         # this rank's images, in step order
    got = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(got, mine)
    t = torch.ones(1) * (rank + 1)
    shard.sum_(t)
    if rank == 0:
        _, full = dataset.get_synthetic_loader(4, n_train=10, size=8)
        full = [b for b in full][:2]             # world 2 drops the partial tail
        steps = [torch.cat([g[2 * k:2 * k + 2] for g in got]) for k in range(2)]
        q.put((all(torch.equal(a, b) for a, b in zip(steps, full)), float(t)))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_loaders_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loader_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    same, total = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert same and total == 3.0
