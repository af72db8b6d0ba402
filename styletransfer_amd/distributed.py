"""Process-group plumbing for data-parallel fast_st training.

The reference is single-device (no torch.distributed anywhere);
north_star asks for `fast_st` training to shard COCO image batches across the
GPUs of one node with an RCCL all-reduce of the ImageTransformNet gradients.
The arrangement is one process per GPU (`torchrun --nproc-per-node N`), each
process owning `cuda:LOCAL_RANK`:

  * every rank reads a disjoint shard of each global batch (ShardedBatchSampler:
    global batch k = indices perm[k*B : (k+1)*B], rank r takes the r-th
    contiguous slice of B/W), so the W shards together are exactly the batch a
    single device would see;
  * parameters start identical (broadcast from rank 0, FastStTrainer) and the
    replicated Adam keeps them identical;
  * the only collective on the data path is one SUM all-reduce of the flat
    gradient per step (train.FastStTrainer._exchange); logging, the test-set
    evaluation and checkpoint writes happen on rank 0.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist
from torch.utils.data import Sampler


@dataclass
class Shard:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    group: object = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    def sum_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM over ranks (no-op at world 1)."""
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t


def from_env(backend: str | None = None) -> Shard:
    """The current data-parallel arrangement.

    An initialised default process group is used as is.  Otherwise, when the
    launcher set WORLD_SIZE > 1 (torchrun), the group is created here: backend
    "nccl" (= RCCL on ROCm) with the rank's GPU bound, or $STX_DIST_BACKEND
    (e.g. "gloo").  Without either it is a single-rank Shard."""
    if dist.is_available() and dist.is_initialized():
        return Shard(dist.get_rank(), dist.get_world_size(),
                     int(os.environ.get("LOCAL_RANK", dist.get_rank())), None)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return Shard()
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    backend = backend or os.environ.get("STX_DIST_BACKEND") or (
        "nccl" if torch.cuda.device_count() > 0 else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        if torch.cuda.device_count() > 0:
            torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend)
    return Shard(rank, world, local, None)


def device_for(shard: Shard) -> torch.device:
    """cuda:LOCAL_RANK (one process per GPU)."""
    n = torch.cuda.device_count()
    if n > 0:
        return torch.device("cuda", shard.local_rank % max(n, 1))
    return torch.device("cpu")


class ShardedBatchSampler(Sampler):
    """Per-rank batches of one global batch sequence.

    Global batch k (of size `global_batch`) is perm[k*B:(k+1)*B] where perm is a
    seeded permutation of range(n) (identity when shuffle=False) re-drawn per
    epoch (`set_epoch`); rank r yields the r-th contiguous slice of B/W indices.
    A trailing partial global batch is dropped when world > 1 (every rank must
    take part in every all-reduce with an equal shard) and kept at world 1 (the
    reference's DataLoader keeps it, stransfer/dataset.py:344-358)."""

    def __init__(self, n: int, global_batch: int, rank: int = 0, world: int = 1,
                 shuffle: bool = True, seed: int = 0, drop_last: bool | None = None):
        if global_batch % world:
            raise ValueError(f"global batch {global_batch} is not divisible by the "
                             f"{world} data-parallel ranks")
        self.n, self.B, self.rank, self.world = int(n), int(global_batch), int(rank), int(world)
        self.shuffle, self.seed, self.epoch = shuffle, int(seed), 0
        self.drop_last = (world > 1) if drop_last is None else drop_last
        self.b = self.B // self.world

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def _perm(self):
        if not self.shuffle:
            return list(range(self.n))
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + self.epoch)
        return torch.randperm(self.n, generator=g).tolist()

    def __len__(self):
        full = self.n // self.B
        if not self.drop_last and self.n % self.B:
            return full + 1
        return full

    def __iter__(self):
        perm = self._perm()
        for k in range(len(self)):
            glob = perm[k * self.B:(k + 1) * self.B]
            if len(glob) < self.B:  # partial tail (world 1 only)
                yield glob
                continue
            yield glob[self.rank * self.b:(self.rank + 1) * self.b]
