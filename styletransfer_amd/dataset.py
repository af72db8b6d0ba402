"""Datasets (host side; mirror of stransfer/dataset.py without network access).

The reference downloads COCO test2017 and four sample videos on demand
(stransfer/dataset.py:86-139); this environment has no network, so:
  * `CocoDataset` reads whatever images already sit in `data/coco_dataset/images/`
    (same transform as the reference, :141-197) and `get_coco_loader` raises a
    clear error when none are present;
  * `SyntheticImageDataset` provides seeded [3, IMSIZE, IMSIZE] ImageNet-normalised
    images of the COCO batch shape for training smoke runs and benchmarks.
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch
from PIL import Image
from torch.utils.data import DataLoader, Dataset

from . import c_logging, constants, img_utils
from . import weights as W

LOGGER = c_logging.get_logger()

BASE_COCO_PATH = "data/coco_dataset/"
IMAGE_FOLDER_PATH = os.path.join(BASE_COCO_PATH, "images")
VIDEO_DATA_PATH = "data/video/"


class CocoDataset(Dataset):
    """Images under `path` (jpg/png), loaded like stransfer/dataset.py:141-197
    (a corrupt image is replaced by a random other one, as the reference does).
    decode_only=True returns the decoded HxWx3 uint8 array instead of the
    conditioned tensor: the conditioning then runs on the GPU for the whole batch
    (img_utils.ImageConditioner, bit-identical to the PIL path)."""

    def __init__(self, images=None, image_limit=None, path=None, decode_only=False):
        path = path or os.path.join(constants.PROJECT_ROOT_PATH, IMAGE_FOLDER_PATH)
        if images is None:
            images = sorted(f for f in os.listdir(path)
                            if f.lower().endswith((".jpg", ".jpeg", ".png")))
        self.path = path
        self.images = images[:image_limit] if image_limit else images
        self.decode_only = decode_only

    def __len__(self):
        return len(self.images)

    def __getitem__(self, idx):
        try:
            img = Image.open(os.path.join(self.path, self.images[idx]))
            # (convert("RGB") of an RGB image is a full copy: the same pixels without it)
            if img.mode != "RGB":
                img = img.convert("RGB")
            if self.decode_only:
                return np.asarray(img, dtype=np.uint8)
            return img_utils.image_loader_transform(img).cpu()
        except Exception:  # noqa: BLE001  (reference behaviour, :186-197)
            return self[random.randrange(len(self))]


def _list_collate(batch):
    return list(batch)


def _pack_collate(batch):
    """Decoded HxWx3 uint8 images -> (one packed uint8 tensor, int32 [B, 2] shapes):
    runs in the loader's worker, so a batch crosses to the main process as one
    shared-memory tensor (and is pinned there by the DataLoader's pin thread)."""
    arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in batch]
    packed = torch.empty(sum(a.nbytes for a in arrs), dtype=torch.uint8)
    pk = packed.numpy()
    o = 0
    for a in arrs:
        pk[o:o + a.nbytes] = a.reshape(-1)
        o += a.nbytes
    shapes = torch.tensor([a.shape[:2] for a in arrs], dtype=torch.int32).reshape(-1, 2)
    return packed, shapes


def usable_cpus():
    """The CPUs this process may run on: its affinity mask, capped by the cgroup CPU quota
    (on a shared GPU box the box's share, not os.cpu_count())."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def default_workers(local_world=None):
    """Decode workers for the GPU-conditioned loader of ONE rank: the usable CPUs split
    evenly over the ranks of this node (LOCAL_WORLD_SIZE, torchrun's per-node rank count;
    the ranks share the node's CPUs), minus one for the rank's training loop, at most 16."""
    if local_world is None:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    share = usable_cpus() // max(1, local_world)
    return max(0, min(16, share - 1))


class GpuConditionedLoader:
    """Wraps a DataLoader of packed decoded uint8 batches (CocoDataset(decode_only=True),
    _pack_collate; its workers decode the JPEGs) and yields each batch conditioned on
    the GPU as [B, 1, 3, S, S] -- the shape static_train squeezes
    (stransfer/network.py:688).  Pipelined: batch k+depth's upload (pinned -> device)
    and conditioning kernels run on a side stream while the consumer works on batch k;
    the consumer's stream waits on the batch's event, never the host."""

    def __init__(self, loader, size=None, device=None, depth=2):
        self.loader = loader
        self.batch_sampler = getattr(loader, "batch_sampler", None)
        self.cond = img_utils.ImageConditioner(size, device)
        self.depth = max(1, int(depth))

    def __len__(self):
        return len(self.loader)

    def _submit(self, item, side):
        packed, shapes = item
        cond, dev = self.cond, self.cond.device
        metas, coef, max_rows, tmp_bytes, src_bytes = cond._plan(
            [tuple(hw) for hw in shapes.tolist()])
        B, S = shapes.shape[0], cond.size
        if packed.numel() != src_bytes:
            raise ValueError("packed batch size does not match its shapes")
        mb = bytes(metas)
        head = torch.empty(len(mb) + coef.nbytes, dtype=torch.uint8).pin_memory()
        hv = head.numpy()
        hv[:len(mb)] = np.frombuffer(mb, np.uint8)
        hv[len(mb):] = coef.view(np.uint8).reshape(-1)
        with torch.cuda.stream(side):
            src = packed.to(dev, non_blocking=True)
            hd = head.to(dev, non_blocking=True)
            tmp = torch.empty(max(tmp_bytes, 16), dtype=torch.uint8, device=dev)
            out = torch.empty((B, 3, S, S), dtype=torch.float32, device=dev)
            cond._launch(src, hd[:len(mb)], B, max_rows, hd[len(mb):].view(torch.int32), out,
                         tmp)
            ev = torch.cuda.Event()
            ev.record(side)
        return out, ev

    def __iter__(self):
        from collections import deque
        dev = self.cond.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        it = iter(self.loader)
        pending = deque()
        for item in it:
            pending.append(self._submit(item, side))
            if len(pending) >= self.depth:
                break
        while pending:
            out, ev = pending.popleft()
            main = torch.cuda.current_stream(dev)
            main.wait_event(ev)
            out.record_stream(main)
            nxt = next(it, None)
            if nxt is not None:
                pending.append(self._submit(nxt, side))
            yield out.unsqueeze(1)


def _train_loader(ds, batch_size, shard, shuffle=True, seed=0, num_workers=0, collate=None,
                  pin_memory=False, prefetch_factor=None):
    """DataLoader over `ds` whose batches are this rank's shard of each global batch
    of `batch_size` (distributed.ShardedBatchSampler); at world 1 a plain batch."""
    from .distributed import Shard, ShardedBatchSampler
    shard = shard or Shard()
    sampler = ShardedBatchSampler(len(ds), batch_size, shard.rank, shard.world,
                                  shuffle=shuffle, seed=seed)
    kw = {"collate_fn": collate} if collate is not None else {}
    if num_workers > 0:
        kw["persistent_workers"] = True
        if prefetch_factor:
            kw["prefetch_factor"] = prefetch_factor
    return DataLoader(ds, batch_sampler=sampler, num_workers=num_workers, pin_memory=pin_memory,
                      **kw)


def get_coco_loader(batch_size=4, test_split=0.10, test_limit=None, path=None, shard=None,
                    gpu_conditioning=None, num_workers=None):
    """(test_loader, train_loader) over local COCO images (stransfer/dataset.py:314-360).
    `batch_size` is the global batch; with a data-parallel `shard` each rank's train
    loader yields its batch_size/world slice of every global batch.  With
    gpu_conditioning (default: when a GPU is present) the workers only decode (and pack
    the batch), the upload and the crop/resize/normalisation run on the GPU on a side
    stream, pipelined with the consumer (identical output); num_workers defaults to
    default_workers() there and to 0 (the reference's DataLoader) on the PIL path."""
    path = path or os.path.join(constants.PROJECT_ROOT_PATH, IMAGE_FOLDER_PATH)
    if not os.path.isdir(path) or not os.listdir(path):
        raise FileNotFoundError(
            f"No COCO images under {path}. The reference downloads them on demand; this "
            "build has no network access — place images there or use --synthetic.")
    images = sorted(f for f in os.listdir(path) if f.lower().endswith((".jpg", ".jpeg", ".png")))
    n_test = int(len(images) * test_split)
    test_imgs, train_imgs = images[:n_test], images[n_test:]
    if test_limit:
        test_imgs = test_imgs[:test_limit]
    if gpu_conditioning is None:
        gpu_conditioning = constants.DEVICE.type == "cuda"
    if gpu_conditioning:
        nw = default_workers() if num_workers is None else num_workers
        pin = torch.cuda.is_available()
        test = GpuConditionedLoader(DataLoader(CocoDataset(test_imgs, path=path, decode_only=True),
                                               batch_size=batch_size, shuffle=False,
                                               collate_fn=_pack_collate, num_workers=min(nw, 2),
                                               pin_memory=pin))
        train = GpuConditionedLoader(_train_loader(
            CocoDataset(train_imgs, path=path, decode_only=True), batch_size, shard,
            num_workers=nw, collate=_pack_collate, pin_memory=pin,
            prefetch_factor=4 if nw > 0 else None))
        return test, train
    num_workers = num_workers or 0
    test = DataLoader(CocoDataset(test_imgs, path=path), batch_size=batch_size, shuffle=False,
                      num_workers=num_workers)
    train = _train_loader(CocoDataset(train_imgs, path=path), batch_size, shard,
                          num_workers=num_workers)
    return test, train


def write_synthetic_jpegs(path, n, h=480, w=640, seed=0, quality=90):
    """n seeded JPEGs of COCO's typical size (640x480) under `path`: smooth colour
    fields plus sensor-like noise, so the files compress like photographs (~120 KB
    at quality 90) and decode at a photograph's cost.  For loader throughput runs."""
    os.makedirs(path, exist_ok=True)
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    noise = rng.normal(0, 12, (h + 64, w + 64, 3)).astype(np.float32)
    for k in range(n):
        oy, ox = rng.integers(0, 64, 2)
        f = rng.uniform(12, 40, 4)
        base = np.stack([np.sin(x / f[0]) * 60 + np.cos(y / f[1]) * 60 + 128,
                         np.sin((x + y) / f[2]) * 90 + 128,
                         (x * y / (f[3] * 10)) % 255], 2)
        img = np.clip(base + noise[oy:oy + h, ox:ox + w], 0, 255).astype(np.uint8)
        Image.fromarray(img).save(os.path.join(path, f"{k:06d}.jpg"), quality=quality)


class SyntheticImageDataset(Dataset):
    """Seeded uniform RGB images, ImageNet-normalised, [1, 3, S, S] per item (the
    shape `batch.squeeze(1)` expects in static_train, stransfer/network.py:688)."""

    def __init__(self, n=64, size=None, seed=0):
        self.n, self.size, self.seed = n, size or constants.IMSIZE, seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        x = W.synthetic_image(self.seed * 100003 + idx, (1, 3, self.size, self.size))
        return torch.from_numpy(x)


def get_synthetic_loader(batch_size=4, n_train=64, n_test=8, size=None, seed=0, shard=None,
                         shuffle=False):
    """(test, train) loaders of SyntheticImageDataset; train sharded like get_coco_loader."""
    test = DataLoader(SyntheticImageDataset(n_test, size, seed + 1), batch_size=batch_size)
    train = _train_loader(SyntheticImageDataset(n_train, size, seed), batch_size, shard,
                          shuffle=shuffle, seed=seed)
    return test, train


# ------------------------------------------------------------------------------ video
VIDEO_SOURCE_EXTS = (".mp4", ".avi", ".mov", ".mkv", ".gif", ".webm", ".npy")


def make_batches(items, batch_size):
    """Consecutive chunks of `batch_size` (stransfer/dataset.py make_batches)."""
    return [items[i:i + batch_size] for i in range(0, len(items), batch_size)]


class VideoDataset:
    """Batches of videos (stransfer/dataset.py:200-277).  The reference downloads four
    sample videos into data/video/ and opens each with imageio; here every entry of
    data/video/ (or of `videos`) is a video source video.iterate_frames reads: a
    video file (needs imageio), a directory of frame images or a .npy [T, H, W, 3]
    uint8 array (or an in-memory array).  Iterating yields, per batch, one frame
    reader per video; a trailing partial batch is dropped, as the reference does."""

    def __init__(self, videos=None, data_limit=None, batch_size=3, imsize=None,
                 max_frames=90 * 24):
        if videos is None:
            root = os.path.join(constants.PROJECT_ROOT_PATH, VIDEO_DATA_PATH)
            names = sorted(os.listdir(root)) if os.path.isdir(root) else []
            videos = [os.path.join(root, n) for n in names
                      if n.lower().endswith(VIDEO_SOURCE_EXTS) or
                      os.path.isdir(os.path.join(root, n))]
            if not videos:
                raise FileNotFoundError(
                    f"No videos under {root}. The reference downloads its sample videos on "
                    "demand; this build has no network access -- place videos, frame "
                    "directories or .npy frame arrays there.")
        self.videos = list(videos)[:data_limit] if data_limit else list(videos)
        if batch_size > len(self.videos):
            LOGGER.warning("The batch size is larger than the amount of videos in the video "
                           "set. Will use complete set as a batch of size %d", len(self.videos))
            batch_size = len(self.videos)
        self.batch_size = batch_size
        self.imsize, self.max_frames = imsize, max_frames
        self.video_paths = make_batches(self.videos, self.batch_size)
        if self.video_paths and len(self.video_paths[-1]) != self.batch_size:
            self.video_paths = self.video_paths[:-1]

    def __len__(self):
        return len(self.video_paths)

    def __iter__(self):
        from . import video
        for group in self.video_paths:
            yield [video.iterate_frames(v, self.max_frames, self.imsize) for v in group]


def iterate_on_video_batches(batch, max_frames=90 * 24):
    """One [B, 3, H, W] frame batch per time step: frame t of every video in the batch,
    until the shortest video ends (stransfer/dataset.py:280-311)."""
    for _, frames in zip(range(max_frames), zip(*batch)):
        yield torch.cat([f.cpu() for f in frames], dim=0)


def synthetic_video(n_frames=8, size=64, seed=0, shift=1):
    """A [T, size, size, 3] uint8 clip: one seeded image translated by `shift` pixels a
    frame (temporally coherent content for video_train smoke runs and tests)."""
    import numpy as np
    base = W.synthetic_image(seed, (1, 3, size, size + shift * n_frames), normalise=False)[0]
    base = (np.clip(base, 0, 1) * 255).astype(np.uint8).transpose(1, 2, 0)
    return np.stack([base[:, t * shift:t * shift + size] for t in range(n_frames)])
