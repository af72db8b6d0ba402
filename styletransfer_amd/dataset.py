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
    (a corrupt image is replaced by a random other one, as the reference does)."""

    def __init__(self, images=None, image_limit=None, path=None):
        path = path or os.path.join(constants.PROJECT_ROOT_PATH, IMAGE_FOLDER_PATH)
        if images is None:
            images = sorted(f for f in os.listdir(path)
                            if f.lower().endswith((".jpg", ".jpeg", ".png")))
        self.path = path
        self.images = images[:image_limit] if image_limit else images

    def __len__(self):
        return len(self.images)

    def __getitem__(self, idx):
        try:
            img = Image.open(os.path.join(self.path, self.images[idx]))
            return img_utils.image_loader_transform(img.convert("RGB")).cpu()
        except Exception:  # noqa: BLE001  (reference behaviour, :186-197)
            return self[random.randrange(len(self))]


def _train_loader(ds, batch_size, shard, shuffle=True, seed=0):
    """DataLoader over `ds` whose batches are this rank's shard of each global batch
    of `batch_size` (distributed.ShardedBatchSampler); at world 1 a plain batch."""
    from .distributed import Shard, ShardedBatchSampler
    shard = shard or Shard()
    sampler = ShardedBatchSampler(len(ds), batch_size, shard.rank, shard.world,
                                  shuffle=shuffle, seed=seed)
    return DataLoader(ds, batch_sampler=sampler)


def get_coco_loader(batch_size=4, test_split=0.10, test_limit=None, path=None, shard=None):
    """(test_loader, train_loader) over local COCO images (stransfer/dataset.py:314-360).
    `batch_size` is the global batch; with a data-parallel `shard` each rank's train
    loader yields its batch_size/world slice of every global batch."""
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
    test = DataLoader(CocoDataset(test_imgs, path=path), batch_size=batch_size, shuffle=False)
    train = _train_loader(CocoDataset(train_imgs, path=path), batch_size, shard)
    return test, train


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
