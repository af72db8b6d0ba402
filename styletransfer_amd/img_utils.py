"""Image loading/saving (mirror of stransfer/img_utils.py, host-side PIL code).

torchvision is not part of this stack; the transforms the reference composes
(stransfer/img_utils.py:20-27: CenterCrop(min side) -> Resize(IMSIZE) ->
ToTensor) are restated on PIL with torchvision 0.3 semantics (the reference's
pin): round-half centre crop offsets, bilinear resize of the shorter side,
uint8/255 tensors; ImageNet normalisation as :32-42; `imshow` de-normalises,
clamps to [0, 255] (sic) and converts with mul(255).byte() (:95-117)."""
from __future__ import annotations

import numpy as np
import torch
from PIL import Image

from . import constants


def _center_crop(img: Image.Image, size: int) -> Image.Image:
    w, h = img.size
    top = int(round((h - size) / 2.0))
    left = int(round((w - size) / 2.0))
    return img.crop((left, top, left + size, top + size))


def _resize(img: Image.Image, size: int) -> Image.Image:
    w, h = img.size
    if (w <= h and w == size) or (h <= w and h == size):
        return img
    if w < h:
        ow, oh = size, int(size * h / w)
    else:
        oh, ow = size, int(size * w / h)
    return img.resize((ow, oh), Image.BILINEAR)


def _to_tensor(img: Image.Image) -> torch.Tensor:
    a = np.asarray(img.convert("RGB"), dtype=np.uint8)
    return torch.from_numpy(a.copy()).permute(2, 0, 1).float().div(255)


def image_loader_transform(image: Image.Image, imsize: int | None = None) -> torch.Tensor:
    """PIL image -> normalised [1, 3, IMSIZE, IMSIZE] tensor on DEVICE."""
    imsize = constants.IMSIZE if imsize is None else imsize
    min_dimension = min(image.size)
    t = _to_tensor(_resize(_center_crop(image, min_dimension), imsize)).unsqueeze(0)
    mean = torch.tensor(constants.IMAGENET_MEAN).view(-1, 1, 1)
    std = torch.tensor(constants.IMAGENET_STD).view(-1, 1, 1)
    return ((t - mean) / std).to(constants.DEVICE, torch.float)


def concat_images(im1, im2, dim=2) -> torch.Tensor:
    return torch.cat([im1, im2], dim=dim)


def image_loader(image_path: str, imsize: int | None = None) -> torch.Tensor:
    return image_loader_transform(Image.open(image_path), imsize)


def to_pil(image_tensor: torch.Tensor, denormalize=True) -> Image.Image:
    """The byte conversion of `imshow`, returned instead of saved."""
    t = image_tensor.detach().cpu()
    if denormalize:
        mean = torch.tensor(constants.IMAGENET_MEAN).view(-1, 1, 1)
        std = torch.tensor(constants.IMAGENET_STD).view(-1, 1, 1)
        t = (t * std) + mean
    t = torch.clamp(t.clone(), min=0, max=255).squeeze(0)
    a = t.mul(255).byte().permute(1, 2, 0).numpy()
    return Image.fromarray(a, mode="RGB")


def imshow(image_tensor: torch.Tensor, ground_truth_image: torch.Tensor = None,
           denormalize=True, path="out.bmp") -> None:
    if ground_truth_image is not None:
        image_tensor = concat_images(image_tensor, ground_truth_image)
    to_pil(image_tensor, denormalize).save(path)
