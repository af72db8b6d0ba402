"""Image loading/saving (mirror of stransfer/img_utils.py, host-side PIL code).

torchvision is not part of this stack; the transforms the reference composes
(stransfer/img_utils.py:20-27: CenterCrop(min side) -> Resize(IMSIZE) ->
ToTensor) are restated on PIL with torchvision 0.3 semantics (the reference's
pin): round-half centre crop offsets, bilinear resize of the shorter side,
uint8/255 tensors; ImageNet normalisation as :32-42; `imshow` de-normalises,
clamps to [0, 255] (sic) and converts with mul(255).byte() (:95-117)."""
from __future__ import annotations

import ctypes as C

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


# ------------------------------------------------------------------ GPU conditioning
class ImageConditioner:
    """image_loader_transform for a batch of decoded images on the GPU
    (csrc/image.hip, stx_image_condition): centre crop -> Pillow-exact BILINEAR
    resize -> /255 -> ImageNet normalisation, bit-identical to the PIL path above
    (tests/test_image_pipeline.py).  Host work per batch is the JPEG decode (done by
    the loader's workers) and one copy of the packed uint8 images, so COCO-rate
    training input does not bottleneck on PIL's resize."""

    def __init__(self, size: int | None = None, device=None):
        self.size = int(size or constants.IMSIZE)
        self.device = torch.device(device) if device is not None else constants.DEVICE
        self._tables = {}  # crop side -> (int32 table, ksize, y0, y1)
        mean = np.asarray(constants.IMAGENET_MEAN, np.float32)
        std = np.asarray(constants.IMAGENET_STD, np.float32)
        self._mean = (C.c_float * 3)(*mean.tolist())
        self._std = (C.c_float * 3)(*std.tolist())

    def _table(self, m: int):
        t = self._tables.get(m)
        if t is None:
            from ._native import lib
            L, S = lib(), self.size
            k = L.stx_resample_coeffs(m, S, None, None, 0)
            bounds = np.zeros((S, 2), np.int32)
            kk = np.zeros((S, k), np.int32)
            if L.stx_resample_coeffs(m, S, bounds.ctypes.data, kk.ctypes.data, k) != k:
                raise RuntimeError("stx_resample_coeffs failed")
            y0, y1 = int(bounds[0, 0]), int(bounds[-1, 0] + bounds[-1, 1])
            t = self._tables[m] = (np.concatenate([bounds.ravel(), kk.ravel()]), k, y0, y1)
        return t

    def _plan(self, shapes):
        """Per-image metadata, the coefficient tables and workspace sizes of a batch of
        HxW images: (metas, coef int32 array, max_rows, tmp bytes, src bytes)."""
        from ._native import ImageMeta
        B, S = len(shapes), self.size
        metas = (ImageMeta * B)()
        tables, coef_off, chunks, max_rows = {}, 0, [], 0
        src_off, tmp_off = 0, 0
        for i, (h, w) in enumerate(shapes):
            m = min(h, w)
            top, left = int(round((h - m) / 2.0)), int(round((w - m) / 2.0))
            md = metas[i]
            md.offset, md.h, md.w, md.top, md.left = src_off, h, w, top, left
            src_off += h * w * 3
            if m == S:  # torchvision Resize is a no-op at the target size
                md.y0, md.y1, md.resize_w, md.resize_h = 0, m, 0, 0
            else:
                if m not in tables:
                    tab, k, y0, y1 = self._table(m)
                    tables[m] = (coef_off, k, y0, y1)
                    chunks.append(tab)
                    coef_off += tab.size
                off, k, y0, y1 = tables[m]
                md.y0, md.y1, md.resize_w, md.resize_h = y0, y1, 1, 1
                md.xcoef = md.ycoef = off
                md.xk = md.yk = k
                md.tmp_offset = tmp_off
                tmp_off += (y1 - y0) * S * 3
                max_rows = max(max_rows, y1 - y0)
        coef = np.concatenate(chunks) if chunks else np.zeros(1, np.int32)
        return metas, coef, max_rows, tmp_off, src_off

    def _launch(self, src, meta, b, max_rows, coef, out, tmp):
        from ._native import check, lib
        check(lib().stx_image_condition(src.data_ptr(), meta.data_ptr(), b, max_rows,
                                        coef.data_ptr(), self.size, self._mean, self._std,
                                        out.data_ptr(), tmp.data_ptr(), tmp.numel(),
                                        torch.cuda.current_stream(self.device).cuda_stream),
              "stx_image_condition")

    def __call__(self, images) -> torch.Tensor:
        """images: sequence of HxWx3 uint8 arrays (or PIL images) -> [B, 3, S, S]."""
        arrs = [np.ascontiguousarray(np.asarray(im.convert("RGB") if isinstance(im, Image.Image)
                                                else im, dtype=np.uint8)) for im in images]
        B, S = len(arrs), self.size
        if B == 0:
            raise ValueError("empty image batch")
        for i, a in enumerate(arrs):
            if a.ndim != 3 or a.shape[2] != 3:
                raise ValueError(f"image {i}: HxWx3 uint8 expected, got {a.shape}")
        metas, coef, max_rows, tmp_bytes, src_bytes = self._plan([a.shape[:2] for a in arrs])
        dev = self.device
        packed = torch.empty(src_bytes, dtype=torch.uint8, pin_memory=True)
        pk = packed.numpy()
        o = 0
        for a in arrs:
            pk[o:o + a.nbytes] = a.reshape(-1)
            o += a.nbytes
        src = packed.to(dev, non_blocking=True)
        meta = torch.frombuffer(bytearray(bytes(metas)), dtype=torch.uint8).to(dev)
        coef = torch.from_numpy(coef).to(dev)
        tmp = torch.empty(max(tmp_bytes, 16), dtype=torch.uint8, device=dev)
        out = torch.empty((B, 3, S, S), dtype=torch.float32, device=dev)
        self._launch(src, meta, B, max_rows, coef, out, tmp)
        return out

    def fixed(self, h: int, w: int, out: torch.Tensor | None = None) -> "FixedConditioner":
        """A conditioner for a stream of HxW frames with static buffers (video_st)."""
        return FixedConditioner(self, h, w, out)


class FixedConditioner:
    """image_loader_transform of a stream of same-size frames (video_st: every decoded
    frame of a clip, stransfer/dataset.py:280-306) with everything static: the
    coefficient tables and metadata are uploaded once, the frame's bytes go into a
    device buffer `src` ([H][W][3] uint8) and the [1, 3, S, S] result into `out` (which
    may be a view into a caller's buffer, e.g. FrameEngine's 6-channel input).  `run()`
    is two kernel launches and no allocation or host transfer, so a hipGraph can
    capture it."""

    def __init__(self, cond: ImageConditioner, h: int, w: int, out: torch.Tensor | None = None):
        self.cond, self.h, self.w = cond, int(h), int(w)
        dev, S = cond.device, cond.size
        metas, coef, self.max_rows, tmp_bytes, src_bytes = cond._plan([(self.h, self.w)])
        self.meta = torch.frombuffer(bytearray(bytes(metas)), dtype=torch.uint8).to(dev)
        self.coef = torch.from_numpy(coef).to(dev)
        self.tmp = torch.empty(max(tmp_bytes, 16), dtype=torch.uint8, device=dev)
        self.src = torch.empty((self.h, self.w, 3), dtype=torch.uint8, device=dev)
        if out is None:
            out = torch.empty((1, 3, S, S), dtype=torch.float32, device=dev)
        if tuple(out.shape) != (1, 3, S, S) or not out.is_contiguous() or \
                out.dtype != torch.float32 or out.device != self.src.device:
            raise ValueError(f"out must be a contiguous fp32 [1, 3, {S}, {S}] device tensor")
        self.out = out

    def load(self, frame) -> None:
        """Copy one HxWx3 uint8 frame (numpy array or tensor, host or device) into src."""
        t = frame if isinstance(frame, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frame))
        if tuple(t.shape) != (self.h, self.w, 3) or t.dtype != torch.uint8:
            raise ValueError(f"frame must be uint8 [{self.h}, {self.w}, 3], got {tuple(t.shape)}")
        self.src.copy_(t, non_blocking=True)

    def run(self) -> torch.Tensor:
        self.cond._launch(self.src, self.meta, 1, self.max_rows, self.coef, self.out, self.tmp)
        return self.out
