"""ORACLE — test infrastructure only (never imported by the product path).

numpy restatement of the image conditioning the reference applies to every image
(`stransfer/img_utils.py:13-44`: CenterCrop(min side) -> Resize(IMSIZE) ->
ToTensor -> ImageNet normalisation), with the resize exactly as the pinned image
library computes it: Pillow's convolution resampler for 8-bit images
(`ImagingResample`, BILINEAR = triangle filter, support 1), two separable passes
(horizontal, then vertical) with fixed-point coefficients:

  * per output index: scale = in/out, filterscale = max(scale, 1),
    support = filterscale, center = (x + 0.5) * scale,
    taps xmin = max(int(center - support + 0.5), 0) ..
         xmax = min(int(center + support + 0.5), in) (exclusive),
    w_k = triangle((xmin + k - center + 0.5) / filterscale), normalised to sum 1;
  * coefficients to int32 with 22 fractional bits, rounded half away from zero;
  * each pass: acc = 2^21 + sum(u8 * coeff), out = clip(acc >> 22, 0, 255).

The vertical pass only runs over the rows the vertical kernel needs, on the
horizontally resampled uint8 rows (Pillow keeps the intermediate image 8-bit).

Pinned in tests/test_image_pipeline.py: equal, byte for byte, to PIL.Image.resize
(Pillow in this image) on random and real images of many sizes; the GPU kernel
(stx_image_condition) is then held to this oracle and to PIL directly.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _triangle(x: float) -> float:
    x = -x if x < 0 else x
    return 1.0 - x if x < 1.0 else 0.0


def coeffs(in_size: int, out_size: int):
    """(bounds [out, 2] = (xmin, n), int32 coefficients [out, ksize]) for one axis."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_triangle((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(0.5 + k * (1 << PRECISION_BITS)) if k >= 0 else \
                int(-0.5 + k * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _pass(img: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One 8-bit resampling pass along `axis` (0 rows, 1 columns) of an HxWxC image."""
    src = np.moveaxis(img, axis, 0).astype(np.int64)
    out = np.empty((len(bounds),) + src.shape[1:], np.uint8)
    for o, (xmin, n) in enumerate(bounds):
        acc = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for k in range(n):
            acc += src[xmin + k] * int(kk[o, k])
        out[o] = np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)
    return np.moveaxis(out, 0, axis)


def resize_bilinear_u8(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """PIL Image.resize((out_w, out_h), BILINEAR) of an HxWx3 uint8 image."""
    h, w = img.shape[:2]
    if (w, h) == (out_w, out_h):
        return img.copy()
    ybounds, ykk = coeffs(h, out_h)
    if w != out_w:
        # the horizontal pass covers only the rows the vertical pass reads
        if h != out_h:
            y0 = int(ybounds[0, 0])
            y1 = int(ybounds[-1, 0] + ybounds[-1, 1])
        else:
            y0, y1 = 0, h
        xb, xk = coeffs(w, out_w)
        tmp = _pass(img[y0:y1], xb, xk, axis=1)
        ybounds = ybounds.copy()
        ybounds[:, 0] -= y0
    else:
        tmp = img
    if h != out_h:
        return _pass(tmp, ybounds, ykk, axis=0)
    return tmp


def center_crop_box(w: int, h: int, size: int):
    """torchvision 0.3 CenterCrop offsets (round half to even, as python round)."""
    top = int(round((h - size) / 2.0))
    left = int(round((w - size) / 2.0))
    return left, top


def resize_shape(w: int, h: int, size: int):
    """torchvision 0.3 Resize(int) output (w, h): shorter side -> size."""
    if (w <= h and w == size) or (h <= w and h == size):
        return w, h
    if w < h:
        return size, int(size * h / w)
    return int(size * w / h), size


def condition(img: np.ndarray, size: int, mean, std) -> np.ndarray:
    """image_loader_transform on an HxWx3 uint8 image -> [3, size, size] float32."""
    h, w = img.shape[:2]
    m = min(w, h)
    left, top = center_crop_box(w, h, m)
    crop = img[top:top + m, left:left + m]
    ow, oh = resize_shape(m, m, size)
    r = resize_bilinear_u8(crop, ow, oh)
    t = r.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    mean = np.asarray(mean, np.float32).reshape(3, 1, 1)
    std = np.asarray(std, np.float32).reshape(3, 1, 1)
    return ((t - mean) / std).astype(np.float32)
