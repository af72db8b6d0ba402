"""Image conditioning (stransfer/img_utils.py:13-44: CenterCrop(min side) ->
Resize(IMSIZE) -> ToTensor -> Normalize), SURVEY §8f row 4.

CPU: the numpy oracle of Pillow's 8-bit BILINEAR resampler (oracle/pil_resample.py)
equals PIL.Image.resize byte for byte, and libstx's host-side coefficient builder
(stx_resample_coeffs) equals the oracle's tables.  GPU (-m gpu): the HIP
conditioning kernel (img_utils.ImageConditioner, csrc/image.hip) equals the PIL
path (img_utils.image_loader_transform) bit for bit, image by image and through
the GPU-conditioned COCO loader."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import REPO
from oracle import pil_resample as R

SIZES = [(444, 444, 256), (100, 100, 256), (37, 53, 16), (300, 200, 256), (480, 640, 256),
         (256, 300, 256), (513, 513, 256), (7, 5, 3), (1, 1, 4), (480, 640, 512), (96, 97, 64)]


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("h,w,s", SIZES)
def test_oracle_resize_equals_pil(h, w, s):
    img = _img(h, w, h * 7 + w)
    for ow, oh in ((s, s), (s + 3, max(1, s - 2))):
        want = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
        assert np.array_equal(R.resize_bilinear_u8(img, ow, oh), want), (ow, oh)


def test_oracle_condition_equals_image_loader():
    from styletransfer_amd import constants, img_utils
    for name in ("dancing.jpg", "styles/picasso.jpg"):
        im = Image.open(os.path.join(REPO, "data", name)).convert("RGB")
        want = img_utils.image_loader_transform(im, 256).cpu()[0].numpy()
        got = R.condition(np.asarray(im), 256, constants.IMAGENET_MEAN, constants.IMAGENET_STD)
        assert np.array_equal(got, want), name


@pytest.mark.parametrize("n_in,n_out", [(444, 256), (100, 256), (513, 256), (5, 3), (1, 4),
                                        (4000, 256), (640, 512), (256, 255),
                                        (9000, 256), (20000, 64)])  # ksize > 64
def test_native_coeffs_equal_oracle(n_in, n_out):
    import ctypes as C
    from styletransfer_amd import _native as N
    L = N.lib()
    bounds, kk = R.coeffs(n_in, n_out)
    k = L.stx_resample_coeffs(n_in, n_out, None, None, 0)
    assert k == kk.shape[1]
    b = np.zeros((n_out, 2), np.int32)
    q = np.zeros((n_out, k), np.int32)
    assert L.stx_resample_coeffs(n_in, n_out, b.ctypes.data_as(C.c_void_p),
                                 q.ctypes.data_as(C.c_void_p), k) == k
    assert np.array_equal(b, bounds) and np.array_equal(q, kk)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_gpu_conditioning_equals_pil(dev):
    from styletransfer_amd import img_utils
    imgs = [_img(h, w, i) for i, (h, w, _) in enumerate(SIZES) if min(h, w) >= 3]
    imgs += [np.asarray(Image.open(os.path.join(REPO, "data", n)).convert("RGB"))
             for n in ("dancing.jpg", "styles/picasso.jpg")]
    for size in (256, 64):
        cond = img_utils.ImageConditioner(size, dev)
        got = cond(imgs).cpu()
        want = torch.cat([img_utils.image_loader_transform(Image.fromarray(a), size).cpu()
                          for a in imgs])
        assert got.shape == want.shape
        bad = [i for i in range(len(imgs)) if not torch.equal(got[i], want[i])]
        assert not bad, (size, bad, [imgs[i].shape for i in bad])


@pytest.mark.gpu
def test_gpu_conditioned_coco_loader(dev, tmp_path):
    """get_coco_loader with GPU conditioning == the PIL loader, batch by batch."""
    from styletransfer_amd import dataset
    for i, (h, w) in enumerate([(480, 640), (427, 640), (640, 480), (300, 300), (256, 400),
                                (612, 612), (375, 500), (500, 333)]):
        Image.fromarray(_img(h, w, 100 + i)).save(tmp_path / f"{i:03d}.jpg", quality=90)
    g_test, g_train = dataset.get_coco_loader(batch_size=4, test_split=0.25, path=str(tmp_path),
                                              gpu_conditioning=True)
    c_test, c_train = dataset.get_coco_loader(batch_size=4, test_split=0.25, path=str(tmp_path),
                                              gpu_conditioning=False)
    for a, b in zip(list(g_test) + list(g_train), list(c_test) + list(c_train)):
        assert a.is_cuda and a.shape == b.shape
        assert torch.equal(a.cpu(), b.cpu())
