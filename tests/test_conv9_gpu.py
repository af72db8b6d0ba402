"""The ImageTransformNet's 9x9 layers on the split MFMA (conv9.hip) vs fp64.

conv0 forward (3 -> 32), conv22 forward (32 -> 3) and conv22's data gradient
(3 -> 32 over the transposed, flipped slab) -- stransfer/network.py:525-527, :607-609.
Held to 2e-6 of fp64 like every split kernel (fp32 summation alone is ~1e-7), over
ragged tiles (the 32 -> 3 tile is 56 output columns wide), ReLU input, bias /
relu_out / accumulate / out_amax epilogues, channel counts that are not chunk
multiples, and block-local scales across a 1e4 dynamic-range step."""
import pytest
import torch
import torch.nn.functional as F

from styletransfer_amd import _native as N
from styletransfer_amd import ops

pytestmark = pytest.mark.gpu
TOL64 = 2e-6


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def rnd(*shape, dev, seed=0, scale=1.0, shift=0.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g) * scale + shift).to(dev)


def ref_conv(x, wgt, b, relu_in=False):
    x = x.double().cpu()
    if relu_in:
        x = F.relu(x)
    return F.conv2d(x, wgt.double().cpu(), None if b is None else b.double().cpu(), padding=4)


@pytest.mark.parametrize("case", [
    # n, cin, cout, h, w, relu_in
    (2, 32, 3, 24, 20, False),
    (1, 32, 3, 37, 131, True),     # ragged rows and a 56-column tile past the edge
    (2, 20, 3, 16, 56, False),     # channels not a multiple of 16, exact tile width
    (1, 64, 2, 9, 113, False),
    (3, 8, 1, 5, 7, True),         # smaller than one tile
    (1, 32, 3, 256, 256, True),    # the ITN shape
])
def test_conv9_out3_fwd(dev, case):
    n, cin, cout, h, w, relu_in = case
    mode = N.STX_IN_RELU if relu_in else N.STX_IN_RAW
    x = rnd(n, cin, h, w, dev=dev, seed=1, scale=2, shift=-1)
    wgt = rnd(cout, cin, 9, 9, dev=dev, seed=2, scale=0.2, shift=-0.1)
    b = rnd(cout, dev=dev, seed=3)
    wt = ops.conv_weight_prep(wgt)
    am = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
    # the split kernel takes the producer's max|x| bound (an exact one, then a loose one)
    y = ops.conv2d(x, wt, cin, cout, 9, in_mode=mode, bias=b, out_amax=am, in_amax=ops.amax(x))
    ref = ref_conv(x, wgt, b, relu_in)
    y_loose = ops.conv2d(x, wt, cin, cout, 9, in_mode=mode, bias=b,
                         in_amax=ops.amax(x) * 37.0)
    assert rel(y_loose, ref) < TOL64
    torch.cuda.synchronize()
    assert y.shape == ref.shape
    assert rel(y, ref) < TOL64
    assert float(am.max()) == float(y.abs().max())
    old = rnd(n, cout, h, w, dev=dev, seed=4)
    out = old.clone()
    ops.conv2d(x, wt, cin, cout, 9, in_mode=mode, bias=b, out=out, accumulate=True,
               relu_out=True, in_amax=ops.amax(x))
    assert rel(out, F.relu(ref + old.double().cpu())) < TOL64


@pytest.mark.parametrize("case", [(2, 32, 24, 20, False), (1, 32, 37, 131, True),
                                  (3, 17, 5, 7, False), (8, 32, 256, 256, False)])
def test_conv9_in3_fwd(dev, case):
    """3 -> cout 9x9 (ITN conv0), ReLU input, relu_out, out_amax; a half-zero /
    half-1e4 input checks the block-local scales."""
    n, cout, h, w, relu_in = case
    mode = N.STX_IN_RELU if relu_in else N.STX_IN_RAW
    x = rnd(n, 3, h, w, dev=dev, seed=5, scale=2, shift=-1)
    wgt = rnd(cout, 3, 9, 9, dev=dev, seed=6, scale=0.2, shift=-0.1)
    b = rnd(cout, dev=dev, seed=7)
    wt = ops.conv_weight_prep(wgt)
    am = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
    y = ops.conv2d(x, wt, 3, cout, 9, in_mode=mode, bias=b, out_amax=am, relu_out=True)
    if n * h * w > 100_000:  # the ITN shape: against the fp32 reference on the GPU
        ref = F.relu(F.conv2d(F.relu(x) if relu_in else x, wgt, b, padding=4))
        assert rel(y, ref) < 1e-5
    else:
        ref = F.relu(ref_conv(x, wgt, b, relu_in))
        assert rel(y, ref) < TOL64
    torch.cuda.synchronize()
    assert float(am.max()) == float(y.abs().max())
    x2 = x.clone()
    x2[..., : w // 2] = 0
    x2[..., w // 2:] *= 1e4
    y2 = ops.conv2d(x2, wt, 3, cout, 9, in_mode=mode, bias=b)
    if n * h * w <= 100_000:
        assert rel(y2, ref_conv(x2, wgt, b, relu_in)) < TOL64


@pytest.mark.parametrize("case", [(2, 32, 24, 20), (1, 32, 37, 131), (2, 32, 64, 64)])
def test_conv9_dgrad(dev, case):
    """conv22's data gradient: dy (3 channels) through the transposed, flipped slab."""
    n, cin, h, w = case
    x = rnd(n, cin, h, w, dev=dev, seed=8, scale=2, shift=-1).double().cpu().requires_grad_()
    wgt = rnd(3, cin, 9, 9, dev=dev, seed=9, scale=0.2, shift=-0.1)
    y = F.conv2d(x, wgt.double().cpu(), padding=4)
    dy = rnd(*y.shape, dev=dev, seed=10, scale=2e-3, shift=-1e-3)
    (ref,) = torch.autograd.grad(y, x, dy.double().cpu())
    wtT = ops.conv_weight_prep(wgt, transpose=True)
    dx = ops.conv2d(dy, wtT, 3, cin, 9)
    assert rel(dx, ref) < TOL64
