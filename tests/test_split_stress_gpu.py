"""fp16 hi/lo split MFMA under realistic dynamic range (VERDICT r1 "split-precision
robustness"): channels whose magnitudes span 1e-6 ... 1e3, and weights with
outliers, against fp64 -- per channel, next to plain fp32 on the same inputs.

Error model of the split.  A tensor is scaled by one power of two
s = 2^(15 - e) (max|v| < 2^e) and each element split as s*v = hi + lo + err with
|err| <= 2^-24 |s v| + 2^-25 (the last term: fp16's subnormal spacing), i.e. in the
original units |err| <= 2^-24 |v| + 2^-39 max|v| (max|v| >= 2^(e-1)) -- a floor set
by the TENSOR's max.  A product keeps hi*hi + hi*lo + lo*hi, dropping
lo*lo <= 2^-22 |a b|.  So for a dot product of rows a, b (length N):

    |err| <= 2^-21 ||a|| ||b|| + 2^-39 max|v| sqrt(N) (||a|| + ||b||)
             + fp32 accumulation (~ sqrt(N) 2^-24 ||a|| ||b||, as plain fp32)

-- relative accuracy for every channel within ~1e-5 of the tensor max (fp32-class),
and, far below it, an absolute error floor: such channels lose relative precision
(a 1e-9-of-max channel keeps ~3 bits).  The tests assert the bound element-wise
(with a 4x margin) and print the per-channel relative errors of the split path and
of fp32.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from styletransfer_amd import ops

pytestmark = pytest.mark.gpu


def _decades(c, lo=-6, hi=3):
    """Per-channel magnitudes spanning 10^lo ... 10^hi (log-uniform over channels)."""
    return torch.logspace(lo, hi, c, dtype=torch.float64)


def _field(shape, seed, mags):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(*shape, generator=g, dtype=torch.float64)
    return x * mags.view(1, -1, 1, 1)


@pytest.mark.parametrize("c,h,w", [(64, 64, 64), (128, 32, 32), (256, 16, 16)])
def test_split_gram_dynamic_range(dev, c, h, w):
    z64 = _field((1, c, h, w), 7, _decades(c))
    z = z64.float()
    zd = z.double()                                   # the fp32 input is the truth's input
    n = h * w
    f = zd.reshape(c, n)
    ref = (f @ f.T) / (c * n)
    g16 = ops.gram(z.to(dev), z_amax=ops.amax(z.to(dev)))[0].double().cpu()
    g32 = ((z.reshape(c, n) @ z.reshape(c, n).T) / (c * n)).double()  # plain fp32 (CPU)
    nrm = f.norm(dim=1)
    amax = float(zd.abs().max())
    rmax = f.abs().max(dim=1).values
    # split terms + fp32 accumulation (module docstring)
    outer = nrm[:, None] * nrm[None, :]
    bound = ((2.0 ** -21 + np.sqrt(n) * 2.0 ** -24) * outer
             + 2.0 ** -39 * amax * np.sqrt(n) * (nrm[:, None] + nrm[None, :])) / (c * n)
    err = (g16 - ref).abs()
    assert bool((err <= 4.0 * bound).all()), float((err / bound).max())
    d16 = (torch.diagonal(g16) - torch.diagonal(ref)).abs() / torch.diagonal(ref)
    d32 = (torch.diagonal(g32) - torch.diagonal(ref)).abs() / torch.diagonal(ref)
    big = rmax >= 1e-5 * amax
    print(f"\nGram C={c}: per-channel diag rel err, channels >= 1e-5 max: split "
          f"{float(d16[big].max()):.1e} fp32 {float(d32[big].max()):.1e}; below: split "
          f"{float(d16[~big].max()) if (~big).any() else 0:.1e} fp32 "
          f"{float(d32[~big].max()) if (~big).any() else 0:.1e}")
    assert float(d16[big].max()) <= 2e-6


def test_split_conv_dynamic_range_and_weight_outliers(dev):
    """3x3 conv (the split kernel's VGG/ITN shapes) with input channels over 9 decades
    and 1 % of the weights 1e4x larger than the rest."""
    cin, cout, h, w = 64, 64, 48, 48
    x64 = _field((1, cin, h, w), 11, _decades(cin))
    g = torch.Generator().manual_seed(12)
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * 0.01
    out = torch.rand(wt.shape, generator=g) < 0.01
    wt[out] *= 1e4
    x, wf = x64.float(), wt.float()
    ref = F.conv2d(x.double(), wf.double(), padding=1)
    y32 = F.conv2d(x, wf, padding=1).double()
    w16 = ops.conv_weight_prep16(wf.to(dev))
    y16 = ops.conv2d(x.to(dev), None, cin, cout, 3, wt16=w16, in_amax=ops.amax(x.to(dev)))
    y16 = y16.double().cpu()
    # element-wise bound: |w| * |x| products (2^-21 relative) + each tensor's floor
    aw, ax = wf.double().abs(), x.double().abs()
    mag = F.conv2d(ax, aw, padding=1)
    floor = (2.0 ** -39) * (float(ax.max()) * F.conv2d(torch.ones_like(ax), aw, padding=1)
                            + float(aw.max()) * F.conv2d(ax, torch.ones_like(aw), padding=1))
    bound = (2.0 ** -21 + 2.0 ** -22 * 3 * cin ** 0.5) * mag + floor  # + fp32 accumulation
    err = (y16 - ref).abs()
    assert bool((err <= 4.0 * bound).all()), float((err / bound).max())
    e16 = (y16 - ref).norm(dim=(2, 3)) / ref.norm(dim=(2, 3))
    e32 = (y32 - ref).norm(dim=(2, 3)) / ref.norm(dim=(2, 3))
    print(f"\nconv per-output-channel rel err: split max {float(e16.max()):.1e} median "
          f"{float(e16.median()):.1e}; fp32 max {float(e32.max()):.1e} median "
          f"{float(e32.median()):.1e}")
    assert float(e16.max()) <= 2e-6
