"""Numerics study: what does a bf16x3 split conv (hi*hi + hi*lo + lo*hi, fp32
accumulate) do to the Gatys losses and image gradient, compared with plain fp32
and an fp64 ground truth?  CPU only (emulated in fp64 over the split operands).

    python tools/split_numerics.py [--size 128]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import weights as W  # noqa: E402


def split(t):
    hi = t.float().to(torch.bfloat16).to(torch.float64)
    lo = (t.float().to(torch.float64) - hi).float().to(torch.bfloat16).to(torch.float64)
    return hi, lo


class SplitConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, terms):
        ctx.save_for_backward(x, w)
        ctx.terms = terms
        return _conv(x, w, terms) + b.view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        # dgrad = conv_transpose(gy, w): emulate by splitting gy and w
        gh, gl = split(gy)
        wh, wl = split(w)
        tr = lambda a, b: F.conv_transpose2d(a, b, padding=1)  # noqa: E731
        if ctx.terms == 3:
            dx = tr(gh, wh) + tr(gh, wl) + tr(gl, wh)
        else:
            dx = tr(gy.double(), w.double())
        return dx.to(x.dtype), None, None, None


def _conv(x, w, terms):
    if terms == 0:
        return F.conv2d(x, w, padding=1)
    xh, xl = split(x)
    wh, wl = split(w)
    y = F.conv2d(xh, wh, padding=1) + F.conv2d(xh, wl, padding=1) + F.conv2d(xl, wh, padding=1)
    return y.to(x.dtype)


def gram(z):
    b, c, h, w = z.shape
    f = z.reshape(b, c, h * w)
    return torch.bmm(f, f.transpose(1, 2)) / (c * h * w)


def gatys(x, convs, terms, targets=None, c4=None, dtype=torch.float32):
    zs = []
    cur = x
    for i, (w, b) in enumerate(convs):
        if i in (1, 3):
            cur = F.relu(cur)
        if i in (2, 4):
            cur = F.max_pool2d(F.relu(cur), 2)
        if terms == 0:
            cur = F.conv2d(cur, w.to(dtype), b.to(dtype), padding=1)
        else:
            cur = SplitConv.apply(cur, w.to(dtype), b.to(dtype), terms)
        zs.append(cur)
    gs = [gram(z) for z in zs]
    return zs, gs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=128)
    a = ap.parse_args()
    H = a.size
    convs = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in W.vgg19_synthetic(1234, 5)]
    s = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H)))
    c = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H)))
    res = {}
    for name, terms, dt in (("fp64", 0, torch.float64), ("fp32", 0, torch.float32),
                            ("bf16x3", 3, torch.float32)):
        with torch.no_grad():
            _, tg = gatys(s.to(dt), convs, terms, dtype=dt)
            zc, _ = gatys(c.to(dt), convs, terms, dtype=dt)
        x = (c + 0.05 * torch.from_numpy(W.synthetic_image(77, (1, 3, H, H)))).to(dt).requires_grad_()
        zs, gs = gatys(x, convs, terms, dtype=dt)
        sl = [((g - t) ** 2).mean() for g, t in zip(gs, tg)]
        cl = ((zs[3] - zc[3]) ** 2).mean()
        tot = 1e5 * sum(sl) + cl
        tot.backward()
        res[name] = dict(sl=[float(v) for v in sl], cl=float(cl), tot=float(tot),
                         g=x.grad.double().numpy(), G=[g.detach().double().numpy() for g in gs])
    ref = res["fp64"]
    for name in ("fp32", "bf16x3"):
        r = res[name]
        sl = max(abs(a - b) / abs(b) for a, b in zip(r["sl"], ref["sl"]))
        gram_err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(r["G"], ref["G"]))
        gram_el = max(np.abs(a - b).max() / np.abs(b).max() for a, b in zip(r["G"], ref["G"]))
        ge = np.linalg.norm(r["g"] - ref["g"]) / np.linalg.norm(ref["g"])
        gmax = np.abs(r["g"] - ref["g"]).max() / np.abs(ref["g"]).max()
        print(f"{name:7s} style-loss rel {sl:.2e}  content rel {abs(r['cl'] - ref['cl']) / ref['cl']:.2e}"
              f"  total rel {abs(r['tot'] - ref['tot']) / ref['tot']:.2e}  gram norm {gram_err:.2e}"
              f" gram max/max {gram_el:.2e}  grad norm {ge:.2e}  grad max/max {gmax:.2e}")
    r, f = res["bf16x3"], res["fp32"]
    print("bf16x3 vs fp32: total rel %.2e grad norm %.2e" % (
        abs(r["tot"] - f["tot"]) / f["tot"],
        np.linalg.norm(r["g"] - f["g"]) / np.linalg.norm(f["g"])))


if __name__ == "__main__":
    main()
