"""ImageTransformNet backward, layer by layer, against fp64 (VERDICT r1 "parity
holes" 1: a 1 %-level bug in wgrad16 / wgrad9 / the InstanceNorm backward must not
hide behind the end-to-end tolerance).

The pinned oracle (oracle/reference_cpu.py) runs the golden ITN case (itn.npz
inputs, the reference's loss) in float64 with hooks that record, for every conv
and InstanceNorm(+ReLU) of the network, its input and the gradient arriving at
its output.  Each layer is then re-run alone -- on exactly those activations and
upstream gradients, rounded to fp32 -- through the HIP autograd Functions the
ITN uses (split-MFMA 3x3 convs incl. the stride-2 and fused nearest-upsample
loaders, the 9x9 few-channel convs, wgrad16 / wgrad9, the fused IN+ReLU), and
through torch fp32 on the CPU.  Per layer and per gradient (dx, dW, db /
dgamma, dbeta): HIP error vs fp64 <= max(3 x torch-fp32 error, 2e-6).

End to end, gradients through 15 IN+ReLU layers are subject to ReLU-mask flips
of elements within rounding of 0 (tests/test_parity_gpu.py); the layer-local
check has no such cascade, so it pins every kernel at the fp32-class level.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from conftest import GOLDEN
from styletransfer_amd import _native as N
from styletransfer_amd import autograd as A
from styletransfer_amd import weights as W

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


@pytest.fixture(scope="module")
def records():
    from oracle import reference_cpu as O
    d = np.load(os.path.join(GOLDEN, "itn.npz"))
    style = torch.from_numpy(d["style"]).double()
    batch = torch.from_numpy(d["batch"]).double()
    cimg = torch.from_numpy(W.synthetic_image(23, (1, 3, 64, 64))).double()
    net = O.image_transform_net(4321).double()
    ln = O.StyleNetwork(style, cimg, vgg=O.vgg19_features(1234).double())
    rec = {}
    mods = dict(net.named_modules())

    def fwd_hook(name):
        def h(m, inp):
            rec.setdefault(name, {})["x"] = inp[0].detach().clone()
        return h

    def bwd_hook(name):
        def h(m, gin, gout):
            r = rec.setdefault(name, {})
            r["dy"] = gout[0].detach().clone()
            r["dx"] = gin[0].detach().clone() if gin[0] is not None else None
        return h
    for name, m in mods.items():
        if isinstance(m, (nn.Conv2d, nn.InstanceNorm2d, nn.ReLU, nn.Upsample)):
            m.register_forward_pre_hook(fwd_hook(name))
            m.register_full_backward_hook(bwd_hook(name))
    batch.requires_grad_()  # so the first conv's input gradient is hooked too
    O.fast_st_closure(net, ln, batch)
    for name, m in mods.items():
        if isinstance(m, (nn.Conv2d, nn.InstanceNorm2d)):
            rec[name]["params"] = [(p.detach().clone(), p.grad.detach().clone())
                                   for p in (m.weight, m.bias)]
    return net, rec


def _conv_cases(net):
    """(conv name, input-record name, in_mode): the ITN's convs; the two after an
    Upsample take the pre-upsample input through the fused nearest-x2 loader."""
    out = []
    for name, m in net.named_modules():
        if isinstance(m, nn.Conv2d):
            src, mode = name, N.STX_IN_RAW
            if "." not in name:
                prev = str(int(name) - 1)
                if isinstance(net[int(prev)], nn.Upsample):
                    src, mode = prev, N.STX_IN_UPSAMPLE2
            out.append((name, src, mode))
    return out


def _in_cases(net):
    """(IN name, name whose output gradient is the fused op's dy, relu)."""
    out = []
    names = [n for n, _ in net.named_modules()]
    for name, m in net.named_modules():
        if not isinstance(m, nn.InstanceNorm2d):
            continue
        if "." in name:                     # ResidualBlock: insn1 -> relu; insn2 alone
            blk = name.rsplit(".", 1)[0]
            relu = name.endswith("insn1")
            out.append((name, f"{blk}.relu" if relu else name, relu))
        else:                               # top level: IN followed by ReLU
            nxt = str(int(name) + 1)
            relu = nxt in names and isinstance(net[int(nxt)], nn.ReLU)
            out.append((name, nxt if relu else name, relu))
    return out


def _check(tag, got, ref32, truth, floor=2e-6):
    e, r = _rel(got, truth), _rel(ref32, truth)
    assert e <= max(3.0 * r, floor), f"{tag}: hip {e:.2e} vs fp32 {r:.2e}"
    return e, r


def test_itn_conv_layers_vs_fp64(records, dev):
    net, rec = records
    worst = []
    for name, src, mode in _conv_cases(net):
        m = dict(net.named_modules())[name]
        (w64, dw64), (b64, db64) = rec[name]["params"]
        x64 = rec[src]["x"]
        dy64 = rec[name]["dy"]
        dx64 = rec[src]["dx"]
        stride, pad = m.stride[0], m.padding[0]
        # HIP
        x = x64.float().to(dev).requires_grad_()
        w = w64.float().to(dev).requires_grad_()
        b = b64.float().to(dev).requires_grad_()
        y = A.conv2d(x, w, b, stride, pad, in_mode=mode)
        y.backward(dy64.float().to(dev))
        # torch fp32 (CPU) on the same rounded inputs
        xc = x64.float().requires_grad_()
        wc, bc = w64.float().requires_grad_(), b64.float().requires_grad_()
        xin = F.interpolate(xc, scale_factor=2, mode="nearest") if mode == N.STX_IN_UPSAMPLE2 else xc
        F.conv2d(xin, wc, bc, stride, pad).backward(dy64.float())
        worst.append((_check(f"{name} dW", w.grad, wc.grad, dw64)[0], name, "dW"))
        if dx64 is not None:
            worst.append((_check(f"{name} dx", x.grad, xc.grad, dx64)[0], name, "dx"))
        if db64.norm() > 1e-8 * dw64.norm():
            worst.append((_check(f"{name} db", b.grad, bc.grad, db64)[0], name, "db"))
        else:  # bias feeding InstanceNorm: exactly 0; both sides hold rounding noise
            assert float(b.grad.norm()) <= 1e-4 * float(dy64.norm()), name
    print("worst conv-layer errors vs fp64:", sorted(worst)[-4:])


def test_itn_instnorm_layers_vs_fp64(records, dev):
    net, rec = records
    worst = []
    for name, dy_from, relu in _in_cases(net):
        (g64, dg64), (b64, db64) = rec[name]["params"]
        x64, dx64 = rec[name]["x"], rec[name]["dx"]
        dy64 = rec[dy_from]["dy"]
        x = x64.float().to(dev).requires_grad_()
        gm = g64.float().to(dev).requires_grad_()
        bt = b64.float().to(dev).requires_grad_()
        A.instance_norm(x, gm, bt, eps=1e-5, relu=relu).backward(dy64.float().to(dev))
        xc = x64.float().requires_grad_()
        gc, bc = g64.float().requires_grad_(), b64.float().requires_grad_()
        yc = F.instance_norm(xc, weight=gc, bias=bc, eps=1e-5)
        (F.relu(yc) if relu else yc).backward(dy64.float())
        for tag, got, r32, t in (("dx", x.grad, xc.grad, dx64), ("dgamma", gm.grad, gc.grad, dg64),
                                 ("dbeta", bt.grad, bc.grad, db64)):
            worst.append((_check(f"{name} {tag}", got, r32, t)[0], name, tag))
    print("worst IN-layer errors vs fp64:", sorted(worst)[-4:])


@pytest.mark.parametrize("shape", [(2, 4, 256, 256), (1, 3, 128, 256), (1, 2, 256, 512)])
@pytest.mark.parametrize("relu", [True, False])
def test_instnorm_large_planes_vs_fp64(dev, shape, relu):
    """InstanceNorm(+ReLU) forward / backward on large planes (the ITN's 256^2 layers take
    the segmented two-pass backward: per-4096-float segment sums, merged in segment order)
    vs torch fp64; the parameter gradients through the deferred-partials path agree."""
    g = torch.Generator().manual_seed(7)
    x64 = torch.randn(*shape, generator=g, dtype=torch.float64) * 3 + 1
    dy64 = torch.randn(*shape, generator=g, dtype=torch.float64)
    c = shape[1]
    g64 = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    b64 = torch.randn(c, generator=g, dtype=torch.float64)
    x = x64.float().to(dev).requires_grad_()
    gm = g64.float().to(dev).requires_grad_()
    bt = b64.float().to(dev).requires_grad_()
    y = A.instance_norm(x, gm, bt, eps=1e-5, relu=relu)
    y.backward(dy64.float().to(dev))
    xr = x64.clone().requires_grad_()
    gr, br = g64.clone().requires_grad_(), b64.clone().requires_grad_()
    yr = F.instance_norm(xr, weight=gr, bias=br, eps=1e-5)
    yr = F.relu(yr) if relu else yr
    yr.backward(dy64)
    for tag, got, ref in (("y", y.detach(), yr.detach()), ("dx", x.grad, xr.grad),
                          ("dgamma", gm.grad, gr.grad), ("dbeta", bt.grad, br.grad)):
        e = float((got.double().cpu() - ref).norm() / ref.norm())
        assert e < 2e-5, (tag, e)
