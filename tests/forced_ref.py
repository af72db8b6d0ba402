"""Test helper (not a test module): the fast_st loss of the reference with every
ReLU / MaxPool branch decision FORCED to a given set of masks.

Why: the ITN backward crosses 15 InstanceNorm(+ReLU) layers and the VGG loss
network's ReLU / MaxPool layers.  An element whose pre-activation is within
rounding of 0 can land on either side of the kink in any fp32 implementation,
and every parameter upstream of such a "mask flip" then inherits a gradient
change far above fp32 rounding.  Comparing the HIP gradient with an fp64 run
that makes its OWN branch decisions therefore mixes two things.  Here the fp64
(and fp32) reference is re-run with the HIP forward's branch decisions (its ReLU
masks and 2x2 argmax indices): that is the gradient of exactly the piecewise-
linear branch HIP differentiated, so HIP must match it to fp32-class rounding
everywhere, and the flips themselves are counted separately against the fp64
run's own decisions.

The functional forward restates the reference (oracle/reference_cpu.py, i.e.
stransfer/network.py:461-611 for the ImageTransformNet -- zero padding, IN eps
1e-5 affine -- and :204-401 for the VGG-19 prefix and the losses of the fast_st
closure :690-731) with plain torch.nn.functional ops in the dtype of its inputs.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class Branches:
    """Records (masks=None) or replays (masks given) the branch decisions of one
    forward, in execution order: bool masks of the ReLUs, (mask, argmax index)
    pairs of the ReLU+MaxPool layers."""

    def __init__(self, masks=None):
        self.replay = masks is not None
        self.it = iter(masks) if masks is not None else None
        self.rec = []

    def relu(self, v):
        m = next(self.it) if self.replay else (v > 0)
        self.rec.append(m)
        return v * m.to(v.dtype)

    def relu_pool(self, z):
        """maxpool2x2(relu(z)) with the argmax taken as a gather (ties -> first)."""
        if self.replay:
            m, idx = next(self.it)
        else:
            m = z > 0
            _, idx = F.max_pool2d(F.relu(z), 2, 2, return_indices=True)
        self.rec.append((m, idx))
        b, c, h, w = z.shape
        a = (z * m.to(z.dtype)).reshape(b, c, h * w)
        return a.gather(2, idx.reshape(b, c, -1)).reshape(b, c, h // 2, w // 2)


def itn_forward(sd, x, br: Branches):
    """ImageTransformNet forward (stransfer/network.py:520-611) from a state_dict
    with the reference's keys ('0.weight' ... '22.bias')."""
    def conv(k, v, stride, pad):
        return F.conv2d(v, sd[f"{k}.weight"], sd[f"{k}.bias"], stride, pad)

    def inorm(k, v):
        return F.instance_norm(v, weight=sd[f"{k}.weight"], bias=sd[f"{k}.bias"], eps=1e-5)

    h = br.relu(inorm(1, conv(0, x, 1, 4)))
    h = br.relu(inorm(4, conv(3, h, 2, 1)))
    h = br.relu(inorm(7, conv(6, h, 2, 1)))
    for b in range(9, 14):  # ResidualBlock :461-506
        t = br.relu(inorm(f"{b}.insn1", conv(f"{b}.conv1", h, 1, 1)))
        h = inorm(f"{b}.insn2", conv(f"{b}.conv2", t, 1, 1) + h)
    h = F.interpolate(h, scale_factor=2, mode="nearest")
    h = br.relu(inorm(16, conv(15, h, 1, 1)))
    h = F.interpolate(h, scale_factor=2, mode="nearest")
    h = br.relu(inorm(20, conv(19, h, 1, 1)))
    return conv(22, h, 1, 4)


def vgg_forward(vw, x, br: Branches | None = None):
    """Z1..Z5 of VGG-19 conv1_1 .. conv3_1 (pre-ReLU conv outputs)."""
    br = br if br is not None else Branches()
    (w1, b1), (w2, b2), (w3, b3), (w4, b4), (w5, b5) = vw
    z1 = F.conv2d(x, w1, b1, 1, 1)
    z2 = F.conv2d(br.relu(z1), w2, b2, 1, 1)
    z3 = F.conv2d(br.relu_pool(z2), w3, b3, 1, 1)
    z4 = F.conv2d(br.relu(z3), w4, b4, 1, 1)
    z5 = F.conv2d(br.relu_pool(z4), w5, b5, 1, 1)
    return [z1, z2, z3, z4, z5]


def gram(z):
    b, c, h, w = z.shape
    f = z.reshape(b, c, h * w)
    return torch.bmm(f, f.transpose(1, 2)) / (c * h * w)


def fast_st_total(y, zs, targets, c4, style_weight=100_000, content_weight=1, tv=1e-6):
    """The static_train closure's scalar (stransfer/network.py:690-731): style
    (5 Gram MSEs, batch mean) + content (MSE at conv2_2, pre-ReLU) + TV (batch sum)."""
    style = torch.stack([F.mse_loss(gram(z), t.expand(z.shape[0], *t.shape[-2:]))
                         for z, t in zip(zs, targets)]).sum()
    content = F.mse_loss(zs[3], c4)
    tvl = tv * (torch.sum(torch.abs(y[:, :, :, :-1] - y[:, :, :, 1:]))
                + torch.sum(torch.abs(y[:, :, :-1, :] - y[:, :, 1:, :])))
    return style_weight * style + content_weight * content + tvl


def forced_grads(sd_np, vgg_np, style, batch, itn_masks, vgg_masks, dtype):
    """Parameter gradients (name -> tensor) of the fast_st total with every branch
    forced; targets (style Grams, content conv2_2) from unforced passes as the
    reference computes them (constants, no gradient)."""
    sd = {k: torch.tensor(v, dtype=dtype, requires_grad=True) for k, v in sd_np}
    vw = [(torch.tensor(w, dtype=dtype), torch.tensor(b, dtype=dtype)) for w, b in vgg_np]
    s = torch.as_tensor(style, dtype=dtype)
    x = torch.as_tensor(batch, dtype=dtype)
    with torch.no_grad():
        targets = [gram(z) for z in vgg_forward(vw, s)]
        c4 = vgg_forward(vw, x)[3]
    y = itn_forward(sd, x, Branches(itn_masks))
    zs = vgg_forward(vw, y, Branches(vgg_masks))
    total = fast_st_total(y, zs, targets, c4)
    total.backward()
    return {k: t.grad for k, t in sd.items()}, float(total.detach())


def natural_branches(sd_np, vgg_np, batch, dtype=torch.float64):
    """The branch decisions an unforced run in `dtype` makes: (itn, vgg) lists."""
    sd = {k: torch.tensor(v, dtype=dtype) for k, v in sd_np}
    vw = [(torch.tensor(w, dtype=dtype), torch.tensor(b, dtype=dtype)) for w, b in vgg_np]
    with torch.no_grad():
        bi, bv = Branches(), Branches()
        y = itn_forward(sd, torch.as_tensor(batch, dtype=dtype), bi)
        vgg_forward(vw, y, bv)
    return bi.rec, bv.rec


def count_flips(a, b):
    """Elements whose branch decision differs between two branch records."""
    n = 0
    for u, v in zip(a, b):
        if isinstance(u, tuple):
            n += int((u[0] != v[0]).sum()) + int((u[1] != v[1]).sum())
        else:
            n += int((u != v).sum())
    return n


def vgg_branches_from_z(zs):
    """HIP's VGG branch decisions from its own pre-ReLU outputs Z1..Z4 (the masks its
    backward applies: [Z>0]; its ReLU+MaxPool argmax, ties -> first)."""
    z1, z2, z3, z4 = [z.detach().float().cpu() for z in zs[:4]]
    out = [z1 > 0]
    _, i2 = F.max_pool2d(F.relu(z2), 2, 2, return_indices=True)
    out.append((z2 > 0, i2))
    out.append(z3 > 0)
    _, i4 = F.max_pool2d(F.relu(z4), 2, 2, return_indices=True)
    out.append((z4 > 0, i4))
    return out


# the ImageTransformNet's ReLU sites in forward order (the InstanceNorm each follows)
ITN_RELU_SITES = ["1", "4", "7"] + [f"{b}.insn1" for b in range(9, 14)] + ["16", "20"]


def flip_upstream(keys, itn_a, itn_b, vgg_a, vgg_b):
    """Indices (into the state_dict key list `keys`) of every parameter whose gradient a
    branch difference between records a and b can move beyond rounding: a flip at an
    ITN ReLU site moves the gradients of every parameter up to that site's
    InstanceNorm; a flip in the loss network moves all of them."""
    if count_flips(vgg_a, vgg_b):
        return set(range(len(keys)))
    last = -1
    for site, u, v in zip(ITN_RELU_SITES, itn_a, itn_b):
        if int((u != v).sum()):
            last = keys.index(f"{site}.bias")
    return set(range(last + 1))


class HipBranchSpy:
    """Context manager recording the HIP forward's branch decisions: the ReLU mask of
    every fused InstanceNorm+ReLU of `net` (forward hooks) and, from the loss
    network's own pre-ReLU outputs Z1..Z4 (a spy on `vgg_mod.loss_forward`, the fused
    engine both the reference-API StyleNetwork and the trainers call), the VGG masks
    and argmax indices.  Use `with HipBranchSpy(net, V, monkeypatch) as spy: ...`, then
    spy.itn, spy.vgg."""

    def __init__(self, net, vgg_mod, monkeypatch):
        self.net, self.V, self.mp = net, vgg_mod, monkeypatch
        self.itn, self.zs = [], []

    def __enter__(self):
        def hook(m, args, kwargs, out):
            if kwargs.get("relu", False):
                self.itn.append((out.detach() > 0).cpu())
        self.hs = [m.register_forward_hook(hook, with_kwargs=True) for m in self.net.modules()
                   if isinstance(m, torch.nn.InstanceNorm2d)]
        self.orig = self.V.loss_forward

        def spy(*a, **k):
            st = self.orig(*a, **k)
            self.zs[:] = [z.detach().clone() for z in st.z]
            return st
        self.mp.setattr(self.V, "loss_forward", spy)
        return self

    def __exit__(self, *exc):
        self.mp.setattr(self.V, "loss_forward", self.orig)
        for h in self.hs:
            h.remove()

    @property
    def vgg(self):
        return vgg_branches_from_z(self.zs)
