"""ImageTransformNet / fast_st gradients against fp64 with the branch decisions
forced (tests/forced_ref.py), replacing the "first jump => 3e-2 upstream" walk.

For each case the HIP training step (train.FastStTrainer: fused IN+ReLU, ResLink
skip gradients, pool_sum up-conv data gradients, the fused VGG loss network) runs
with hooks that record its branch decisions: the ReLU mask of every fused
InstanceNorm+ReLU output and, from the loss network's own pre-ReLU outputs Z1..Z4,
the VGG ReLU masks and 2x2 argmax indices.  Then, on the host:

  * flips: the number of elements whose HIP decision differs from an unforced fp64
    run's -- an element within rounding of a kink; must be a handful;
  * gradients: fp64 and fp32 (torch CPU) re-runs of the reference loss with the HIP
    decisions forced; every parameter's HIP gradient must be within K x the fp32
    run's error against the fp64 run (both relative to the fp64 gradient norm).

Reference: stransfer/network.py:461-611 (ImageTransformNet, ResidualBlock),
:690-731 (the static_train closure), :204-401 (loss network).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import forced_ref as R
from conftest import GOLDEN
from styletransfer_amd import _native as N
from styletransfer_amd import autograd as A
from styletransfer_amd import network
from styletransfer_amd import vgg as V
from styletransfer_amd import weights as W

pytestmark = pytest.mark.gpu

# HIP error vs fp64 <= max(K * (torch-fp32 error vs fp64), FLOOR) (relative norms).  The
# fp16 hi/lo split represents each operand to ~2^-23 and drops the lo*lo product (~2^-24):
# per product ~2-3x fp32's 2^-24 rounding, which is what K allows.  A handful of small
# gradients (the IN affine parameters of the deep residual blocks, where the fp32 error
# itself is ~1e-6) land at 3-6x; FLOOR keeps those at fp32 class: 2e-5 is 5x under the
# north star's 1e-4 and far below the ~1e-2 a real defect (a lost term, a wrong scale,
# a dropped skip gradient) produces.
K = 3.0
FLOOR = 2e-5


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def _hip_step_with_branches(style, batch, sd, dev, monkeypatch):
    """One FastStTrainer forward/backward; returns (grads by name, loss, itn branches,
    vgg branches)."""
    from styletransfer_amd.train import FastStTrainer
    net = network.ImageTransformNet(style, batch.shape[0])
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd})
    tr = FastStTrainer(net, style)
    with R.HipBranchSpy(net, V, monkeypatch) as spy:
        loss = float(tr._fwd_bwd(batch))
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().clone() for k, p in net.named_parameters()}
    return grads, loss, spy.itn, spy.vgg


def _three_way(style, batch, sd, dev, monkeypatch, max_flips):
    vgg = V.load_vgg19_weights()
    g_hip, loss_hip, bi, bv = _hip_step_with_branches(style.to(dev), batch.to(dev), sd, dev,
                                                      monkeypatch)
    s_np, b_np = style.numpy(), batch.numpy()
    ni, nv = R.natural_branches(sd, vgg, b_np)
    flips = R.count_flips(bi, ni) + R.count_flips(bv, nv)
    # the fp32 reference's own flips against the same fp64 run (the count an fp32
    # implementation is entitled to)
    ni32, nv32 = R.natural_branches(sd, vgg, b_np, torch.float32)
    flips32 = R.count_flips(ni32, ni) + R.count_flips(nv32, nv)
    n_el = sum(int(m.numel()) for m in bi) + sum(int(m[0].numel()) for m in bv)
    g64, l64 = R.forced_grads(sd, vgg, s_np, b_np, bi, bv, torch.float64)
    g32, _ = R.forced_grads(sd, vgg, s_np, b_np, bi, bv, torch.float32)
    gmax = max(float(g.norm()) for g in g64.values())
    worst = []
    for k, t in g64.items():
        if float(t.norm()) < 1e-7 * gmax:
            # conv bias feeding an InstanceNorm: exactly 0 in exact arithmetic
            assert float(g_hip[k].norm()) < 1e-5 * gmax, k
            continue
        e, r = _rel(g_hip[k], t), _rel(g32[k], t)
        worst.append((e / max(r, FLOOR), e, r, k))
        assert e <= max(K * r, FLOOR), f"{k}: hip {e:.2e} vs fp32 {r:.2e} (forced branches)"
    worst.sort()
    print(f"flips {flips} (fp32 reference: {flips32}) of {n_el}; loss hip {loss_hip:.7g} "
          f"fp64 {l64:.7g}; worst (ratio, hip, fp32, param): {worst[-3:]}")
    assert abs(loss_hip - l64) <= 1e-4 * abs(l64)
    assert flips <= max(3 * flips32, max_flips), (flips, flips32)
    return flips


def test_itn_grads_forced_branches_golden(dev, monkeypatch):
    """The golden ITN case (itn.npz: B=2, 64^2, hash-PRNG weights 4321)."""
    d = np.load(os.path.join(GOLDEN, "itn.npz"))
    sd = W.itn_synthetic(4321)
    _three_way(torch.from_numpy(d["style"]), torch.from_numpy(d["batch"]), sd, dev,
               monkeypatch, max_flips=8)


def test_fast_st_step_config4_b8_256_forced_branches(dev, monkeypatch):
    """BASELINE config 4's per-GPU step: FastStTrainer at B=8, 256x256 (the shape each
    of the 8 data-parallel ranks trains)."""
    style = torch.from_numpy(W.synthetic_image(41, (1, 3, 256, 256)))
    batch = torch.from_numpy(W.synthetic_image(42, (8, 3, 256, 256)))
    _three_way(style, batch, W.itn_synthetic(4321), dev, monkeypatch, max_flips=32)


# --------------------------------------------------------------- block-level fp64
def _block_sd(sd, b):
    pre = f"{b}."
    return {k[len(pre):]: torch.from_numpy(v) for k, v in sd if k.startswith(pre)}


@pytest.mark.parametrize("batch", [2, 8])
def test_residual_block_reslink_fp64(dev, batch):
    """ResidualBlock (stransfer/network.py:461-506) forward + backward: the skip
    gradient is handed to conv1's data-gradient epilogue (autograd.ResLink) -- dx,
    and every parameter gradient, vs fp64 with insn1's ReLU mask forced."""
    sd = _block_sd(W.itn_synthetic(4321), 11)
    blk = network.ResidualBlock(128, 128, 3).to(dev)
    blk.load_state_dict(sd)
    g = torch.Generator().manual_seed(batch)
    x0 = torch.randn(batch, 128, 64, 64, generator=g)
    up = torch.randn(batch, 128, 64, 64, generator=g)
    mask = []
    h = blk.insn1.register_forward_hook(
        lambda m, a, k, out: mask.append((out.detach() > 0).cpu()), with_kwargs=True)
    x = x0.to(dev).requires_grad_()
    out = blk(x)
    h.remove()
    out.backward(up.to(dev))
    hip = {"x": x.grad.cpu(), **{k: p.grad.cpu() for k, p in blk.named_parameters()}}
    assert blk.conv1.weight.grad is not None

    def ref(dtype):
        p = {k: v.to(dtype).requires_grad_() for k, v in sd.items()}
        xr = x0.to(dtype).requires_grad_()
        t = F.instance_norm(F.conv2d(xr, p["conv1.weight"], p["conv1.bias"], 1, 1),
                            weight=p["insn1.weight"], bias=p["insn1.bias"], eps=1e-5)
        t = t * mask[0].to(dtype)
        o = F.instance_norm(F.conv2d(t, p["conv2.weight"], p["conv2.bias"], 1, 1) + xr,
                            weight=p["insn2.weight"], bias=p["insn2.bias"], eps=1e-5)
        o.backward(up.to(dtype))
        return o.detach(), {"x": xr.grad, **{k: v.grad for k, v in p.items()}}
    o64, r64 = ref(torch.float64)
    o32, r32 = ref(torch.float32)
    assert _rel(out.detach().cpu(), o64) <= max(K * _rel(o32, o64), FLOOR)
    for k, t in r64.items():
        if k.endswith("bias") and k.startswith("conv"):
            continue  # feeds an InstanceNorm: exactly 0
        e, r = _rel(hip[k], t), _rel(r32[k], t)
        assert e <= max(K * r, FLOOR), f"{k}: hip {e:.2e} vs fp32 {r:.2e}"


@pytest.mark.parametrize("batch", [2, 8])
def test_upsample_conv_pool_sum_fp64(dev, batch):
    """nearest x2 upsampling + 3x3 conv 128 -> 64 at 64^2 -> 128^2 (the ITN's first up
    conv, stransfer/network.py:583-605): its data gradient takes the fused 2x2-sum
    (`pool_sum`) epilogue -- dx, dW, db vs fp64."""
    sd = W.itn_synthetic(4321)
    w0 = torch.from_numpy(dict(sd)["15.weight"])
    b0 = torch.from_numpy(dict(sd)["15.bias"])
    g = torch.Generator().manual_seed(100 + batch)
    x0 = torch.randn(batch, 128, 64, 64, generator=g)
    up = torch.randn(batch, 64, 128, 128, generator=g)
    x = x0.to(dev).requires_grad_()
    w = w0.to(dev).requires_grad_()
    b = b0.to(dev).requires_grad_()
    y = A.conv2d(x, w, b, 1, 1, in_mode=N.STX_IN_UPSAMPLE2)
    y.backward(up.to(dev))
    hip = {"y": y.detach().cpu(), "x": x.grad.cpu(), "w": w.grad.cpu(), "b": b.grad.cpu()}

    def ref(dtype):
        xr = x0.to(dtype).requires_grad_()
        wr, br = w0.to(dtype).requires_grad_(), b0.to(dtype).requires_grad_()
        yr = F.conv2d(F.interpolate(xr, scale_factor=2, mode="nearest"), wr, br, 1, 1)
        yr.backward(up.to(dtype))
        return {"y": yr.detach(), "x": xr.grad, "w": wr.grad, "b": br.grad}
    r64, r32 = ref(torch.float64), ref(torch.float32)
    for k in r64:
        e, r = _rel(hip[k], r64[k]), _rel(r32[k], r64[k])
        assert e <= max(K * r, FLOOR), f"{k}: hip {e:.2e} vs fp32 {r:.2e}"
