"""torch.autograd.Functions over libstx so the reference-style module API
(`loss.backward()` on StyleLoss/ContentLoss sums, ImageTransformNet training)
runs on the HIP kernels unchanged."""
from __future__ import annotations

import torch

from . import _native as N
from . import ops
from . import vgg as V


def _c(t):
    return t.contiguous() if t is not None and not t.is_contiguous() else t


def _split_on():
    import os
    return N.knob("STX_CONV_SPLIT", "1") != "0"


def _upsample_fuse_on():
    import os
    return N.knob("STX_UPSAMPLE_FUSE", "1") != "0"


def _upar_on():
    """STX_UPAR=0: upsampled-input convs over the upsampled halo (no parity classes; A/B)."""
    import os
    return N.knob("STX_UPAR", "1") != "0"


def _grad_into(param, g, accumulate_fn):
    """Parameter gradients straight into an existing `param.grad` (e.g. the flat
    gradient buffer of train.FastStTrainer): `accumulate_fn(dst)` adds the gradient
    into dst and the Function returns None for it, which is exactly autograd's
    `param.grad += g` without the extra add launch.  Without a .grad (or for a
    non-leaf) the gradient is returned as usual."""
    if param is not None and param.is_leaf and param.grad is not None and \
            param.grad.is_contiguous() and param.grad.dtype == torch.float32:
        accumulate_fn(param.grad)
        return None
    return g() if callable(g) else g


# ----------------------------------------------------------------------- conv
class ResLink:
    """Hand-off of a residual block's skip gradient (stransfer/network.py:502 `out +=
    residual`): the InstanceNorm that adds the residual stores its du here instead of
    returning it for the block input, and the block's first conv (which reads the same
    input) adds it in its data-gradient epilogue -- autograd's separate sum of the two
    gradient contributions (one elementwise pass per block) disappears.  The IN's
    backward always runs first: the first conv's output gradient depends on it."""

    __slots__ = ("g", "accepted")

    def __init__(self):
        self.g = None
        self.accepted = False  # set by the conv that will add g in its epilogue


class Conv2dFn(torch.autograd.Function):
    """y = conv2d(V(x), w) + b with V = identity / relu / nearest-upsample-x2.
    (nn.Conv2d of VGG-19 and ImageTransformNet; zero padding.)"""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, in_mode, wt=None, wt16=None, wtT=None, wtT16=None,
                link=None, wt16_up=None):
        x = _c(x)
        # link (ResLink): a skip gradient to add into dx (raw-input stride-1 convs only)
        ctx.link = link if (stride == 1 and in_mode == N.STX_IN_RAW) else None
        if link is not None:
            # only a consuming conv takes the hand-off; otherwise the IN returns dres
            link.accepted = ctx.link is not None
        cout, cin, ks, _ = w.shape
        # 3x3 stride-1 layers with cin >= 16 run on the fp16 hi/lo split MFMA kernel
        # (no fp32 slab needed); max|x| is computed once and kept for the wgrad.
        # wtT / wtT16: prepped data-gradient slabs (ops.TrainedSlabs), else prepped here
        split = _split_on() and pad == 1 and ops.split_eligible(cin, cout, ks, stride)
        x_amax = None
        ctx.wtT16, ctx.wtT = wtT16, wtT
        if split:
            if wt16 is None:
                if w.requires_grad and stride == 1 and ops.split_eligible(cout, cin, ks, 1) \
                        and wtT16 is None:
                    # trained layer: both slabs (forward + data gradient) in one go
                    wt16, ctx.wtT16 = ops.conv_weight_prep16_pair(w.detach().contiguous())
                else:
                    wt16 = ops.conv_weight_prep16(w.detach().contiguous())
            x_amax = ops.ARENA.lookup(x)  # annotated by the producer (InstanceNorm)
            if x_amax is None:
                x_amax = ops.amax(x)
        elif wt is None:
            wt = ops.conv_weight_prep(w.detach().contiguous())
            if stride == 2 and _split_on() and w.requires_grad:
                x_amax = ops.ARENA.lookup(x)  # for the split stride-2 wgrad (None: computed there)
        if ks == 9 and cout <= 3 and cin <= 32:
            # conv22 (32 -> 3): the split 9x9 kernel takes a max|x| bound -- the producing
            # InstanceNorm's amax group inside the trainers (ops.ARENA), else computed here
            # (the same exact max either way, so both paths give the same bits)
            x_amax = ops.ARENA.lookup(x)
            if x_amax is None:
                x_amax = ops.amax(x)
        if split and in_mode == N.STX_IN_UPSAMPLE2 and wt16_up is None and _upar_on() and \
                ks == 3 and 2 * x.shape[3] > 32:
            # (trained / cached layers hand the parity-class slab in; prepped per call here)
            wt16_up = ops.conv_weight_prep16_up(w.detach().contiguous())
        y = ops.conv2d(x, wt, cin, cout, ks, stride=stride, pad=pad, in_mode=in_mode,
                       bias=None if b is None else b.detach(), wt16=wt16 if split else None,
                       in_amax=x_amax, wt16_up=wt16_up if split and _upar_on() else None)
        ctx.save_for_backward(x, w)
        ctx.x_amax = x_amax
        ctx.b_ref = b
        ctx.cfg = (stride, pad, in_mode, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, in_mode, has_b = ctx.cfg
        dy = _c(dy)
        cout, cin, ks, _ = w.shape
        dx = dw = db = None
        # max|dy| once for the split dgrad and the split wgrad
        dy_amax = None
        split_d = stride == 1 and _split_on() and pad == 1 and ops.split_eligible(cout, cin, ks, 1)
        if (split_d and ctx.needs_input_grad[0]) or (ctx.needs_input_grad[1] and _split_on() and (
                (ks == 3 and stride in (1, 2) and pad == 1) or ks == 9)):
            dy_amax = ops.ARENA.lookup(dy)
            if dy_amax is None:
                dy_amax = ops.amax(dy)
        if ctx.needs_input_grad[0]:
            h, wd = x.shape[2], x.shape[3]
            hv, wv = ops.virtual_hw(h, wd, in_mode)
            if stride == 1:
                wtT = wtT16 = None
                if split_d:
                    wtT16 = ctx.wtT16 if ctx.wtT16 is not None else ops.conv_weight_prep16(
                        w.detach().contiguous(), transpose=True)
                else:
                    wtT = ctx.wtT if ctx.wtT is not None else ops.conv_weight_prep(
                        w.detach().contiguous(), transpose=True)
                link = ctx.link
                skip = link.g if link is not None else None
                if link is not None:
                    link.g = None
                if split_d and in_mode == N.STX_IN_UPSAMPLE2 and skip is None and wv > 32 \
                        and hv % 2 == 0 and wv % 2 == 0 and hv == 2 * h and wv == 2 * wd \
                        and _upsample_fuse_on():
                    # UpsampleConvLayer (stransfer/network.py:583-605): the nearest-x2
                    # backward (2x2 sums) is fused into the data gradient's epilogue
                    dx = torch.empty_like(x)
                    ops.conv2d(dy, wtT, cout, cin, ks, pad=ks - 1 - pad, wt16=wtT16,
                               in_amax=dy_amax, pool_out=dx, pool_sum=True)
                    dv = None
                else:
                    dv = ops.conv2d(dy, wtT, cout, cin, ks, pad=ks - 1 - pad, wt16=wtT16,
                                    in_amax=dy_amax, aux=skip, aux_scale=1.0 if skip is not None
                                    else 0.0)
            elif stride == 2:
                # stride-1 conv over the zero-dilated dy; the split kernel takes it too
                if _split_on() and pad == 1 and ops.split_eligible(cout, cin, ks, 1):
                    wtT16 = ctx.wtT16 if ctx.wtT16 is not None else ops.conv_weight_prep16(
                        w.detach().contiguous(), transpose=True)
                    dv = ops.conv2d(dy, None, cout, cin, ks, pad=ks - 1 - pad,
                                    in_mode=N.STX_IN_DILATE2, hv=hv, wv=wv, wt16=wtT16,
                                    in_amax=dy_amax if dy_amax is not None else ops.amax(dy))
                else:
                    wtT = ctx.wtT if ctx.wtT is not None else ops.conv_weight_prep(
                        w.detach().contiguous(), transpose=True)
                    dv = ops.conv2d(dy, wtT, cout, cin, ks, pad=ks - 1 - pad,
                                    in_mode=N.STX_IN_DILATE2, hv=hv, wv=wv)
            else:
                raise NotImplementedError("stride > 2")
            if dv is None:
                pass  # dx came out of the fused epilogue
            elif in_mode == N.STX_IN_UPSAMPLE2:
                dx = ops.upsample2x_bwd(dv)
            elif in_mode == N.STX_IN_RELU:
                dx = ops.relu_bwd(dv, x)
            elif in_mode == N.STX_IN_RAW:
                dx = dv
            else:
                raise NotImplementedError("in_mode backward")
        if ctx.needs_input_grad[1]:
            # into the trainer's flat gradient: on the weight-gradient side stream
            # (ops.SIDE, active inside a training step) next to the data gradients
            dw = _grad_into(w, lambda: ops.conv2d_wgrad(
                x, dy, cin, cout, ks, stride=stride, pad=pad, in_mode=in_mode,
                x_amax=ctx.x_amax, dy_amax=dy_amax),
                lambda dst: ops.SIDE.run(lambda: ops.conv2d_wgrad(
                    x, dy, cin, cout, ks, stride=stride, pad=pad, in_mode=in_mode,
                    dw=dst.view(w.shape), accumulate=True, x_amax=ctx.x_amax,
                    dy_amax=dy_amax), x, dy, ctx.x_amax, dy_amax))
        if has_b and ctx.needs_input_grad[2]:
            b = ctx.b_ref
            db = _grad_into(b, lambda: ops.bias_grad(dy),
                            lambda dst: ops.bias_grad(dy, db=dst, accumulate=True))
        return dx, dw, db, None, None, None, None, None, None, None, None, None


def conv2d(x, w, b=None, stride=1, pad=None, in_mode=N.STX_IN_RAW, wt=None, wt16=None,
           wtT=None, wtT16=None, link=None, wt16_up=None):
    ks = w.shape[-1]
    return Conv2dFn.apply(x, w, b, stride, ks // 2 if pad is None else pad, in_mode, wt, wt16,
                          wtT, wtT16, link, wt16_up)


# ----------------------------------------------------------------------- relu / pool
class ReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = ops.relu(_c(x))
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return ops.relu_bwd(_c(dy), y)


class MaxPool2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _c(x)
        y, idx = ops.maxpool2x2(x)
        ctx.save_for_backward(idx)
        ctx.hw = x.shape[2:]
        ctx.mark_non_differentiable(idx)
        return y, idx

    @staticmethod
    def backward(ctx, dy, _didx):
        (idx,) = ctx.saved_tensors
        return ops.maxpool2x2_bwd(_c(dy), idx, *ctx.hw)


class Upsample2xFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return ops.upsample2x(_c(x))

    @staticmethod
    def backward(ctx, dy):
        return ops.upsample2x_bwd(_c(dy))


# ----------------------------------------------------------------------- instance norm
class InstanceNormFn(torch.autograd.Function):
    """y = [relu](IN(x (+ res)) * gamma + beta), per-instance stats (eps 1e-5)."""

    @staticmethod
    def forward(ctx, x, res, gamma, beta, eps, relu, conv_bias=None, res_link=None):
        # conv_bias: the bias of the conv that produced x, given when that conv ran with a
        # detached bias -- its gradient sum(du) comes out of this backward's kernel
        x, res = _c(x), _c(res)
        g = ops.ARENA.take(x.device)
        y, mean, rstd = ops.instnorm_fwd(x, None if gamma is None else gamma.detach(),
                                         None if beta is None else beta.detach(), res=res,
                                         eps=eps, relu=relu, out_amax=g)
        ops.ARENA.annotate(y, g)
        ctx.save_for_backward(x, res, gamma, mean, rstd)  # (the ReLU mask is recomputed)
        ctx.beta_ref = beta
        ctx.cb_ref = conv_bias
        ctx.relu = relu
        ctx.has_res = res is not None
        ctx.res_link = res_link if res is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, res, gamma, mean, rstd = ctx.saved_tensors
        c = x.shape[1]
        cb = ctx.cb_ref if ctx.needs_input_grad[6] else None
        params = (gamma, ctx.beta_ref if gamma is not None else None, cb)
        # straight into existing .grad buffers (FastStTrainer's flat gradient)
        acc = all(p is None or (p.is_leaf and p.grad is not None and p.grad.is_contiguous())
                  for p in params)
        bufs = [None if p is None else (p.grad if acc else torch.empty(c, device=x.device))
                for p in params]
        ga = ops.ARENA.take(x.device)
        beta = ctx.beta_ref
        du = ops.instnorm_bwd(_c(dy), None if beta is None else beta.detach(), x, res,
                              None if gamma is None else gamma.detach(),
                              mean, rstd, relu=ctx.relu, dgamma=bufs[0], dbeta=bufs[1],
                              dbias_in=bufs[2], accumulate=acc, out_amax=ga)
        ops.ARENA.annotate(du, ga)
        dg, db, dcb = (None, None, None) if acc else bufs
        dres = None
        if ctx.has_res:
            if ctx.res_link is not None and ctx.res_link.accepted and ctx.needs_input_grad[1]:
                ctx.res_link.g = du  # added by the block's first conv (ResLink)
            else:
                dres = du
        return du, dres, dg, db, None, None, dcb, None


def instance_norm(x, gamma, beta, res=None, eps=1e-5, relu=False, conv_bias=None,
                  res_link=None):
    return InstanceNormFn.apply(x, res, gamma, beta, eps, relu, conv_bias, res_link)


# ----------------------------------------------------------------------- losses
class GramFn(torch.autograd.Function):
    """StyleLoss.gram_matrix: G = F Fᵀ / (C·H·W) (stransfer/network.py:92-108)."""

    @staticmethod
    def forward(ctx, z):
        z = _c(z)
        ctx.save_for_backward(z)
        return ops.gram(z)

    @staticmethod
    def backward(ctx, dG):
        (z,) = ctx.saved_tensors
        b, c = z.shape[:2]
        n = z[0].numel()
        cp = ops.coef_pitch(c)
        # dz = (dG + dGᵀ) F / N as a per-image 1x1 MFMA conv
        coef = torch.zeros((b, cp, cp), device=z.device, dtype=torch.float32)
        coef[:, :c, :c] = (dG + dG.transpose(1, 2)) / n
        return ops.gram_bwd(coef, z)


class StyleLossFn(torch.autograd.Function):
    """mean((gram(z) - T)^2) (StyleLoss.forward, stransfer/network.py:110-123)."""

    @staticmethod
    def forward(ctx, z, target):
        z = _c(z)
        loss, coef = ops.style_loss(z, _c(target.detach()), weight=1.0)
        ctx.save_for_backward(z, coef)
        return loss

    @staticmethod
    def backward(ctx, g):
        z, coef = ctx.saved_tensors
        return ops.gram_bwd(coef, z, acc_scale=_c(g.reshape(1))), None


class MSELossFn(torch.autograd.Function):
    """F.mse_loss(x, target) (ContentLoss.forward, stransfer/network.py:155-164)."""

    @staticmethod
    def forward(ctx, x, target):
        x, target = _c(x), _c(target.detach())
        out = ops.mse(x, target)
        ctx.save_for_backward(x, target)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        x, t = ctx.saved_tensors
        return ops.diff_scale(x, t, 2.0 / x.numel(), s1=_c(g.reshape(1))), None


class FeatureLossFn(torch.autograd.Function):
    """mse(x, t)^2 / numel (FeatureReconstructionLoss.forward, :186-201)."""

    @staticmethod
    def forward(ctx, x, target):
        x, target = _c(x), _c(target.detach())
        # relu=False: the inputs are already what the tap sees
        out = torch.empty(2, device=x.device, dtype=torch.float32)
        ops.mse(x, target, mode=1, out=out)
        ctx.save_for_backward(x, target, out)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        x, t, out = ctx.saved_tensors
        n = float(x.numel())
        return ops.diff_scale(x, t, 4.0 / (n * n), s1=_c(g.reshape(1)), s2=out[1:2]), None


class TVLossFn(torch.autograd.Function):
    """get_total_variation_regularization_loss (stransfer/network.py:621-641)."""

    @staticmethod
    def forward(ctx, y, factor):
        y = _c(y)
        ctx.save_for_backward(y)
        ctx.factor = factor
        return ops.tv_loss(y, factor)

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        grad = torch.empty_like(y)
        ops.tv_loss(y, ctx.factor, grad=grad, gscale_dev=_c(g.reshape(1)))
        return grad, None


class TemporalLossFn(torch.autograd.Function):
    """VideoTransformNet.get_temporal_loss (stransfer/network.py:885-903):
    ||y - y_old|| / (||x - x_old|| + 1) * w, differentiable in y (the reference's
    old frames are detached tensors; content frames carry no gradient)."""

    @staticmethod
    def forward(ctx, y, y_old, x, x_old, weight):
        y, y_old = _c(y), _c(y_old.detach())
        out = ops.temporal_loss(y, y_old, _c(x.detach()), _c(x_old.detach()), weight)
        ctx.save_for_backward(y, y_old, out)
        ctx.weight = weight
        return out[0]

    @staticmethod
    def backward(ctx, g):
        y, y_old, out = ctx.saved_tensors
        dy = ops.temporal_loss_bwd(y, y_old, out, ctx.weight, g=_c(g.reshape(1)))
        return dy, None, None, None, None


class FastStLossFn(torch.autograd.Function):
    """The fast_st closure's scalar (stransfer/network.py:690-731):
        total = sw * sum(style) + cw * content + TV(y, tv_factor)
    in one pass: the loss weights are folded into the backward operators (vgg.py
    folded mode: no per-loss scale vector, the content term rides on A_4), the TV loss
    and its gradient come from one kernel in the forward, and the weighted total is
    summed in the same launch as the five style losses.  The backward computes the
    gradient for a unit upstream gradient and scales it by the device-side g (no
    host sync), so `k * total` or a weighted sum with other terms is exact too."""

    @staticmethod
    def forward(ctx, y, c4, feat, targets, sw, cw, tv_factor):
        y = _c(y)
        dev = y.device
        st = V.LossState()
        # the amax groups of the loss network from the training step's arena (zeroed by its
        # one fill at the step's start) instead of a fill of their own
        st.amax = ops.ARENA.take_span(V.LOSS_AMAX_GROUPS, dev)
        st.amax_cleared = st.amax is not None
        st.losses = torch.empty(V.N_LOSSES + 2, device=dev, dtype=torch.float32)
        st.fmean = st.losses[6:8]
        tvg = torch.empty_like(y)  # MINUS the TV gradient (see backward)
        ops.tv_loss(y, tv_factor, grad=tvg, gscale=-1.0, out=st.losses[8])
        total = torch.empty((), device=dev, dtype=torch.float32)
        V.loss_forward(feat, targets, y, _c(c4), st=st, folded_weights=(sw, cw), total=total,
                       extra_slot=True)
        ctx.st, ctx.feat, ctx.tvg = st, feat, tvg
        return total

    @staticmethod
    def backward(ctx, g):
        dx = V.loss_backward(ctx.feat, ctx.st, feature_grad=False)
        # dx = g * (d(VGG losses) + d(TV)) in one launch: g * (dx - (-dTV))
        ops.diff_scale(dx, ctx.tvg, 1.0, s1=g.reshape(1), out=dx)
        ctx.st = ctx.tvg = None
        return dx, None, None, None, None, None, None


class VGGLossFn(torch.autograd.Function):
    """All 7 StyleNetwork losses of a batch in one fused forward/backward:
    returns [style1..5, content, feature] for input x given the style targets and
    the content target c4 (engine: styletransfer_amd/vgg.py)."""

    @staticmethod
    def forward(ctx, x, c4, feat, targets, feature_grad=True):
        st = V.loss_forward(feat, targets, _c(x), _c(c4))
        ctx.st, ctx.feat, ctx.feature_grad = st, feat, feature_grad
        return V.loss_values(st).clone()

    @staticmethod
    def backward(ctx, g):
        dx = V.loss_backward(ctx.feat, ctx.st, _c(g), feature_grad=ctx.feature_grad)
        ctx.st = None
        return dx, None, None, None, None
