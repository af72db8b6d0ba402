"""Functional wrappers over libstx (include/stx.h) for torch tensors.

PyTorch supplies device memory, the current HIP stream and autograd plumbing;
every arithmetic op here is a hand-written HIP kernel in libstx.so.  Nothing in
this module falls back to a torch/CPU implementation: a non-CUDA tensor or a
missing library raises.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import gc

import os

import torch

from . import _native as N
from ._native import ConvParams, check, lib

__all__ = [
    "conv_weight_dims", "conv_weight_prep", "conv_weight_prep16", "split_eligible", "amax",
    "conv2d", "conv_out_hw", "conv2d_wgrad",
    "bias_grad", "gram", "style_loss", "gram_bwd", "mse", "diff_scale", "loss_combine",
    "maxpool2x2", "maxpool2x2_bwd", "relupool_bwd", "relu", "relu_bwd", "adam_step",
    "instnorm_fwd", "instnorm_bwd", "upsample2x", "upsample2x_bwd", "tv_loss",
    "temporal_loss", "temporal_loss_bwd",
]


def _p(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _req(t: torch.Tensor, name: str = "tensor"):
    if not t.is_cuda:
        raise N.NativeError(f"{name}: the HIP path needs a device tensor (got {t.device}); "
                            "there is no CPU fallback")
    if t.dtype != torch.float32:
        raise N.NativeError(f"{name}: fp32 required (got {t.dtype})")
    if not t.is_contiguous():
        raise N.NativeError(f"{name}: contiguous NCHW required")
    return t


class _Workspace:
    """Per-device scratch buffer, grown on demand.  All users are stream-ordered
    on the same stream and finish with the scratch inside one C call.

    A captured hipGraph (GatysEngine, FastStTrainer.capture, FrameEngine) bakes the
    scratch pointer of its capture into its kernels, so a buffer is never freed
    once handed out: when a larger one is needed the old one is retired, not
    released to the caching allocator (growth is geometric, so the retired
    buffers sum to less than the live one)."""

    def __init__(self):
        self.buf = {}
        self.retired = []

    def get(self, nbytes: int, device) -> tuple:
        nbytes = max(int(nbytes), 256)
        key = (device.index if isinstance(device, torch.device) else device)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            size = max(nbytes, 1 << 20) if b is None else max(nbytes, 2 * b.numel())
            if b is not None:
                self.retired.append(b)
            b = torch.empty(size, dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b.data_ptr(), b.numel()


WS = _Workspace()
WS_SIDE = _Workspace()  # the weight-gradient side stream's own scratch (SideStream)


class SideStream:
    """Weight gradients off the data-gradient chain.  In a training step's backward
    (train.FastStTrainer / VideoTrainer between begin() and end()) every conv's dW --
    which nothing in the backward reads -- runs on a side stream that waits for the
    work issued so far (dy is ready), while the data gradients continue on the main
    stream; end() joins the side stream back before the gradient exchange / Adam.  The
    small B=8 grids of the ImageTransformNet (2 blocks per CU) leave room for a
    concurrent kernel.  The side work has its own scratch (WS_SIDE) and keeps its
    inputs referenced until the join (no cross-stream reuse of their memory, eager or
    captured).  Opt-in (STX_WGRAD_SIDE=1) until measured."""

    def __init__(self):
        self.active = False
        self.streams = {}
        self.stream = None
        self.keep = []

    def begin(self, device):
        import os
        if N.knob("STX_WGRAD_SIDE", "0") != "1":
            return
        key = torch.device(device).index or 0
        if key not in self.streams:
            self.streams[key] = torch.cuda.Stream(device)
        self.stream = self.streams[key]
        self.active = True
        self.keep = []

    def on_side(self):
        return self.active and torch.cuda.current_stream() == self.stream

    def run(self, fn, *keep):
        if not self.active:
            return fn()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            r = fn()
        self.keep.extend(t for t in keep if t is not None)
        return r

    def end(self):
        if self.active:
            torch.cuda.current_stream().wait_stream(self.stream)
            self.keep = []
            self.active = False


SIDE = SideStream()


def _scratch():
    return WS_SIDE if SIDE.on_side() else WS


@contextlib.contextmanager
def graph_capture(graph, **kw):
    """torch.cuda.graph(graph, **kw) with Python's cyclic garbage collector held off for
    the capture (after one collection): a CUDAGraph left in a reference cycle by earlier
    work (a finished engine) and collected while this stream captures would be destroyed
    mid-capture, which HIP refuses (hipErrorStreamCaptureUnsupported -> abort)."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(graph, **kw):
            yield
    finally:
        if was:
            gc.enable()


class AmaxArena:
    """Pre-zeroed amax groups for producers that annotate their outputs (InstanceNorm
    forward/backward -> the next split conv's input scale).  A training step calls
    begin() (one fill of all groups) and end(); outside a step take() returns None
    and consumers compute max|x| themselves.  Annotations carry the arena epoch, so a
    tensor kept across steps is never trusted with a re-zeroed group."""

    def __init__(self, groups=128):
        self.groups = groups
        self.buf = None
        self.i = 0
        self.epoch = 0
        self.active = False

    def begin(self, device):
        dev = torch.device(device)
        if self.buf is None or self.buf.device != dev:
            self.buf = torch.zeros((self.groups, N.STX_AMAX_SLOTS), device=dev,
                                   dtype=torch.float32)
        else:
            self.buf.zero_()
        self.i = 0
        self.epoch += 1
        self.active = True

    def end(self):
        self.active = False

    def take(self, device):
        if not self.active or self.i >= self.groups or self.buf.device != device:
            return None
        g = self.buf[self.i]
        self.i += 1
        return g

    def take_span(self, k, device):
        """k consecutive zeroed groups as one flat slot vector (vgg.slot layout)."""
        if not self.active or self.i + k > self.groups or self.buf.device != device:
            return None
        g = self.buf[self.i:self.i + k].view(-1)
        self.i += k
        return g

    def annotate(self, t, g):
        if g is not None:
            t._stx_amax = (g, self.epoch)
        return t

    def lookup(self, t):
        a = getattr(t, "_stx_amax", None)
        if a is None or not self.active or a[1] != self.epoch:
            return None
        return a[0]


ARENA = AmaxArena()


class ParamGradBatch:
    """Deferred InstanceNorm parameter reductions of one training step: between
    begin() and flush() each instnorm_bwd given dgamma/dbeta/dbias_in keeps its
    per-plane partials in a buffer of its own and records a job; flush() reduces all
    of them in one launch (stx_instnorm_param_grads).  Outside a step the reductions
    run per call."""

    def __init__(self):
        self.active = False
        self.jobs, self.keep = [], []

    def begin(self):
        self.active = True
        self.jobs, self.keep = [], []

    def add(self, parts, n, c, dgamma, dbeta, dbias, accumulate):
        self.keep.append(parts)
        self.jobs.append(N.PGradJob(parts.data_ptr(), _p(dgamma), _p(dbeta), _p(dbias), n, c,
                                    int(accumulate), 0))
        if len(self.jobs) == N.STX_PGRAD_MAX:
            self._launch()

    def _launch(self):
        if self.jobs:
            arr = (N.PGradJob * len(self.jobs))(*self.jobs)
            check(lib().stx_instnorm_param_grads(arr, len(self.jobs), _stream()),
                  "stx_instnorm_param_grads")
        self.jobs, self.keep = [], []

    def flush(self):
        self._launch()
        self.active = False


PGRADS = ParamGradBatch()


# ----------------------------------------------------------------------- conv
def conv_weight_dims(cin, cout, ks):
    a, b = C.c_int(), C.c_int()
    check(lib().stx_conv_weight_dims(cin, cout, ks, C.byref(a), C.byref(b)), "weight_dims")
    return a.value, b.value


def conv_weight_prep(w: torch.Tensor, transpose: bool = False) -> torch.Tensor:
    """[cout][cin][k][k] -> k-major GEMM slab (transpose=True: data-gradient slab)."""
    _req(w, "weight")
    cout, cin, ks, _ = w.shape
    gin, gout = (cout, cin) if transpose else (cin, cout)
    cp, op = conv_weight_dims(gin, gout, ks)
    wt = torch.empty((cp * ks * ks, op), device=w.device, dtype=torch.float32)
    check(lib().stx_conv_weight_prep(w.data_ptr(), wt.data_ptr(), cout, cin, ks, int(transpose),
                                     _stream()), "conv_weight_prep")
    return wt


def conv_weight_prep16(w: torch.Tensor, transpose: bool = False):
    """[cout][cin][3][3] -> (fp16 hi/lo split slab, device max|w|) for the split-MFMA
    path of stx_conv2d (transpose=True: the data-gradient slab)."""
    _req(w, "weight")
    cout, cin, ks, _ = w.shape
    L = lib()
    nb = L.stx_conv_weight16_bytes(cin, cout, ks, int(transpose))
    if nb == 0:
        raise N.NativeError(f"no fp16-split slab for a {ks}x{ks} conv")
    wt16 = torch.empty(nb, device=w.device, dtype=torch.uint8)
    w_amax = torch.empty(N.STX_AMAX_SLOTS, device=w.device, dtype=torch.float32)
    check(L.stx_conv_weight_prep16(w.data_ptr(), wt16.data_ptr(), w_amax.data_ptr(), cout, cin,
                                   ks, int(transpose), _stream()), "conv_weight_prep16")
    return wt16, w_amax


def conv_weight_prep16_up(w: torch.Tensor):
    """[cout][cin][3][3] -> (parity-class split slab, device max|w|) of a conv over a
    nearest x2 upsampled input (stx_conv_weight_prep16_up; conv2d(wt16_up=...))."""
    _req(w, "weight")
    cout, cin, ks, _ = w.shape
    assert ks == 3, ks
    L = lib()
    slab = torch.empty(L.stx_conv_weight16up_bytes(cin, cout), device=w.device, dtype=torch.uint8)
    w_amax = torch.empty(N.STX_AMAX_SLOTS, device=w.device, dtype=torch.float32)
    check(L.stx_conv_weight_prep16_up(w.data_ptr(), slab.data_ptr(), w_amax.data_ptr(), cout,
                                      cin, _stream()), "conv_weight_prep16_up")
    return slab, w_amax


def conv_weight_compose16(coef, coef_amax, w: torch.Tensor, w_amax, out_amax, scale=None,
                          out=None):
    """The data-gradient split slab of w' = scale * A w (A = coef [cout][pitch], one image's
    Gram-backward operator, coef_amax >= max|A|; w [cout][cin][3][3], w_amax >= max|w|):
    conv^T_w(A z) = conv^T_{w'}(z) (stx_conv_weight_compose16, one launch).  out_amax (an
    amax group) receives the slab's scale bound; the conv takes wt16=(slab, out_amax).
    out: the slab buffer to reuse.  Returns the slab."""
    _req(w, "weight")
    _req(coef, "coef")
    cout, cin, ks, _ = w.shape
    assert ks == 3 and coef.shape[-2] == cout and coef.numel() == cout * coef.shape[-1], coef.shape
    L = lib()
    if out is None:
        out = torch.empty(L.stx_conv_weight16_bytes(cin, cout, ks, 1), device=w.device,
                          dtype=torch.uint8)
    check(L.stx_conv_weight_compose16(coef.data_ptr(), coef.shape[-1], coef_amax.data_ptr(),
                                      w.data_ptr(), w_amax.data_ptr(), cout, cin, _p(scale),
                                      out.data_ptr(), out_amax.data_ptr(), _stream()),
          "stx_conv_weight_compose16")
    return out


def conv_weight_prep16_pair(w: torch.Tensor):
    """(forward slab, data-gradient slab), sharing one device max|w| (two launches)."""
    _req(w, "weight")
    cout, cin, ks, _ = w.shape
    L = lib()
    wt16 = torch.empty(L.stx_conv_weight16_bytes(cin, cout, ks, 0), device=w.device,
                       dtype=torch.uint8)
    wtT16 = torch.empty(L.stx_conv_weight16_bytes(cin, cout, ks, 1), device=w.device,
                        dtype=torch.uint8)
    w_amax = torch.empty(N.STX_AMAX_SLOTS, device=w.device, dtype=torch.float32)
    check(L.stx_conv_weight_prep16_pair(w.data_ptr(), wt16.data_ptr(), wtT16.data_ptr(),
                                        w_amax.data_ptr(), cout, cin, ks, _stream()),
          "conv_weight_prep16_pair")
    return (wt16, w_amax), (wtT16, w_amax)


class TrainedSlabs:
    """The GEMM weight slabs of a trained network's conv layers, re-prepped after
    every parameter update in two launches (stx_conv_weight_prep_batch) instead of
    ~2 per slab.  For each layer the slabs the forward and the input-gradient kernels
    of autograd.Conv2dFn will select: the fp16 hi/lo split slab (shapes the split
    kernel takes) or the fp32 k-major slab, for the forward and the transposed
    data-gradient GEMM; forward and data-gradient split slabs share one max|w| group.

    `prep()` enqueues the batch and hands each layer `_train_slabs = (key, wt, wt16,
    wtT, wtT16, wt16_up)` keyed on the weight's (pointer, version): layers.Conv2d uses
    the slabs only while the key matches, so a weight changed behind the trainer's back
    falls back to per-call preps.  wt16_up: the parity-class slab of a conv that reads a
    nearest x2 upsampled input (layers.Conv2d._up_input), sharing the max|w| group."""

    def __init__(self, convs):
        self.convs = list(convs)
        self.generation = 0
        self._retired = []
        self.slabs = None
        self._build()

    def _build(self):
        split = N.knob("STX_CONV_SPLIT", "1") != "0"
        L = lib()
        jobs = []
        if self.slabs is not None:
            # a hipGraph captured earlier still holds the old slab / job pointers: keep
            # them alive (as _Workspace retires scratch buffers) and bump the generation
            # so the owner re-captures (train.FastStTrainer checks it before a replay)
            self._retired.append((self.slabs, self._jobs))
            self.generation += 1
        self.slabs = []
        for conv in self.convs:
            w = conv.weight
            cout, cin, ks, _ = w.shape
            stride, pad = conv.stride[0], conv.padding[0]
            f16 = split and pad == 1 and split_eligible(cin, cout, ks, stride)
            b16 = split and pad == 1 and split_eligible(cout, cin, ks, 1)
            dev = w.device
            am = torch.empty(N.STX_AMAX_SLOTS, device=dev, dtype=torch.float32) \
                if (f16 or b16) else None
            out = []
            for t, is16 in ((0, f16), (1, b16)):
                if is16:
                    slab = torch.empty(L.stx_conv_weight16_bytes(cin, cout, ks, t), device=dev,
                                       dtype=torch.uint8)
                    jobs.append(N.WprepJob(w.data_ptr(), slab.data_ptr(), am.data_ptr(),
                                           N.STX_WPREP_F16, cout, cin, ks, t, 0))
                    out.append((None, (slab, am)))
                else:
                    gin, gout = (cout, cin) if t else (cin, cout)
                    cp, op = conv_weight_dims(gin, gout, ks)
                    slab = torch.empty((cp * ks * ks, op), device=dev, dtype=torch.float32)
                    jobs.append(N.WprepJob(w.data_ptr(), slab.data_ptr(), None,
                                           N.STX_WPREP_F32, cout, cin, ks, t, 0))
                    out.append((slab, None))
            up = None
            if f16 and stride == 1 and ks == 3 and getattr(conv, "_up_input", False) and \
                    N.knob("STX_UPAR", "1") != "0":
                up = torch.empty(L.stx_conv_weight16up_bytes(cin, cout), device=dev,
                                 dtype=torch.uint8)
                jobs.append(N.WprepJob(w.data_ptr(), up.data_ptr(), am.data_ptr(),
                                       N.STX_WPREP_F16UP, cout, cin, ks, 0, 0))
            self.slabs.append((w.data_ptr(), out[0][0], out[0][1], out[1][0], out[1][1], up))
        if len(jobs) > N.STX_WPREP_MAX:
            raise N.NativeError(f"{len(jobs)} weight slabs > STX_WPREP_MAX")
        self._jobs = (N.WprepJob * len(jobs))(*jobs)
        self._njobs = len(jobs)

    def release_retired(self):
        """Drop the slabs of earlier generations: call after the owner re-captured its
        graphs (a graph of an older generation refuses to replay, so nothing reads
        them any more)."""
        self._retired.clear()

    def prep(self):
        if any(c.weight.data_ptr() != s[0] for c, s in zip(self.convs, self.slabs)):
            self._build()  # a parameter was re-homed
        if self._njobs:
            check(lib().stx_conv_weight_prep_batch(self._jobs, self._njobs, _stream()),
                  "conv_weight_prep_batch")
        for c, (_, wt, wt16, wtT, wtT16, up) in zip(self.convs, self.slabs):
            w = c.weight
            c._train_slabs = ((w.data_ptr(), w._version, w.device), wt, wt16, wtT, wtT16,
                              None if up is None else (up, wt16[1]))


_S2_FWD = N.knob("STX_S2_FWD", "1") != "0"


def split_eligible(cin, cout, ks, stride=1):
    """Shapes stx_conv2d runs on the fp16 hi/lo split MFMA kernel (conv16.hip)."""
    # stride 2 (raw input only): STX_S2_FWD=0 keeps it on the fp32 kernel (A/B switch)
    return ks == 3 and cin >= 16 and cout > 4 and (
        stride == 1 or (stride == 2 and _S2_FWD))


def amax(x: torch.Tensor, out=None):
    """max|x| as an amax group (STX_AMAX_SLOTS floats whose max is the value)."""
    _req(x, "x")
    if out is None:
        out = torch.empty(N.STX_AMAX_SLOTS, device=x.device, dtype=torch.float32)
    check(lib().stx_amax(x.data_ptr(), x.numel(), out.data_ptr(), _stream()), "stx_amax")
    return out


def vdot(a, b, out, mul=None, add=None, sgn=1.0, op=0):
    """*out = add + sgn * mul * r, r = dot(a, b) (op 0), sum|a| (1), max|a| (2); a
    fixed-order reduction (stx_vec_reduce).  out/mul/add: 1-element device tensors."""
    _req(a, "a")
    L = lib()
    wp, wn = WS.get(L.stx_vec_ws(), a.device)
    check(L.stx_vec_reduce(a.data_ptr(), _p(b), a.numel(), op, out.data_ptr(), _p(mul), _p(add),
                           float(sgn), wp, wn, _stream()), "stx_vec_reduce")
    return out


def virtual_hw(h, w, in_mode, hv=None, wv=None):
    if in_mode in (N.STX_IN_RAW, N.STX_IN_RELU):
        return h, w
    if in_mode == N.STX_IN_RELU_POOL2:
        return h // 2, w // 2
    if in_mode == N.STX_IN_UPSAMPLE2:
        return 2 * h, 2 * w
    return hv, wv  # DILATE2: explicit


def conv_out_hw(hv, wv, ks, stride, pad):
    return (hv + 2 * pad - ks) // stride + 1, (wv + 2 * pad - ks) // stride + 1


def conv2d(x, wt, cin, cout, ks, stride=1, pad=None, in_mode=N.STX_IN_RAW, bias=None,
           out=None, mask=None, aux=None, aux_scale=0.0, acc_scale=None, accumulate=False,
           relu_out=False, wt_batch_stride=0, hv=None, wv=None, p2_z=None, p2_coef=None,
           p2_scale=None, up_dp=None, up_z=None, wt16=None, in_amax=None, out_amax=None,
           pool_out=None, p2_amax=None, split_1x1=False, gram_part=None, pool_sum=False,
           gram_cnt=None, p2_wt_amax=None, mse_ref=None, mse_parts=None, wt16_up=None,
           unpool_out=None, pool_only=False):
    """stx_conv2d on x [n][cin][h][w] with a prepped slab `wt`.
    p2_z/p2_coef: fused Gram-backward phase (value += s2 * A[n] . p2_z[n]);
    up_dp/up_z: fused ReLU+MaxPool2d backward epilogue.
    wt16=(slab, w_amax) from conv_weight_prep16 selects the fp16 hi/lo split MFMA
    kernel for eligible shapes; in_amax (device >= max|x|) is computed when absent;
    out_amax (device scalar, zeroed by the caller) receives max|out|; pool_out
    [n][cout][ho/2][wo/2] receives maxpool2x2(relu(out)) (split path, wo > 32);
    gram_part [n * conv_gram_tiles(...) * 4096] receives the fused per-tile Gram
    partials of out (stx_conv_params.gram_part); pool_sum: pool_out receives the 2x2
    SUM of the output instead and the full-resolution output is not written (returned:
    pool_out) -- the nearest-x2 upsampling backward fused into a data gradient.
    p2_wt_amax: amax group >= max|p2_coef| over the batch (a FinalizeBatch job's
    coef_amax): the split path's Gram-backward phase then runs on the fp16 split MFMA.
    mse_ref/mse_parts (with gram_part, cout 128): the content target and the per-tile
    content / feature MSE sums of the output (stx_conv_params.mse_ref).
    wt16_up=(slab, w_amax) from conv_weight_prep16_up: an upsampled-input conv with the
    plain epilogue runs as four output-parity 2x2 convs (stx_conv_params.wt16_up).
    unpool_out=(z, coef, coef_amax, z_amax, scale): the result d is the gradient of
    maxpool2x2(relu(z)) and `out` [n][cout][2 ho][2 wo] receives unpool(d) [z > 0] +
    scale * A[n] . z (stx_conv_params.unpool_out: a pooled tap's ReLU+MaxPool and Gram
    backward in this data gradient's epilogue).
    pool_only (with pool_out, split path): the full-resolution output is not written
    (stx_conv_params.y = NULL); returns pool_out."""
    _req(x, "x")
    n, c, h, w = x.shape
    assert c == cin, (c, cin)
    if pad is None:
        pad = ks // 2
    hv, wv = virtual_hw(h, w, in_mode, hv, wv)
    ho, wo = conv_out_hw(hv, wv, ks, stride, pad)
    if pool_sum:
        assert pool_out is not None and out is None, "pool_sum writes pool_out only"
        out = pool_out  # p.y must be set; the kernel never writes it with pool_sum
    elif unpool_out is not None:
        oshape = (n, cout, 2 * ho, 2 * wo)
        if out is None:
            out = torch.empty(oshape, device=x.device, dtype=torch.float32)
        _req(out, "out")
        assert out.shape == oshape, (out.shape, oshape)
    elif out is None:
        out = torch.empty((n, cout, ho, wo), device=x.device, dtype=torch.float32)
    else:
        _req(out, "out")
        assert out.shape == (n, cout, ho, wo), (out.shape, (n, cout, ho, wo))
    cp, op = conv_weight_dims(cin, cout, ks)
    p = ConvParams(x=x.data_ptr(), wt=_p(wt), bias=_p(bias), y=out.data_ptr(),
                   mask=_p(mask), aux=_p(aux), aux_scale=float(aux_scale),
                   acc_scale=_p(acc_scale), accumulate=int(accumulate), relu_out=int(relu_out),
                   n=n, cin=cin, h=h, w=w, cout=cout, ks=ks, stride=stride, pad=pad,
                   in_mode=in_mode, hv=hv, wv=wv, ho=ho, wo=wo, cin_pad=cp, cout_pad=op,
                   wt_batch_stride=int(wt_batch_stride))
    if p2_z is not None:
        assert p2_coef is not None and p2_coef.shape[-1] == op, (p2_coef.shape, op)
        p.p2_z, p.p2_wt, p.p2_scale = p2_z.data_ptr(), p2_coef.data_ptr(), _p(p2_scale)
        p.p2_c = p2_z.shape[1]
        p.p2_wt_batch_stride = p2_coef.shape[-1] * p2_coef.shape[-2]
    if up_dp is not None:
        p.up_dp, p.up_z = up_dp.data_ptr(), up_z.data_ptr()
    if wt16 is not None and split_eligible(cin, cout, ks, stride) and wt_batch_stride == 0:
        if in_amax is None:
            in_amax = amax(x)
        p.wt16, p.w_amax, p.in_amax = wt16[0].data_ptr(), wt16[1].data_ptr(), in_amax.data_ptr()
        if wt16_up is not None and in_mode == N.STX_IN_UPSAMPLE2 and ks == 3 and stride == 1 \
                and pad == 1 and wo > 32 and (hv, wv) == (2 * h, 2 * w) and not any(
                    v is not None for v in (mask, aux, acc_scale, p2_z, up_dp, pool_out,
                                            gram_part)) and not accumulate:
            p.wt16_up, p.w_amax = wt16_up[0].data_ptr(), wt16_up[1].data_ptr()
        if p2_z is not None:
            p.p2_amax = (p2_amax if p2_amax is not None else amax(p2_z)).data_ptr()
            if p2_wt_amax is not None:
                p.p2_wt_amax = p2_wt_amax.data_ptr()
    elif split_1x1:
        # Gram backward as the split phase alone (per-image weights, include/stx.h)
        assert ks == 1 and wt_batch_stride and mask is None and p2_z is None
        p.wt16 = 1
        p.in_amax = (in_amax if in_amax is not None else amax(x)).data_ptr()
    if unpool_out is not None:
        uz, ucoef, ucoef_amax, uz_amax, uscale = unpool_out
        _req(uz, "unpool z")
        assert uz.shape == out.shape and ucoef.shape[-1] == op, (uz.shape, ucoef.shape, op)
        p.unpool_out = 1
        p.up_z, p.p2_wt, p.p2_scale = uz.data_ptr(), ucoef.data_ptr(), _p(uscale)
        p.p2_c = uz.shape[1]
        p.p2_wt_batch_stride = ucoef.shape[-1] * ucoef.shape[-2]
        p.p2_amax = (uz_amax if uz_amax is not None else amax(uz)).data_ptr()
        p.p2_wt_amax = ucoef_amax.data_ptr()
    if in_amax is not None and not p.in_amax:
        # the non-split kernels that take an input bound (convfew.hip's split 64->3
        # data gradient) read it too; the others ignore it
        p.in_amax = in_amax.data_ptr()
    if out_amax is not None:
        p.out_amax = out_amax.data_ptr()
    if pool_out is not None:
        _req(pool_out, "pool_out")
        assert pool_out.shape == (n, cout, ho // 2, wo // 2), pool_out.shape
        p.pool_out = pool_out.data_ptr()
        p.pool_sum = int(bool(pool_sum))
    assert mse_ref is None or gram_part is not None, "mse_ref rides on the fused Gram"
    if gram_part is not None:
        _req(gram_part, "gram_part")
        nt = lib().stx_conv_gram_tiles(C.byref(p))
        ng = lib().stx_conv_gram_groups(C.byref(p)) if gram_cnt is not None else 0
        ntu = gram_tile_units(cout)
        assert nt > 0 and gram_part.numel() >= n * (ntu * nt + ng) * 4096, \
            (nt, ng, gram_part.numel())
        p.gram_part = gram_part.data_ptr()
        if mse_ref is not None:
            _req(mse_ref, "mse_ref")
            _req(mse_parts, "mse_parts")
            assert mse_ref.shape == out.shape and mse_parts.numel() >= 2 * n * nt, \
                (mse_ref.shape, mse_parts.numel(), n * nt)
            p.mse_ref, p.mse_parts = mse_ref.data_ptr(), mse_parts.data_ptr()
        if gram_cnt is not None:
            assert gram_cnt.is_cuda and gram_cnt.dtype == torch.int32 and \
                gram_cnt.numel() >= n * ng, (gram_cnt.dtype, gram_cnt.numel(), n * ng)
            p.gram_cnt = gram_cnt.data_ptr()
    if pool_only:
        assert pool_out is not None and not pool_sum and gram_part is None, "pool_only"
        p.y = None
        out = pool_out
    check(lib().stx_conv2d(C.byref(p), _stream()), "stx_conv2d")
    return out


def gram_tile_units(c):
    """64 x 64 tiles of the upper triangle of a c x c Gram (the partial slab's U)."""
    nt = (c + 63) // 64
    return nt * (nt + 1) // 2


def conv_gram_tiles(cin, cout, ho, wo, n=1, in_mode=N.STX_IN_RAW):
    """Gram partials per image (one per output tile) of a split 3x3 stride-1 conv with a
    fused Gram over a batch of n (stx_conv_gram_tiles; 0: not fusable)."""
    p = ConvParams(cin=cin, cout=cout, ks=3, stride=1, pad=1, ho=ho, wo=wo, wt16=2, n=n,
                   in_mode=in_mode)
    return lib().stx_conv_gram_tiles(C.byref(p))


def conv_gram_groups(cin, cout, ho, wo, n=1, in_mode=N.STX_IN_RAW):
    """In-kernel group sums per image of the fused Gram with gram_cnt
    (stx_conv_gram_groups: ceil(tiles / STX_GRAM_GROUP); 0: not fusable).  The slab then
    holds n * (tiles + groups) * 4096 floats: the per-tile scratch, then the group sums
    (conv2d(gram_part=slab, gram_cnt=counters); style_loss_from_parts on the sums)."""
    p = ConvParams(cin=cin, cout=cout, ks=3, stride=1, pad=1, ho=ho, wo=wo, wt16=2, n=n,
                   in_mode=in_mode)
    return lib().stx_conv_gram_groups(C.byref(p))


def conv2d_wgrad(x, dy, cin, cout, ks, stride=1, pad=None, in_mode=N.STX_IN_RAW, dw=None,
                 accumulate=False, split=True, x_amax=None, dy_amax=None):
    """dW (+)= sum dy * V(x); 3x3 stride-1 / stride-2 shapes run on the fp16 hi/lo split
    MFMA (stx_conv2d_wgrad16[_s2]) unless split=False or STX_CONV_SPLIT=0."""
    _req(x, "x")
    _req(dy, "dy")
    n, _, h, w = x.shape
    if pad is None:
        pad = ks // 2
    hv, wv = virtual_hw(h, w, in_mode)
    ho, wo = dy.shape[2], dy.shape[3]
    if dw is None:
        dw = torch.empty((cout, cin, ks, ks), device=x.device, dtype=torch.float32)
    L = lib()
    import os
    split = split and N.knob("STX_CONV_SPLIT", "1") != "0"
    if split and ks == 9 and stride == 1 and pad == 4 and in_mode == N.STX_IN_RAW:
        # ITN conv0 / conv22: the 3-channel side expanded per tap row (wgrad9.hip)
        need9 = L.stx_conv2d_wgrad_few16_ws(n, cin, cout, ks, h, w)
        if need9 and ho == h and wo == w:
            xa = x_amax if x_amax is not None else amax(x)
            da = dy_amax if dy_amax is not None else amax(dy)
            wp, wn = _scratch().get(need9, x.device)
            check(L.stx_conv2d_wgrad_few16(x.data_ptr(), dy.data_ptr(), dw.data_ptr(),
                                           int(accumulate), n, cin, h, w, cout, ks, pad,
                                           xa.data_ptr(), da.data_ptr(), wp, wn, _stream()),
                  "stx_conv2d_wgrad_few16")
            return dw
    if split and ks == 3 and stride == 1 and pad == 1:
        need16 = L.stx_conv2d_wgrad16_ws(n, cin, cout, in_mode, ho, wo)
        if need16:
            _req(dy, "dy")
            xa = x_amax if x_amax is not None else amax(x)
            da = dy_amax if dy_amax is not None else amax(dy)
            wp, wn = _scratch().get(need16, x.device)
            check(L.stx_conv2d_wgrad16(x.data_ptr(), dy.data_ptr(), dw.data_ptr(),
                                       int(accumulate), n, cin, h, w, cout, in_mode, ho, wo,
                                       xa.data_ptr(), da.data_ptr(), wp, wn, _stream()),
                  "stx_conv2d_wgrad16")
            return dw
    if split and ks == 3 and stride == 2 and pad == 1 and in_mode == N.STX_IN_RAW \
            and N.knob("STX_WG16_S2", "1") != "0" \
            and h == 2 * ho and w == 2 * wo:
        need16 = L.stx_conv2d_wgrad16_s2_ws(n, cin, cout, ho, wo)
        if need16:
            xa = x_amax if x_amax is not None else amax(x)
            da = dy_amax if dy_amax is not None else amax(dy)
            wp, wn = _scratch().get(need16, x.device)
            check(L.stx_conv2d_wgrad16_s2(x.data_ptr(), dy.data_ptr(), dw.data_ptr(),
                                          int(accumulate), n, cin, h, w, cout, ho, wo,
                                          xa.data_ptr(), da.data_ptr(), wp, wn, _stream()),
                  "stx_conv2d_wgrad16_s2")
            return dw
    need = L.stx_conv2d_wgrad_ws(n, cin, cout, ks, stride, ho, wo)
    wp, wn = _scratch().get(need, x.device)
    check(L.stx_conv2d_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), int(accumulate), n, cin,
                             h, w, cout, ks, stride, pad, in_mode, hv, wv, ho, wo, wp, wn,
                             _stream()), "stx_conv2d_wgrad")
    return dw


def bias_grad(dy, db=None, accumulate=False):
    _req(dy, "dy")
    n, c = dy.shape[:2]
    hw = dy[0, 0].numel()
    if db is None:
        db = torch.empty(c, device=dy.device, dtype=torch.float32)
    L = lib()
    wp, wn = WS.get(L.stx_bias_grad_ws(n, c), dy.device)
    check(L.stx_bias_grad(dy.data_ptr(), db.data_ptr(), n, c, hw, int(accumulate), wp, wn,
                          _stream()), "stx_bias_grad")
    return db


# ----------------------------------------------------------------------- gram
def gram(z, scale=None, z_amax=None):
    """G[b] = F F^T * scale (default 1/(C*H*W), StyleLoss.gram_matrix).  z_amax
    (device >= max|z|) selects the fp16 hi/lo split MFMA partials."""
    _req(z, "z")
    b, c = z.shape[:2]
    hw = z[0, 0].numel()
    if scale is None:
        scale = 1.0 / (c * hw)
    g = torch.empty((b, c, c), device=z.device, dtype=torch.float32)
    L = lib()
    wp, wn = WS.get(L.stx_gram_ws(b, c, hw), z.device)
    check(L.stx_gram(z.data_ptr(), g.data_ptr(), b, c, hw, float(scale), _p(z_amax), wp, wn,
                     _stream()),
          "stx_gram")
    return g


def coef_pitch(c):
    return lib().stx_gram_coef_pitch(c)


class FinalizeBatch:
    """Deferred Gram finalizes of one forward (stx_gram_finalize_batch): the style-loss ops
    given `fin=` append a job instead of launching their finalize; flush() runs them all
    in one launch.  The job structs (and what they point at, via `keep`) live until then."""

    def __init__(self):
        self.jobs, self.keep = [], []

    def new(self):
        j = N.GramFinJob()
        self.jobs.append(j)
        return j

    def flush(self):
        if self.jobs:
            arr = (N.GramFinJob * len(self.jobs))(*self.jobs)
            check(lib().stx_gram_finalize_batch(arr, len(self.jobs), _stream()),
                  "stx_gram_finalize_batch")
        self.jobs, self.keep = [], []


def style_loss(z, target, weight=1.0, diag_alpha=0.0, want_coef=True, g_out=None, loss=None,
               coef=None, z_amax=None, defer_ws=None, fin=None):
    """mean((gram(z) - target)^2) -> 0-d loss; coef = d(weight*loss)/dz operator.
    defer_ws (uint8 device buffer >= stx_gram_ws): the loss is not reduced here; its
    partials stay in defer_ws for loss_finalize (returns (LossPart, coef))."""
    _req(z, "z")
    _req(target, "target")
    b, c = z.shape[:2]
    hw = z[0, 0].numel()
    # target [c][c] / [1][c][c] broadcast over the batch (expand_as), or [b][c][c]
    tb = target.numel() == b * c * c and b > 1
    if not tb and target.numel() != c * c:
        raise ValueError(f"style target {tuple(target.shape)} cannot expand to ({b},{c},{c})")
    if loss is None and defer_ws is None:
        loss = torch.empty((), device=z.device, dtype=torch.float32)
    if want_coef and coef is None:
        cp = coef_pitch(c)
        coef = torch.empty((b, cp, cp), device=z.device, dtype=torch.float32)
    L = lib()
    need = L.stx_gram_ws(b, c, hw)
    if defer_ws is not None:
        assert defer_ws.numel() >= need, (defer_ws.numel(), need)
        wp, wn = defer_ws.data_ptr(), defer_ws.numel()
    else:
        wp, wn = WS.get(need, z.device)
    if fin is not None:  # finalize deferred to fin.flush()
        assert defer_ws is not None and g_out is None and want_coef
        check(L.stx_style_loss_deferred(z.data_ptr(), target.data_ptr(), coef.data_ptr(), b, c,
                                        hw, int(tb), float(weight), float(diag_alpha),
                                        _p(z_amax), wp, wn, C.byref(fin.new()), _stream()),
              "stx_style_loss_deferred")
    else:
        check(L.stx_style_loss(z.data_ptr(), target.data_ptr(), _p(g_out), _p(coef) if want_coef
                               else None, _p(loss), b, c, hw, int(tb), float(weight),
                               float(diag_alpha), _p(z_amax), wp, wn, _stream()), "stx_style_loss")
    if defer_ws is not None:
        npart = C.c_int()
        off = L.stx_style_loss_parts(b, c, hw, C.byref(npart))
        return (wp + off, npart.value, 1.0 / (b * c * c)), (coef if want_coef else None)
    return loss, (coef if want_coef else None)


def style_content_loss(z, target, content, mse_out, weight=1.0, diag_alpha=0.0, coef=None,
                       z_amax=None, defer_ws=None, fin=None):
    """style_loss(z, target, ..., defer_ws=...) and mse(z, content, mode=2, out=mse_out) in
    one pass over z where the Gram kernel allows it.  defer_ws >= stx_style_content_ws.
    Returns (deferred LossPart, coef)."""
    _req(z, "z")
    _req(target, "target")
    _req(content, "content")
    assert content.numel() == z.numel() and mse_out.numel() >= 3
    b, c = z.shape[:2]
    hw = z[0, 0].numel()
    tb = target.numel() == b * c * c and b > 1
    if not tb and target.numel() != c * c:
        raise ValueError(f"style target {tuple(target.shape)} cannot expand to ({b},{c},{c})")
    if coef is None:
        cp = coef_pitch(c)
        coef = torch.empty((b, cp, cp), device=z.device, dtype=torch.float32)
    L = lib()
    need = L.stx_style_content_ws(b, c, hw)
    assert defer_ws is not None and defer_ws.numel() >= need, need
    wp, wn = defer_ws.data_ptr(), defer_ws.numel()
    if fin is not None:
        check(L.stx_style_content_loss_deferred(z.data_ptr(), target.data_ptr(), coef.data_ptr(),
                                                b, c, hw, int(tb), float(weight),
                                                float(diag_alpha), _p(z_amax), content.data_ptr(),
                                                mse_out.data_ptr(), wp, wn, C.byref(fin.new()),
                                                _stream()), "stx_style_content_loss_deferred")
    else:
        check(L.stx_style_content_loss(z.data_ptr(), target.data_ptr(), coef.data_ptr(), None, b,
                                       c, hw, int(tb), float(weight), float(diag_alpha),
                                       _p(z_amax), content.data_ptr(), mse_out.data_ptr(), wp, wn,
                                       _stream()), "stx_style_content_loss")
    npart = C.c_int()
    off = L.stx_style_loss_parts(b, c, hw, C.byref(npart))
    return (wp + off, npart.value, 1.0 / (b * c * c)), coef


def style_loss_from_parts(gparts, nparts, b, c, hw, target, weight=1.0, diag_alpha=0.0,
                          coef=None, defer_ws=None, fin=None, mse_parts=None, mse_out=None):
    """style_loss from the fused Gram partials a conv wrote (conv2d(gram_part=...)):
    gparts [b][U][nparts][64][64] (U = 3 for c = 128, else 1).  mse_parts (the content
    tap: conv2d(mse_ref=content, mse_parts=...)) with mse_out [3]: the content, feature
    and feature-mse values as style_content_loss writes them, from the same launch.
    Returns (deferred LossPart, coef) as style_loss with defer_ws."""
    _req(gparts, "gram partials")
    _req(target, "target")
    if (mse_parts is None) != (mse_out is None):
        raise ValueError("mse_parts and mse_out go together")
    if mse_parts is not None:
        _req(mse_parts, "mse_parts")
        assert mse_parts.numel() >= 2 * b * nparts and mse_out.numel() >= 3
    tb = target.numel() == b * c * c and b > 1
    if not tb and target.numel() != c * c:
        raise ValueError(f"style target {tuple(target.shape)} cannot expand to ({b},{c},{c})")
    if coef is None:
        cp = coef_pitch(c)
        coef = torch.empty((b, cp, cp), device=gparts.device, dtype=torch.float32)
    L = lib()
    need = L.stx_gram_ws(b, c, hw)
    assert defer_ws is not None and defer_ws.numel() >= need, need
    wp, wn = defer_ws.data_ptr(), defer_ws.numel()
    if mse_parts is not None:
        if fin is not None:
            check(L.stx_style_content_loss_from_parts_deferred(
                gparts.data_ptr(), int(nparts), target.data_ptr(), coef.data_ptr(), b, c, hw,
                int(tb), float(weight), float(diag_alpha), mse_parts.data_ptr(),
                mse_out.data_ptr(), wp, wn, C.byref(fin.new()), _stream()),
                "stx_style_content_loss_from_parts_deferred")
        else:
            check(L.stx_style_content_loss_from_parts(
                gparts.data_ptr(), int(nparts), target.data_ptr(), coef.data_ptr(), None, b, c,
                hw, int(tb), float(weight), float(diag_alpha), mse_parts.data_ptr(),
                mse_out.data_ptr(), wp, wn, _stream()), "stx_style_content_loss_from_parts")
    elif fin is not None:
        check(L.stx_style_loss_from_parts_deferred(gparts.data_ptr(), int(nparts),
                                                   target.data_ptr(), coef.data_ptr(), b, c, hw,
                                                   int(tb), float(weight), float(diag_alpha), wp,
                                                   wn, C.byref(fin.new()), _stream()),
              "stx_style_loss_from_parts_deferred")
    else:
        check(L.stx_style_loss_from_parts(gparts.data_ptr(), int(nparts), target.data_ptr(), None,
                                          coef.data_ptr(), None, b, c, hw, int(tb), float(weight),
                                          float(diag_alpha), wp, wn, _stream()),
              "stx_style_loss_from_parts")
    npart = C.c_int()
    off = L.stx_style_loss_parts(b, c, hw, C.byref(npart))
    return (wp + off, npart.value, 1.0 / (b * c * c)), coef


def loss_finalize(parts, losses, extra=None, weights=None, total=None):
    """One launch: losses[i] = reduced deferred style-loss partials (parts from
    style_loss(defer_ws=...)), and optionally total = sum w_i losses_i + sum w extra."""
    lp = N.LossParts()
    assert len(parts) <= 8
    for i, (ptr, n, inv) in enumerate(parts):
        lp.parts[i], lp.nparts[i], lp.inv[i] = ptr, n, inv
    lp.k = len(parts)
    m = 0 if extra is None else extra.numel()
    w = None
    if weights is not None:
        w = (C.c_float * len(weights))(*[float(x) for x in weights])
    check(lib().stx_loss_finalize(C.byref(lp), losses.data_ptr(), _p(extra), m, w, _p(total),
                                  _stream()), "stx_loss_finalize")
    return losses


def gram_bwd_fused(coef, z, out=None, acc_scale=None, up_dp=None, aux=None, aux_scale=0.0,
                   out_amax=None, z_amax=None):
    """out = s*A[n].z[n] (+ unpool(up_dp)*(z>0)) (+ aux_scale*aux): the Gram backward
    as a 1x1 MFMA conv with the ReLU+MaxPool backward fused into its epilogue.
    z_amax (device >= max|z|) runs it on the fp16 hi/lo split MFMA."""
    b, c = z.shape[:2]
    return conv2d(z, coef, c, c, 1, pad=0, out=out, acc_scale=acc_scale, aux=aux,
                  aux_scale=aux_scale, wt_batch_stride=coef.shape[-1] * coef.shape[-2],
                  up_dp=up_dp, up_z=z if up_dp is not None else None, out_amax=out_amax,
                  in_amax=z_amax, split_1x1=z_amax is not None)


def gram_bwd(coef, z, dz=None, acc_scale=None, mask=None, aux=None, aux_scale=0.0,
             accumulate=False):
    _req(z, "z")
    b, c, h, w = z.shape
    if dz is None:
        dz = torch.empty_like(z)
    check(lib().stx_gram_bwd(coef.data_ptr(), z.data_ptr(), dz.data_ptr(), b, c, h, w,
                             _p(acc_scale), _p(mask), _p(aux), float(aux_scale), int(accumulate),
                             _stream()), "stx_gram_bwd")
    return dz


# ----------------------------------------------------------------------- mse etc
def mse(a, b, relu=False, mode=0, out=None, grad=None, gscale=1.0):
    """mode 0: F.mse_loss (mean); mode 1: FeatureReconstructionLoss (out[1] = mean)."""
    _req(a, "a")
    _req(b, "b")
    assert a.numel() == b.numel()
    n = a.numel()
    if out is None:
        out = torch.empty({0: 1, 1: 2, 2: 3}[mode], device=a.device, dtype=torch.float32)
    L = lib()
    wp, wn = WS.get(L.stx_mse_ws(n), a.device)
    check(L.stx_mse(a.data_ptr(), b.data_ptr(), n, int(relu), mode, out.data_ptr(), _p(grad),
                    float(gscale), wp, wn, _stream()), "stx_mse")
    return out


def diff_scale(a, b, s0, s1=None, s2=None, relu=False, out=None, accumulate=False):
    if out is None:
        out = torch.empty_like(a)
    check(lib().stx_diff_scale(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), float(s0),
                               _p(s1), _p(s2), int(relu), int(accumulate), _stream()),
          "stx_diff_scale")
    return out


def loss_combine(s, weights, out):
    k = len(weights)
    arr = (C.c_float * k)(*[float(x) for x in weights])
    check(lib().stx_loss_combine(s.data_ptr(), k, arr, out.data_ptr(), _stream()),
          "stx_loss_combine")
    return out


# ----------------------------------------------------------------------- pooling / relu
def maxpool2x2(x, relu_input=False, want_idx=True):
    _req(x, "x")
    n, c, h, w = x.shape
    y = torch.empty((n, c, h // 2, w // 2), device=x.device, dtype=torch.float32)
    idx = torch.empty(y.shape, device=x.device, dtype=torch.int64) if want_idx else None
    check(lib().stx_maxpool2x2_fwd(x.data_ptr(), y.data_ptr(), _p(idx), n * c, h, w,
                                   int(relu_input), _stream()), "stx_maxpool2x2_fwd")
    return y, idx


def maxpool2x2_bwd(dy, idx, h, w):
    n, c = dy.shape[:2]
    dx = torch.empty((n, c, h, w), device=dy.device, dtype=torch.float32)
    check(lib().stx_maxpool2x2_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), n * c, h, w,
                                   _stream()), "stx_maxpool2x2_bwd")
    return dx


def relupool_bwd(dp, z, out=None):
    n, c, h, w = z.shape
    if out is None:
        out = torch.empty_like(z)
    check(lib().stx_relupool_bwd(dp.data_ptr(), z.data_ptr(), out.data_ptr(), n * c, h, w,
                                 _stream()), "stx_relupool_bwd")
    return out


def relu(x):
    _req(x, "x")
    y = torch.empty_like(x)
    check(lib().stx_relu_fwd(x.data_ptr(), y.data_ptr(), x.numel(), _stream()), "stx_relu_fwd")
    return y


def relu_bwd(dy, y):
    dx = torch.empty_like(dy)
    check(lib().stx_relu_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dy.numel(), _stream()),
          "stx_relu_bwd")
    return dx


# ----------------------------------------------------------------------- adam
def adam_step(p, g, m, v, step_dev, ws, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
              clear=None):
    """Adam update (stx_adam_step); clear: a float32 device tensor (<= 2^31 elements)
    zeroed in the same launch sequence (stx_adam_step_clear)."""
    if clear is not None:
        _req(clear, "clear")
        check(lib().stx_adam_step_clear(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                                        p.numel(), float(lr), float(beta1), float(beta2),
                                        float(eps), step_dev.data_ptr(), ws.data_ptr(),
                                        clear.data_ptr(), clear.numel(), _stream()),
              "stx_adam_step_clear")
        return
    check(lib().stx_adam_step(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                              float(lr), float(beta1), float(beta2), float(eps),
                              step_dev.data_ptr(), ws.data_ptr(), _stream()), "stx_adam_step")


# ----------------------------------------------------------------------- instance norm
def instnorm_fwd(x, gamma, beta, res=None, eps=1e-5, relu=False, out=None, out_amax=None):
    _req(x, "x")
    n, c = x.shape[:2]
    hw = x[0, 0].numel()
    if out is None:
        out = torch.empty_like(x)
    mean = torch.empty(n * c, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    check(lib().stx_instnorm_fwd(x.data_ptr(), _p(res), _p(gamma), _p(beta), out.data_ptr(),
                                 mean.data_ptr(), rstd.data_ptr(), n, c, hw, float(eps),
                                 int(relu), _p(out_amax), _stream()), "stx_instnorm_fwd")
    return out, mean, rstd


def instnorm_bwd(dy, beta, x, res, gamma, mean, rstd, relu=False, dgamma=None, dbeta=None,
                 accumulate=False, out_amax=None, dbias_in=None):
    """du of y = [relu](IN(x (+res))*gamma + beta); dgamma / dbeta / dbias_in (the bias
    gradient of the conv that produced x, sum du) written or accumulated when given.
    beta: the forward's beta (None if it had none): with relu the kernel recomputes the
    forward's y > 0 from x (+ res), mean, rstd, gamma, beta bit for bit (include/stx.h)."""
    n, c = x.shape[:2]
    hw = x[0, 0].numel()
    du = torch.empty_like(x)
    L = lib()
    need = L.stx_instnorm_bwd_ws(n, c)
    # deferred only when accumulating into persistent buffers (.grad views): a fresh
    # gradient tensor handed back to autograd must be complete on return
    defer = PGRADS.active and accumulate and (
        dgamma is not None or dbeta is not None or dbias_in is not None)
    job = None
    if defer:  # partials kept for the step's single parameter-reduction launch
        parts = torch.empty(need, device=x.device, dtype=torch.uint8)
        job = (parts, n, c, dgamma, dbeta, dbias_in, accumulate)
        wp, wn = parts.data_ptr(), need
        dgamma = dbeta = dbias_in = None
    else:
        wp, wn = WS.get(need, x.device)
    check(L.stx_instnorm_bwd(dy.data_ptr(), _p(beta), x.data_ptr(), _p(res), _p(gamma),
                             mean.data_ptr(), rstd.data_ptr(), du.data_ptr(), _p(dgamma),
                             _p(dbeta), _p(dbias_in), n, c, hw, int(relu), int(accumulate),
                             _p(out_amax), wp,
                             wn, _stream()), "stx_instnorm_bwd")
    if job is not None:
        PGRADS.add(*job)  # after the kernel that writes its partials
    return du


# ----------------------------------------------------------------------- upsample / tv
def upsample2x(x):
    n, c, h, w = x.shape
    y = torch.empty((n, c, 2 * h, 2 * w), device=x.device, dtype=torch.float32)
    check(lib().stx_upsample2x_fwd(x.data_ptr(), y.data_ptr(), n * c, h, w, _stream()),
          "stx_upsample2x_fwd")
    return y


def upsample2x_bwd(dy):
    n, c, H, W = dy.shape
    dx = torch.empty((n, c, H // 2, W // 2), device=dy.device, dtype=torch.float32)
    check(lib().stx_upsample2x_bwd(dy.data_ptr(), dx.data_ptr(), n * c, H // 2, W // 2,
                                   _stream()), "stx_upsample2x_bwd")
    return dx


def tv_loss(y, factor=1e-6, grad=None, gscale=1.0, gscale_dev=None, out=None):
    _req(y, "y")
    n, c, h, w = y.shape
    if out is None:
        out = torch.empty((), device=y.device, dtype=torch.float32)
    L = lib()
    wp, wn = WS.get(L.stx_tv_ws(n, c, h, w), y.device)
    check(L.stx_tv_loss(y.data_ptr(), out.data_ptr(), _p(grad), float(gscale), _p(gscale_dev),
                        n, c, h, w, float(factor), wp, wn, _stream()), "stx_tv_loss")
    return out


# ----------------------------------------------------------------------- temporal loss
def temporal_loss(y, y_old, x, x_old, weight=1.0, out=None):
    """[loss, ||y - y_old||, ||x - x_old||] (device [3]), loss =
    ||y - y_old|| / (||x - x_old|| + 1) * weight (get_temporal_loss)."""
    for t, nm in ((y, "y"), (y_old, "y_old"), (x, "x"), (x_old, "x_old")):
        _req(t, nm)
    assert y.numel() == y_old.numel() == x.numel() == x_old.numel(), \
        (y.shape, y_old.shape, x.shape, x_old.shape)
    if out is None:
        out = torch.empty(3, device=y.device, dtype=torch.float32)
    L = lib()
    wp, wn = WS.get(L.stx_temporal_loss_ws(), y.device)
    check(L.stx_temporal_loss(y.data_ptr(), y_old.data_ptr(), x.data_ptr(), x_old.data_ptr(),
                              y.numel(), float(weight), out.data_ptr(), wp, wn, _stream()),
          "stx_temporal_loss")
    return out


def temporal_loss_bwd(y, y_old, fwd, weight=1.0, g=None, grad=None, accumulate=False):
    """d loss / d y of temporal_loss (fwd: its output), times the device scalar g."""
    if grad is None:
        grad = torch.empty_like(y)
    check(lib().stx_temporal_loss_bwd(y.data_ptr(), y_old.data_ptr(), y.numel(), fwd.data_ptr(),
                                      float(weight), _p(g), grad.data_ptr(), int(accumulate),
                                      _stream()), "stx_temporal_loss_bwd")
    return grad
