"""nn layers whose forward runs on libstx.  They subclass the torch.nn layers
the reference builds its networks from (so `isinstance(layer, nn.Conv2d)`,
parameter names and `state_dict()` keys are unchanged) and keep the same class
names, because the reference names VGG layers by `type(layer).__name__`
(stransfer/network.py:273-274: 'Conv2d_4', 'ReLU_4', ...)."""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _native as N
from . import autograd as A


class Conv2d(nn.Conv2d):
    """nn.Conv2d on the HIP implicit-GEMM kernel.  `padding_mode='reflection'`
    (stransfer/network.py:473,...,609) is not a torch padding mode; at the
    reference's pinned torch==1.1.0 it fell through to zero padding, which is
    what is implemented here."""

    def __init__(self, *args, padding_mode="zeros", **kwargs):
        if padding_mode == "reflection":
            padding_mode = "zeros"
        super().__init__(*args, padding_mode=padding_mode, **kwargs)
        if self.padding_mode != "zeros":
            raise NotImplementedError(f"padding_mode={self.padding_mode}")
        if self.groups != 1 or self.dilation != (1, 1):
            raise NotImplementedError("groups/dilation")
        if self.kernel_size[0] != self.kernel_size[1] or self.kernel_size[0] not in (1, 3, 9):
            raise NotImplementedError(f"kernel_size {self.kernel_size}")
        self._wt_cache = None
        self._train_slabs = None  # set by ops.TrainedSlabs.prep() (fast_st trainers)
        # reads a nearest x2 upsampled input (ImageTransformNet's UpsampleConvLayer): the
        # split path also gets the parity-class slab (ops.conv_weight_prep16_up)
        self._up_input = False

    def prepped(self):
        """Cached GEMM slabs (fp32, and the fp16 hi/lo split slab where the shape
        takes the split kernel) of a frozen weight; re-prepped when it changes."""
        w = self.weight
        key = (w.data_ptr(), w._version, w.device)
        if self._wt_cache is None or self._wt_cache[0] != key:
            from . import ops
            wd = w.detach().contiguous()
            cout, cin, ks, _ = wd.shape
            w16 = ops.conv_weight_prep16(wd) if (A._split_on() and self.padding[0] == 1 and
                                                 ops.split_eligible(cin, cout, ks, self.stride[0])) \
                else None
            up = ops.conv_weight_prep16_up(wd) if (w16 is not None and self._up_input and
                                                   A._upar_on()) else None
            self._wt_cache = (key, ops.conv_weight_prep(wd), w16, up)
        return self._wt_cache[1], self._wt_cache[2], self._wt_cache[3]

    def forward(self, x, in_mode=N.STX_IN_RAW, bias_grad=True, link=None):
        """bias_grad=False: the bias enters detached -- for a conv feeding an
        InstanceNorm2d that is handed the bias (`conv_bias=`) and produces its gradient."""
        wt = wt16 = wtT = wtT16 = up = None
        ts = self._train_slabs
        w = self.weight
        if ts is not None and ts[0] == (w.data_ptr(), w._version, w.device):
            _, wt, wt16, wtT, wtT16, up = ts  # the trainer's batched prep of this version
        elif not w.requires_grad or not torch.is_grad_enabled():
            wt, wt16, up = self.prepped()  # frozen or inference: slabs cached per weight version
        b = self.bias if bias_grad or self.bias is None else self.bias.detach()
        return A.conv2d(x, w, b, self.stride[0], self.padding[0], in_mode, wt, wt16, wtT, wtT16,
                        link, wt16_up=up)


class ReLU(nn.ReLU):
    def forward(self, x):
        return A.ReLUFn.apply(x)


class MaxPool2d(nn.MaxPool2d):
    def __init__(self, kernel_size=2, stride=2, **kw):
        super().__init__(kernel_size, stride, **kw)
        if self.kernel_size not in (2, (2, 2)) or self.stride not in (2, (2, 2)) or \
                self.padding not in (0, (0, 0)) or self.ceil_mode or self.dilation not in (1,):
            raise NotImplementedError("only MaxPool2d(2, 2)")

    def forward(self, x):
        y, idx = A.MaxPool2dFn.apply(x)
        return (y, idx) if self.return_indices else y


class InstanceNorm2d(nn.InstanceNorm2d):
    def forward(self, x, relu=False, res=None, conv_bias=None, res_link=None):
        if self.track_running_stats:
            raise NotImplementedError("track_running_stats")
        return A.instance_norm(x, self.weight, self.bias, res=res, eps=self.eps, relu=relu,
                               conv_bias=conv_bias, res_link=res_link)


class Upsample(nn.Upsample):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        if self.mode != "nearest" or float(self.scale_factor) != 2.0:
            raise NotImplementedError("only nearest x2 upsampling")

    def forward(self, x):
        return A.Upsample2xFn.apply(x)
