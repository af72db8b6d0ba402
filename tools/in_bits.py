"""Dump InstanceNorm fwd/bwd outputs at the ITN plane sizes (for comparing kernel
variants across processes: STX_IN_BUF=0/1).  usage: python tools/in_bits.py out.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import _native as N  # noqa: E402
from styletransfer_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(0)
out = {}
for (n, c, h) in [(3, 32, 64), (3, 64, 32), (3, 128, 16), (8, 128, 64), (2, 32, 9)]:
    x = torch.randn(n, c, h, h, generator=g).to(dev)
    r = torch.randn(n, c, h, h, generator=g).to(dev)
    gm = torch.rand(c, generator=g).to(dev) + 0.5
    bt = torch.randn(c, generator=g).to(dev)
    dy = torch.randn(n, c, h, h, generator=g).to(dev)
    for relu in (False, True):
        for res in (None, r):
            am = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
            y, mean, rstd = ops.instnorm_fwd(x, gm, bt, res=res, relu=relu, out_amax=am)
            ga = torch.zeros(c, device=dev)
            gb = torch.zeros(c, device=dev)
            am2 = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
            du = ops.instnorm_bwd(dy, y, x, res, gm, mean, rstd, relu=relu, dgamma=ga, dbeta=gb,
                                  out_amax=am2)
            k = f"{n}x{c}x{h} relu{int(relu)} res{int(res is not None)}"
            out[k] = [t.detach().cpu() for t in (y, mean, rstd, am, du, ga, gb, am2)]
torch.save(out, sys.argv[1])
