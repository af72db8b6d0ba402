"""Microbenchmark of the few-channel convs: the 9x9 ITN layers (conv9.hip) at B=8 256^2
(conv0 fwd 3->32, conv22 fwd 32->3 with a max|x| bound) and VGG conv1_1's data
gradient (64->3 @ 512^2, convfew.hip), HIP events on the launch stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import ops  # noqa: E402


def ev(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    n, h, w = 8, 256, 256
    x3 = torch.randn(n, 3, h, w, generator=g).to(dev)
    x32 = torch.randn(n, 32, h, w, generator=g).to(dev).relu_()
    w0 = (torch.randn(32, 3, 9, 9, generator=g) * 0.05).to(dev)
    w22 = (torch.randn(3, 32, 9, 9, generator=g) * 0.05).to(dev)
    wt0 = ops.conv_weight_prep(w0)
    wt22 = ops.conv_weight_prep(w22)
    am = ops.amax(x32)
    gf = 2 * 32 * 3 * 81 * n * h * w / 1e9
    # VGG conv1_1's data gradient to the image (64 -> 3, 3x3 @ 512^2, convfew.hip)
    d1 = torch.randn(1, 64, 512, 512, generator=g).to(dev)
    w11 = (torch.randn(64, 3, 3, 3, generator=g) * 0.05).to(dev)
    wt11 = ops.conv_weight_prep(w11, transpose=True)
    am1 = ops.amax(d1)
    for name, fn in [("conv0 fwd 3->32", lambda: ops.conv2d(x3, wt0, 3, 32, 9)),
                     ("conv22 fwd 32->3", lambda: ops.conv2d(x32, wt22, 32, 3, 9, in_amax=am)),
                     ("vgg dgrad1_1 64->3", lambda: ops.conv2d(d1, wt11, 64, 3, 3, in_amax=am1))]:
        ms = ev(fn)
        print(f"{name:20s} {ms * 1e3:8.1f} us {gf / ms:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
