"""The residual convs' 3x3 weight gradient (128 -> 128 @ 64^2, B=8, split MFMA; raw and
ReLU input; plus small / ragged shapes) under the variants given as NAME=VALUE specs:
HIP-event time of the whole stx_conv2d_wgrad16 call (main kernel + split-K reduce; max|x|,
max|dy| precomputed) and each result's error against an fp64 torch reference.  Each
NAME=VALUE spec is set before its runs; only switches the library reads at every call
(not its static-cached ones) differ within one process.
    python tools/bench_wgrad.py [NAME=VALUE ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import _native as N  # noqa: E402
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
    specs = sys.argv[1:] or ["STX_DEFAULT=1"]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    for (n, c, hw, mode) in ((8, 128, 64, N.STX_IN_RAW), (8, 128, 64, N.STX_IN_RELU),
                             (2, 128, 16, N.STX_IN_RELU), (3, 128, 48, N.STX_IN_RAW),
                             (64, 128, 64, N.STX_IN_RAW)):
        x = torch.randn(n, c, hw, hw, generator=g).to(dev)
        dy = torch.randn(n, c, hw, hw, generator=g).to(dev)
        xa, da = ops.amax(x), ops.amax(dy)
        xr = x.double().cpu()
        if mode == N.STX_IN_RELU:
            xr = xr.clamp_min(0)
        ref = torch.nn.grad.conv2d_weight(xr, (c, c, 3, 3), dy.double().cpu(), padding=1)
        for spec in specs:
            k, v = spec.split("=")
            os.environ[k] = v
            dw = torch.empty(c, c, 3, 3, device=dev)
            fn = lambda: ops.conv2d_wgrad(x, dy, c, c, 3, in_mode=mode, dw=dw,  # noqa: E731
                                          x_amax=xa, dy_amax=da)
            ms = ev(fn)
            err = ((dw.double().cpu() - ref).norm() / ref.norm()).item()
            gf = 2 * c * c * 9 * n * hw * hw / 1e9
            print(f"wgrad {spec:16s} mode={mode} n={n} {hw}^2: {ms * 1e3:7.1f} us "
                  f"{gf / ms:6.1f} TF  rel err vs fp64 {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
