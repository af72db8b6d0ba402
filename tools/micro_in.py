"""InstanceNorm backward of the ITN's 256^2 ReLU layers (B = 8, 32 channels: the
instnorm_bwd_greg kernel) by HIP events; prints the time and a checksum of du so the
STX_GREG_FORM variants of the measurement library can be compared (same bits expected)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(8, 32, 256, 256, generator=g) * 3 - 1).to(dev)
    gamma = (torch.rand(32, generator=g) + 0.5).to(dev)
    beta = torch.rand(32, generator=g).to(dev)
    dy = (torch.rand(8, 32, 256, 256, generator=g) * 2 - 1).to(dev)
    y, mean, rstd = ops.instnorm_fwd(x, gamma, beta, relu=True)

    def run():
        return ops.instnorm_bwd(dy, beta, x, None, gamma, mean, rstd, relu=True)
    du = run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        run()
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) / 20 * 1e3
    mb = 3 * x.numel() * 4 / 1e6
    print(f"instnorm_bwd 256^2 relu B8x32: {us:.1f} us ({mb / us:.2f} TB/s at 3 plane-passes); "
          f"du checksum {float(du.double().abs().sum()):.10e} {float(du.double().sum()):.10e}",
          flush=True)




def main128():
    """The 128^2 layers (B = 8, 64 channels, ReLU): forward and backward."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(6)
    x = (torch.rand(8, 64, 128, 128, generator=g) * 3 - 1).to(dev)
    gamma = (torch.rand(64, generator=g) + 0.5).to(dev)
    beta = torch.rand(64, generator=g).to(dev)
    dy = (torch.rand(8, 64, 128, 128, generator=g) * 2 - 1).to(dev)

    def ev(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            fn()
        b.record()
        b.synchronize()
        return a.elapsed_time(b) / 20 * 1e3
    y, mean, rstd = ops.instnorm_fwd(x, gamma, beta, relu=True)
    tf = ev(lambda: ops.instnorm_fwd(x, gamma, beta, relu=True, out=y))
    du = ops.instnorm_bwd(dy, beta, x, None, gamma, mean, rstd, relu=True)
    tb = ev(lambda: ops.instnorm_bwd(dy, beta, x, None, gamma, mean, rstd, relu=True))
    print(f"instnorm 128^2 relu B8x64: fwd {tf:.1f} us, bwd {tb:.1f} us; checksums "
          f"{float(y.double().sum()):.10e} {float(du.double().abs().sum()):.10e}", flush=True)


if len(sys.argv) > 1 and sys.argv[1] == "128":
    main128()
elif __name__ == "__main__":
    main()
