"""ImageTransformNet forward at fast_st's per-GPU batch (B8 256^2, no grad), HIP events:
a micro for library A/Bs of the ITN's forward kernels (tools/gpu_r6.sh MICRO=...)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import network  # noqa: E402
from styletransfer_amd import weights as W  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    style = torch.from_numpy(W.synthetic_image(3000, (1, 3, 256, 256))).to(dev)
    itn = network.ImageTransformNet(style, batch_size=8).to(dev)
    itn.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
    x = torch.from_numpy(W.synthetic_image(4000, (8, 3, 256, 256))).to(dev)
    with torch.no_grad():
        for _ in range(5):
            itn(x)
        torch.cuda.synchronize()
        res = []
        for _ in range(7):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                itn(x)
            b.record()
            b.synchronize()
            res.append(a.elapsed_time(b) / 20)
    res.sort()
    print(f"itn fwd B8 256: median {res[3] * 1e3:.1f} us  min {res[0] * 1e3:.1f} us")


if __name__ == "__main__":
    main()
