"""Launch targets for the PMC passes (tools/pmc_r3.sh): three EAGER Gatys iterations at
512^2 (every kernel of the iteration, exactly as the engine launches it, outside a
hipGraph so the counters attach to each dispatch), then the fast_st B=8 step once."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import vgg as V  # noqa: E402
from styletransfer_amd import weights as W  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    H = 512
    style = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H))).to(dev)
    content = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H))).to(dev)
    eng = V.GatysEngine(V.VGGFeatures(V.load_vgg19_weights(), dev), style, content)
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    if "--fast" in sys.argv:
        from styletransfer_amd import network
        from styletransfer_amd.train import FastStTrainer
        st = torch.from_numpy(W.synthetic_image(3000, (1, 3, 256, 256))).to(dev)
        itn = network.ImageTransformNet(st, batch_size=8).to(dev)
        itn.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
        tr = FastStTrainer(itn, st)
        b = torch.from_numpy(W.synthetic_image(4000, (8, 3, 256, 256))).to(dev)
        tr.step(b)
        tr.step(b)
        torch.cuda.synchronize()
    print("pmc targets done")


if __name__ == "__main__":
    main()
