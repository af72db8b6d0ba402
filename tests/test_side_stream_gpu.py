"""The trainers' weight-gradient side stream (ops.SIDE): every conv's dW is
issued on a second stream beside the data-gradient chain and joined before Adam.  The
kernels are deterministic, so moving work between streams must not change a single bit:
the parameters after an eager step, a captured step and a replay equal those of the
one-stream run exactly (a missing fork / join or a buffer reused across streams would
show up as a difference here)."""
import os

import pytest
import torch

from styletransfer_amd import network, ops
from styletransfer_amd import weights as W

pytestmark = pytest.mark.gpu


def _run(side, dev, H, B, steps=3):
    from styletransfer_amd.train import FastStTrainer
    old = os.environ.get("STX_WGRAD_SIDE"), os.environ.get("STX_AB")
    os.environ["STX_WGRAD_SIDE"] = "1" if side else "0"
    os.environ["STX_AB"] = "1"  # (a measurement-only switch: N.knob reads it under STX_AB)
    try:
        style = torch.from_numpy(W.synthetic_image(21, (1, 3, H, H))).to(dev)
        batches = [torch.from_numpy(W.synthetic_image(900 + k, (B, 3, H, H))).to(dev)
                   for k in range(steps)]
        net = network.ImageTransformNet(style, batch_size=B)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
        tr = FastStTrainer(net, style)
        losses = [float(tr.step(batches[0]))]
        for b in batches[1:]:       # capture (warm-up step + graphs), then a replay
            losses.append(float(tr.train_step(b)))
        torch.cuda.synchronize()
        return tr.flat.detach().cpu().clone(), tr.flat_grad.detach().cpu().clone(), losses
    finally:
        for k, v in zip(("STX_WGRAD_SIDE", "STX_AB"), old):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("H,B", [(64, 2), (256, 8)])
def test_wgrad_side_stream_bit_identical(H, B):
    dev = torch.device("cuda", 0)
    p0, g0, l0 = _run(False, dev, H, B)
    p1, g1, l1 = _run(True, dev, H, B)
    assert not ops.SIDE.active  # joined and closed after every step
    assert l0 == l1
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)
