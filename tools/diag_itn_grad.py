"""Diagnostic: ITN parameter-gradient error of (a) the HIP path and (b) the fp32
CPU oracle, both against an fp64 CPU oracle (truth).  Run on the GPU box."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("STX_NO_LOGFILE", "1")
from oracle import reference_cpu as O  # noqa: E402
from styletransfer_amd import network  # noqa: E402
from styletransfer_amd import weights as W  # noqa: E402

d = np.load("tests/golden/itn.npz")
style = torch.from_numpy(d["style"])
batch = torch.from_numpy(d["batch"])
cimg = torch.from_numpy(W.synthetic_image(23, (1, 3, 64, 64)))


def oracle_grads(dtype):
    net = O.image_transform_net(4321).to(dtype)
    ln = O.StyleNetwork(style.to(dtype), cimg.to(dtype), vgg=O.vgg19_features(1234).to(dtype))
    total, y = O.fast_st_closure(net, ln, batch.to(dtype))
    return [p.grad.double().numpy() for p in net.parameters()], float(total)


g64, t64 = oracle_grads(torch.float64)
g32, t32 = oracle_grads(torch.float32)
dev = torch.device("cuda", 0)
net = network.ImageTransformNet(style.to(dev), 2)
net.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
ln = network.StyleNetwork(style.to(dev), cimg.to(dev))
y = net(batch.to(dev))
ln(y, content_image=batch.to(dev))
tot = (ln.get_total_current_style_loss(100_000) + ln.get_total_current_content_loss(1)
       + net.get_total_variation_regularization_loss(y))
tot.backward()
gh = [p.grad.double().cpu().numpy() for p in net.parameters()]
keys = [k for k, _ in W.itn_synthetic(4321)]
print(f"total: f64 {t64:.10g}  f32 {t32:.10g}  hip {float(tot):.10g}")


def rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


worst = []
for k, a, b, c in zip(keys, gh, g32, g64):
    worst.append((rel(a, c), rel(b, c), k))
    print(f"{k:20s} hip-vs-f64 {rel(a, c):.2e}   f32oracle-vs-f64 {rel(b, c):.2e}   "
          f"hip-vs-f32 {rel(a, b):.2e}  |g| {np.linalg.norm(c):.3e}")
print("max hip-vs-f64", max(w[0] for w in worst), "max f32-vs-f64", max(w[1] for w in worst))
