"""Count ops.amax call sites over one fast_st training step (launch audit)."""
import collections
import sys
import traceback
import torch
sys.path.insert(0, ".")
from styletransfer_amd import ops, network  # noqa: E402
from styletransfer_amd import weights as W  # noqa: E402
from styletransfer_amd.train import FastStTrainer  # noqa: E402

orig = ops.amax
sites = collections.Counter()


def logged(x, out=None):
    st = traceback.extract_stack()[-4:-1]
    sites[" <- ".join(f"{f.name}:{f.lineno}" for f in reversed(st)) + f" {tuple(x.shape)}"] += 1
    return orig(x, out)


ops.amax = logged
dev = torch.device("cuda", 0)
style = torch.from_numpy(W.synthetic_image(3000, (1, 3, 256, 256))).to(dev)
itn = network.ImageTransformNet(style, batch_size=8).to(dev)
tr = FastStTrainer(itn, style)
batch = torch.from_numpy(W.synthetic_image(4000, (8, 3, 256, 256))).to(dev)
tr.step(batch)
sites.clear()
tr.step(batch)
for k, v in sites.most_common():
    print(v, k)
