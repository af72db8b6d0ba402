"""Log every stx_conv2d call of one fast_st training step that will not take the
split / few-channel paths (shape audit)."""
import sys
import torch
sys.path.insert(0, ".")
from styletransfer_amd import ops, network, _native as N  # noqa: E402
from styletransfer_amd import weights as W  # noqa: E402
from styletransfer_amd.train import FastStTrainer  # noqa: E402

orig = ops.conv2d
seen = {}


def logged(x, wt, cin, cout, ks, stride=1, pad=None, in_mode=N.STX_IN_RAW, **kw):
    split = kw.get("wt16") is not None and ops.split_eligible(cin, cout, ks, stride)
    key = (tuple(x.shape), cin, cout, ks, stride, in_mode, split, kw.get("split_1x1", False),
           kw.get("out_amax") is not None, kw.get("mask") is not None, kw.get("p2_z") is not None)
    seen[key] = seen.get(key, 0) + 1
    return orig(x, wt, cin, cout, ks, stride=stride, pad=pad, in_mode=in_mode, **kw)


ops.conv2d = logged
import styletransfer_amd.vgg as V  # noqa: E402
import styletransfer_amd.autograd as A  # noqa: E402
V.ops.conv2d = logged
A.ops.conv2d = logged
dev = torch.device("cuda", 0)
style = torch.from_numpy(W.synthetic_image(3000, (1, 3, 256, 256))).to(dev)
itn = network.ImageTransformNet(style, batch_size=8).to(dev)
tr = FastStTrainer(itn, style)
batch = torch.from_numpy(W.synthetic_image(4000, (8, 3, 256, 256))).to(dev)
tr.step(batch)
seen.clear()
tr.step(batch)
for k, v in sorted(seen.items(), key=lambda kv: str(kv[0])):
    print(v, "x shape=%s cin=%d cout=%d ks=%d s=%d mode=%d split=%s 1x1=%s oamax=%s mask=%s p2=%s" % ((k[0],) + k[1:]))
