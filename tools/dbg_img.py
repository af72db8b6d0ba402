import sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '.')
from PIL import Image
from styletransfer_amd import img_utils
from oracle import pil_resample as R
dev = torch.device('cuda', 0)
img = np.random.default_rng(0).integers(0, 256, (444, 444, 3), dtype=np.uint8)
got = img_utils.ImageConditioner(256, dev)([img]).cpu()[0]
want = img_utils.image_loader_transform(Image.fromarray(img), 256).cpu()[0]
u8 = R.resize_bilinear_u8(img, 256, 256)
d = (got != want)
print("mismatch", int(d.sum()), "of", d.numel())
idx = d.nonzero()[:10]
for c, y, x in idx.tolist():
    print(c, y, x, "got", float(got[c, y, x]), "want", float(want[c, y, x]), "u8", int(u8[y, x, c]))
# byte-level: invert normalization to recover the GPU's u8
m = np.array([0.485, 0.456, 0.406], np.float32).reshape(3,1,1); s = np.array([0.229, 0.224, 0.225], np.float32).reshape(3,1,1)
g8 = np.rint((got.numpy() * s + m) * 255).astype(int).transpose(1,2,0)
print("u8 diff count", int((g8 != u8).sum()), "max", int(np.abs(g8 - u8.astype(int)).max()))
