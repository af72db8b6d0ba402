"""Cost of the ReLU-mask loads in the Gatys data-gradient launches (conv1_2^T and
conv2_2^T with the split Gram-backward phase): each launch timed by HIP events as the
iteration makes it, and again without the mask (numerically wrong; timing only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import ops, vgg as V, weights as W  # noqa: E402
from styletransfer_amd import _native as N  # noqa: E402


def ev(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    H = 512
    s = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H))).to(dev)
    c = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H))).to(dev)
    feat = V.VGGFeatures(V.load_vgg19_weights(), dev)
    eng = V.GatysEngine(feat, s, c)
    for _ in range(2):
        eng.step()
    torch.cuda.synchronize()
    st, sc = eng.st, eng.scratch
    ca = st.coef_amax
    for l, dzn, zi, ci in ((1, "dz2", 0, 0), (3, "dz4", 2, 2)):
        dz = sc[dzn]
        out = torch.empty_like(st.z[zi])
        am_in = ops.amax(dz)
        z_am = ops.amax(st.z[zi])
        amo = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
        for mask in (st.z[zi], None):
            for p2 in (True, False):
                kw = dict(p2_z=st.z[zi], p2_coef=st.coef[ci], p2_amax=z_am, p2_wt_amax=ca[ci]) \
                    if p2 else {}
                t = ev(lambda: feat.dgrad(l, dz, out, mask=mask, in_amax=am_in, out_amax=amo, **kw))
                print(f"conv{l}^T mask={'yes' if mask is not None else 'no '} phase={p2}: {t:7.1f} us",
                      flush=True)


if __name__ == "__main__":
    main()
