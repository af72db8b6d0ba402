"""Where the v2 split conv's cycles go (diagnostic build: STX_CONV_STAMP=1 selects the
STAMP instantiation of conv3x3_f16x3_v2_kernel for the ReLU-loader 256-pixel launches).
Runs conv1_2's forward at 512^2 exactly as the Gatys iteration launches it (input scale
slot, fused ReLU+MaxPool output, fused Gram partials; tools' copy of bench.py's setup),
once plain (timed) and once stamped, and prints the per-wave shares of the segments:
prologue, tap 0 MFMAs + the step's staging, taps 1-2 MFMAs, the step's barrier wait,
epilogue (shares, not times: the stamps' own waits forbid some overlaps)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import _native as N  # noqa: E402
from styletransfer_amd import ops  # noqa: E402
from styletransfer_amd import vgg as V  # noqa: E402
from styletransfer_amd import weights as W  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    H = 512
    style = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H))).to(dev)
    content = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H))).to(dev)
    feat = V.VGGFeatures(V.load_vgg19_weights(), dev)
    eng = V.GatysEngine(feat, style, content)
    eng.step()
    torch.cuda.synchronize()
    z1 = eng.st.z[0]
    out = torch.empty_like(z1)
    am = ops.amax(z1)  # (the iteration's own slot is zeroed by its Adam launch)
    am_out = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
    pool = torch.empty_like(eng.st.pools[1])
    gp = torch.empty_like(eng.st.grams[1])

    def conv12():
        return ops.conv2d(z1, feat.wt[1], 64, 64, 3, in_mode=N.STX_IN_RELU, bias=feat.b[1],
                          out=out, wt16=feat.wt16[1], in_amax=am, out_amax=am_out,
                          pool_out=pool, gram_part=gp)
    for _ in range(3):
        conv12()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        conv12()
    b.record()
    b.synchronize()
    print(f"conv1_2 fwd (plain build): {a.elapsed_time(b) / 20 * 1e3:.1f} us")
    ref = out.clone()
    os.environ["STX_CONV_STAMP"] = "1"
    conv12()
    torch.cuda.synchronize()
    st1 = out.clone()
    conv12()
    torch.cuda.synchronize()
    os.environ["STX_CONV_STAMP"] = "0"
    d = (out - ref).abs()
    print(f"stamped vs plain output: equal {torch.equal(out, ref)}, max|diff| {d.max().item():.3e}"
          f" (max|out| {ref.abs().max().item():.3e}), differing elements {(d > 0).sum().item()};"
          f" stamped run-to-run equal {torch.equal(out, st1)}")
    conv12()
    torch.cuda.synchronize()
    print(f"plain run-to-run equal {torch.equal(out, ref)}")
    lib = N.lib()
    fn = lib.stx_debug_conv_stamps
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int]
    nw = 1024 * 4
    buf = np.zeros(nw * 8, dtype=np.uint64)
    assert fn(buf.ctypes.data, nw * 8) == 0
    s = buf.reshape(nw, 8).astype(np.float64)
    names = ["prologue", "tap0 MFMA + staging", "taps1-2 MFMA", "barrier wait", "epilogue"]
    tot = s[:, :5].sum(axis=1)
    print(f"waves {nw}, steps per wave {np.median(s[:, 5]):.0f}, wave lifetime median "
          f"{np.median(tot):.0f} clk (p10 {np.percentile(tot, 10):.0f}, p90 "
          f"{np.percentile(tot, 90):.0f})")
    for k, nm in enumerate(names):
        print(f"  {nm:22s} share {np.sum(s[:, k]) / np.sum(tot):6.3f}  median per wave "
              f"{np.median(s[:, k]):9.0f} clk  per step {np.median(s[:, k] / max(1, np.median(s[:, 5]))):7.0f}")


if __name__ == "__main__":
    main()
