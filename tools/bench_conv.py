"""Microbenchmark of the libstx conv / gram kernels at the hot-path shapes (HIP
events on the launch stream).  Prints TFLOP/s per shape (algorithmic 2*MAC)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import _native as N  # noqa: E402
from styletransfer_amd import ops  # noqa: E402


def ev(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="run only cases whose name contains this")
    ap.add_argument("--no-split", action="store_true", help="fp32 MFMA kernels only")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    cases = [
        # name, n, cin, cout, h, w, ks, stride, mode, transpose(dgrad)
        ("vgg conv1_1 fwd 512", 1, 3, 64, 512, 512, 3, 1, N.STX_IN_RAW),
        ("vgg conv1_2 fwd 512", 1, 64, 64, 512, 512, 3, 1, N.STX_IN_RELU),
        ("vgg conv2_1 fwd 512", 1, 64, 128, 512, 512, 3, 1, N.STX_IN_RELU_POOL2),
        ("vgg conv2_2 fwd 256", 1, 128, 128, 256, 256, 3, 1, N.STX_IN_RELU),
        ("vgg conv3_1 fwd 256", 1, 128, 256, 256, 256, 3, 1, N.STX_IN_RELU_POOL2),
        ("vgg dgrad1_1 (64->3) 512", 1, 64, 3, 512, 512, 3, 1, N.STX_IN_RAW),
        ("itn res conv B8 64^2", 8, 128, 128, 64, 64, 3, 1, N.STX_IN_RAW),
        ("itn conv0 9x9 B8 256", 8, 3, 32, 256, 256, 9, 1, N.STX_IN_RAW),
        ("itn conv22 9x9 B8 256", 8, 32, 3, 256, 256, 9, 1, N.STX_IN_RAW),
        ("itn up conv B8 128->64 @128", 8, 128, 64, 64, 64, 3, 1, N.STX_IN_UPSAMPLE2),
        ("itn down s2 B8 32->64", 8, 32, 64, 256, 256, 3, 2, N.STX_IN_RAW),
    ]
    if not args.only or "hbm" in args.only:
        # HBM calibration: 64 MiB write (fill) and 64 MiB copy (read + write)
        a = torch.empty(16 << 20, device=dev)
        bb = torch.empty_like(a)
        ms = ev(lambda: a.fill_(1.0))
        ms2 = ev(lambda: bb.copy_(a))
        print(f"{'hbm fill 64MiB':32s} {ms * 1e3:9.1f} us {64 * 1.048576 / ms / 1e3:7.2f} TB/s | "
              f"copy {ms2 * 1e3:9.1f} us {2 * 64 * 1.048576 / ms2 / 1e3:7.2f} TB/s", flush=True)
    for name, n, cin, cout, h, w, ks, s, mode in cases:
        if args.only not in name:
            continue
        x = torch.randn(n, cin, h, w, generator=g).to(dev)
        wraw = torch.randn(cout, cin, ks, ks, generator=g).to(dev) * 0.05
        wt = ops.conv_weight_prep(wraw)
        hv, wv = ops.virtual_hw(h, w, mode)
        ho, wo = ops.conv_out_hw(hv, wv, ks, s, ks // 2)
        out = torch.empty(n, cout, ho, wo, device=dev)
        ms = ev(lambda: ops.conv2d(x, wt, cin, cout, ks, stride=s, in_mode=mode, out=out))
        gf = 2.0 * n * cin * cout * ks * ks * ho * wo / 1e9
        line = f"{name:32s} fp32 {ms * 1e3:9.1f} us {gf / ms:7.2f} TF"
        if not args.no_split and ops.split_eligible(cin, cout, ks, s):
            w16 = ops.conv_weight_prep16(wraw)
            am = ops.amax(x)
            kw = {}
            if "conv1_2" in name:  # the Gatys launch: + relu/pool output, out_amax
                kw = dict(pool_out=torch.empty(n, cout, ho // 2, wo // 2, device=dev),
                          out_amax=torch.zeros(N.STX_AMAX_SLOTS, device=dev))
            ms16 = ev(lambda: ops.conv2d(x, wt, cin, cout, ks, stride=s, in_mode=mode, out=out,
                                         wt16=w16, in_amax=am, **kw))
            line += f" | f16x3 {ms16 * 1e3:9.1f} us {gf / ms16:7.2f} TF"
        nt = ops.conv_gram_tiles(cin, cout, ho, wo) if s == 1 and mode in (
            N.STX_IN_RAW, N.STX_IN_RELU) else 0
        if nt and not args.no_split and (cin == 3 or ops.split_eligible(cin, cout, ks, s)):
            gp = torch.empty(n * ops.gram_tile_units(cout) * nt * 4096, device=dev)
            kw16 = {}
            if cin != 3:
                kw16 = dict(wt16=ops.conv_weight_prep16(wraw), in_amax=ops.amax(x))
                if "conv1_2" in name:
                    kw16.update(pool_out=torch.empty(n, cout, ho // 2, wo // 2, device=dev),
                                out_amax=torch.zeros(N.STX_AMAX_SLOTS, device=dev))
            msg = ev(lambda: ops.conv2d(x, wt, cin, cout, ks, stride=s, in_mode=mode, out=out,
                                        gram_part=gp, **kw16))
            line += f" | +gram {msg * 1e3:9.1f} us"
        print(line, flush=True)
    for name, n, c, h in (("gram C64 512^2", 1, 64, 512), ("gram C128 256^2", 1, 128, 256),
                          ("gram C256 128^2", 1, 256, 128), ("gram C64 B8 256^2", 8, 64, 256)):
        if args.only not in name:
            continue
        z = torch.randn(n, c, h, h, generator=g).to(dev)
        t = torch.randn(c, c, generator=g).to(dev)
        coef = None
        ms = ev(lambda: ops.style_loss(z, t))
        _, coef = ops.style_loss(z, t)
        dz = torch.empty_like(z)
        ms2 = ev(lambda: ops.gram_bwd(coef, z, dz, accumulate=True))
        if n == 1 and c in (64, 128):  # the Gatys dz2/dz4 launches: split 1x1 + unpool
            dp = torch.randn(n, c, h // 2, h // 2, generator=g).to(dev)
            zam = ops.amax(z)
            ms3 = ev(lambda: ops.gram_bwd_fused(coef, z, out=dz, up_dp=dp, z_amax=zam))
            mb = (2.25 * c * h * h * 4) / 1e6
            print(f"{'gram bwd split+unpool C%d' % c:32s} {ms3 * 1e3:9.1f} us "
                  f"{mb / (ms3 * 1e3):6.2f} TB/s ({mb:.0f} MB)", flush=True)
        gf = 2.0 * n * c * c * h * h / 1e9
        zam2 = ops.amax(z)
        ms16 = ev(lambda: ops.style_loss(z, t, z_amax=zam2))
        print(f"{name:32s} fwd {ms * 1e3:8.1f} us {gf / ms:7.2f} TF | split {ms16 * 1e3:8.1f} us "
              f"{c * h * h * n * 4 / (ms16 * 1e3) / 1e6:5.2f} TB/s | bwd {ms2 * 1e3:8.1f} us "
              f"{gf / ms2:7.2f} TF")
    # wgrad
    up = N.STX_IN_UPSAMPLE2
    for name, n, cin, cout, h, ks, s, mode in (
            ("wgrad res B8 128 64^2", 8, 128, 128, 64, 3, 1, 0),
            ("wgrad up B8 128->64 128^2", 8, 128, 64, 64, 3, 1, up),
            ("wgrad conv0 9x9 B8", 8, 3, 32, 256, 9, 1, 0),
            ("wgrad conv22 9x9 B8", 8, 32, 3, 256, 9, 1, 0),
            ("wgrad down s2 B8 32->64 256", 8, 32, 64, 256, 3, 2, 0),
            ("wgrad down s2 B8 64->128 128", 8, 64, 128, 128, 3, 2, 0)):
        if args.only not in name:
            continue
        x = torch.randn(n, cin, h, h, generator=g).to(dev)
        hv = 2 * h if mode == up else h
        ho = (hv + 2 * (ks // 2) - ks) // s + 1
        dy = torch.randn(n, cout, ho, ho, generator=g).to(dev)
        ms = ev(lambda: ops.conv2d_wgrad(x, dy, cin, cout, ks, stride=s, in_mode=mode,
                                         split=False), reps=10)
        gf = 2.0 * n * cin * cout * ks * ks * ho * ho / 1e9
        line = f"{name:32s} fp32 {ms * 1e3:9.1f} us {gf / ms:7.2f} TF"
        ms16 = ev(lambda: ops.conv2d_wgrad(x, dy, cin, cout, ks, stride=s, in_mode=mode), reps=10)
        line += f" | f16x3 {ms16 * 1e3:9.1f} us {gf / ms16:7.2f} TF (incl. 2 amax passes)"
        print(line, flush=True)

if __name__ == "__main__":
    main()
