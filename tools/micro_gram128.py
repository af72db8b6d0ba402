"""Conv + fused 128-channel Gram (conv_gram_tile128) at the Gatys / fast_st conv2_x
shapes: the plain conv (64-cout blocks), the same conv on 8-wave 128-cout blocks
(STX_FORCE_WM2=1, measurement build only), with the fused Gram, and with the Gram plus
the content MSE sums; beside the standalone Gram kernels it replaces.  HIP events on the
launch stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import _native as N  # noqa: E402
from styletransfer_amd import ops  # noqa: E402


def ev(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    tag = os.environ.get("TAG", "")
    for name, n, cin, h, mode, pool in [("gatys conv2_1", 1, 64, 256, N.STX_IN_RAW, False),
                                        ("gatys conv2_2", 1, 128, 256, N.STX_IN_RELU, True),
                                        ("fast conv2_1 B8", 8, 64, 128, N.STX_IN_RAW, False),
                                        ("fast conv2_2 B8", 8, 128, 128, N.STX_IN_RELU, True)]:
        cout = 128
        x = torch.randn(n, cin, h, h, generator=g).to(dev)
        wr = torch.randn(cout, cin, 3, 3, generator=g).to(dev) * 0.05
        b = torch.randn(cout, generator=g).to(dev) * 0.1
        wt, w16 = ops.conv_weight_prep(wr), ops.conv_weight_prep16(wr)
        am = ops.amax(x)
        y = torch.empty(n, cout, h, h, device=dev)
        po = torch.empty(n, cout, h // 2, h // 2, device=dev) if pool else None
        nt = ops.conv_gram_tiles(cin, cout, h, h, n=n, in_mode=mode)
        if nt == 0:
            print(f"{name}: not fused (more than one round of blocks)")
            continue
        gp = torch.empty(n * 3 * nt * 4096, device=dev)
        c = torch.randn(n, cout, h, h, generator=g).to(dev)
        mp = torch.empty(2 * n * nt, device=dev)
        base = dict(in_mode=mode, bias=b, wt16=w16, in_amax=am, out=y, pool_out=po)

        def run(**kw):
            return ev(lambda: ops.conv2d(x, wt, cin, cout, 3, **base, **kw))
        t_plain = run()
        if os.environ.get("DBG"):  # measurement build: the Gram tile cut after stage k
            print(f"{name:18s} plain {t_plain:7.1f} " + " ".join(
                f"cut{k} {run(gram_part=gp, aux_scale=float(k)):7.1f}" for k in (4, 1, 2, 3))
                + f" full {run(gram_part=gp):7.1f}", flush=True)
            continue
        t_gram = run(gram_part=gp)
        t_mse = run(gram_part=gp, mse_ref=c, mse_parts=mp)
        ws = torch.empty(N.lib().stx_style_content_ws(n, cout, h * h), device=dev,
                         dtype=torch.uint8)
        tgt = torch.zeros(cout, cout, device=dev)
        zam = ops.amax(y)
        mo = torch.empty(3, device=dev)
        t_tri = ev(lambda: ops.style_loss(y, tgt, z_amax=zam, defer_ws=ws))
        t_tri_mse = ev(lambda: ops.style_content_loss(y, tgt, c, mo, z_amax=zam, defer_ws=ws))
        print(f"{tag:6s} {name:18s} plain {t_plain:7.1f}  +gram {t_gram:7.1f}  +gram+mse "
              f"{t_mse:7.1f} us | standalone gram(+fin) {t_tri:6.1f}  gram+mse(+fin) "
              f"{t_tri_mse:6.1f}", flush=True)


def main64():
    """conv1_2 (64 channels, 512^2, fused pool output): the 64-channel Gram tile."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(1)
    for name, n, h in [("gatys conv1_2", 1, 512), ("fast conv1_2 B8", 8, 256)]:
        cin = cout = 64
        x = torch.randn(n, cin, h, h, generator=g).to(dev)
        wr = torch.randn(cout, cin, 3, 3, generator=g).to(dev) * 0.05
        b = torch.randn(cout, generator=g).to(dev) * 0.1
        wt, w16 = ops.conv_weight_prep(wr), ops.conv_weight_prep16(wr)
        am = ops.amax(x)
        y = torch.empty(n, cout, h, h, device=dev)
        po = torch.empty(n, cout, h // 2, h // 2, device=dev)
        nt = ops.conv_gram_tiles(cin, cout, h, h, n=n, in_mode=N.STX_IN_RELU)
        gp = torch.empty(n * nt * 4096, device=dev)
        base = dict(in_mode=N.STX_IN_RELU, bias=b, wt16=w16, in_amax=am, out=y, pool_out=po)
        t0 = ev(lambda: ops.conv2d(x, wt, cin, cout, 3, **base))
        t1 = ev(lambda: ops.conv2d(x, wt, cin, cout, 3, gram_part=gp, **base))
        if os.environ.get("DBG"):
            print(f"{name:18s} " + " ".join(
                f"cut{k} {ev(lambda: ops.conv2d(x, wt, cin, cout, 3, gram_part=gp, aux_scale=float(k), **base)):7.1f}"
                for k in (4, 1, 2, 3)), flush=True)
        print(f"{os.environ.get('TAG', ''):6s} {name:18s} plain {t0:7.1f}  +gram {t1:7.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
    main64()
