"""A/B of the split-conv main loops (conv16.hip v1 vs v2, STX_CONV_V2) in ONE process:
per-launch HIP-event timings at the hot-path shapes with a bitwise comparison of the
outputs (both loops issue the same MFMAs in the same order, so the results must be
identical), then the whole Gatys 512^2 iteration and the fast_st B=8 step, each
captured once per variant, replayed in interleaved rounds, and compared bit for bit."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import _native as N  # noqa: E402
from styletransfer_amd import ops  # noqa: E402
from styletransfer_amd import vgg as V  # noqa: E402
from styletransfer_amd import weights as W  # noqa: E402


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


def setv(v):
    os.environ["STX_CONV_V2"] = str(v)


def conv_cases(dev):
    g = torch.Generator(device="cpu").manual_seed(0)
    out = []
    spec = [
        # name, n, cin, cout, h, w, mode, extras
        ("conv1_2 fwd 512 +pool+gram", 1, 64, 64, 512, 512, N.STX_IN_RELU, "pg"),
        ("conv1_2 fwd 512 plain", 1, 64, 64, 512, 512, N.STX_IN_RELU, ""),
        ("conv2_1 fwd 256", 1, 64, 128, 256, 256, N.STX_IN_RAW, ""),
        ("conv2_2 fwd 256 +pool", 1, 128, 128, 256, 256, N.STX_IN_RELU, "p"),
        ("conv3_1 fwd 128", 1, 128, 256, 128, 128, N.STX_IN_RAW, ""),
        ("dgrad conv1_2 512 mask", 1, 64, 64, 512, 512, N.STX_IN_RAW, "m"),
        ("itn res B8 64^2", 8, 128, 128, 64, 64, N.STX_IN_RAW, ""),
        ("itn up B8 64->128", 8, 128, 64, 64, 64, N.STX_IN_UPSAMPLE2, ""),
        ("itn up B8 128->256", 8, 64, 32, 128, 128, N.STX_IN_UPSAMPLE2, ""),
        ("vgg B8 conv1_2 256", 8, 64, 64, 256, 256, N.STX_IN_RELU, "p"),
    ]
    for name, n, cin, cout, h, w, mode, ex in spec:
        x = torch.randn(n, cin, h, w, generator=g).to(dev)
        wraw = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(dev)
        bias = (torch.randn(cout, generator=g) * 0.1).to(dev)
        w16 = ops.conv_weight_prep16(wraw)
        am = ops.amax(x)
        hv, wv = ops.virtual_hw(h, w, mode)
        ho, wo = hv, wv
        kw = {}
        if "p" in ex:
            kw["pool_out"] = torch.empty(n, cout, ho // 2, wo // 2, device=dev)
        if "g" in ex:
            kw["gram_part"] = torch.empty(n * ops.conv_gram_tiles(cin, cout, ho, wo) * 4096,
                                          device=dev)
        if "m" in ex:
            kw["mask"] = torch.randn(n, cout, ho, wo, generator=g).to(dev)
        out.append((name, 2.0 * n * cin * cout * 9 * ho * wo / 1e9, x, w16, am, bias, cin, cout,
                    mode, kw, (n, cout, ho, wo)))
    return out


def main():
    dev = torch.device("cuda", 0)
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    print("== per-launch (us, median of rounds; bitwise v1 == v2; STX_CONV_TR=0)", flush=True)
    os.environ["STX_CONV_TR"] = "0"
    for name, gf, x, w16, am, bias, cin, cout, mode, kw, oshape in conv_cases(dev):
        outs, ts = {}, {1: [], 2: []}
        for v in (1, 2):
            setv(v - 1)
            y = torch.empty(oshape, device=dev)
            kv = {k: (torch.empty_like(t) if k in ("pool_out", "gram_part") else t)
                  for k, t in kw.items()}
            ops.conv2d(x, None, cin, cout, 3, in_mode=mode, out=y, wt16=w16, in_amax=am,
                       bias=bias, **kv)
            torch.cuda.synchronize()
            outs[v] = (y, kv)
        for _ in range(rounds):
            for v in (1, 2):
                setv(v - 1)
                y, kv = outs[v]
                ts[v].append(ev(lambda: ops.conv2d(x, None, cin, cout, 3, in_mode=mode, out=y,
                                                   wt16=w16, in_amax=am, bias=bias, **kv), 10))
        same = torch.equal(outs[1][0], outs[2][0]) and all(
            torch.equal(outs[1][1][k], outs[2][1][k]) for k in kw if k != "mask")
        m1, m2 = statistics.median(ts[1]) * 1e3, statistics.median(ts[2]) * 1e3
        print(f"{name:30s} v1 {m1:8.1f}  v2 {m2:8.1f}  ({gf / m2 * 1e3:6.1f} TF, "
              f"{gf / m2 * 1e3 / 833.3:.3f})  x{m1 / m2:.3f}  equal={same}", flush=True)

    print("== v2 forward launches: lane-per-pixel vs transposed accumulators (STX_CONV_TR)",
          flush=True)
    setv(1)
    for name, gf, x, w16, am, bias, cin, cout, mode, kw, oshape in conv_cases(dev):
        if "dgrad" in name:
            continue
        outs, ts = {}, {0: [], 1: []}
        for v in (0, 1):
            os.environ["STX_CONV_TR"] = str(v)
            y = torch.empty(oshape, device=dev)
            kv = {k: (torch.empty_like(t) if k in ("pool_out", "gram_part") else t)
                  for k, t in kw.items()}
            ops.conv2d(x, None, cin, cout, 3, in_mode=mode, out=y, wt16=w16, in_amax=am,
                       bias=bias, **kv)
            torch.cuda.synchronize()
            outs[v] = (y, kv)
        for _ in range(rounds):
            for v in (0, 1):
                os.environ["STX_CONV_TR"] = str(v)
                y, kv = outs[v]
                ts[v].append(ev(lambda: ops.conv2d(x, None, cin, cout, 3, in_mode=mode, out=y,
                                                   wt16=w16, in_amax=am, bias=bias, **kv), 10))
        same = torch.equal(outs[0][0], outs[1][0]) and all(
            torch.equal(outs[0][1][k], outs[1][1][k]) for k in kw if k not in ("mask", "gram_part"))
        gerr = ""
        if "gram_part" in kw:
            nt = kw["gram_part"].numel() // 4096
            G = [outs[v][1]["gram_part"].view(nt, 64, 64).double().sum(0) for v in (0, 1)]
            gerr = f" gram rel diff {float((G[0] - G[1]).norm() / G[0].norm()):.2e}"
        m0, m1 = statistics.median(ts[0]) * 1e3, statistics.median(ts[1]) * 1e3
        print(f"{name:30s} lane/pixel {m0:8.1f}  transposed {m1:8.1f}  x{m0 / m1:.3f}  "
              f"equal={same}{gerr}", flush=True)
    os.environ["STX_CONV_TR"] = "1"

    print("== conv1_1 fwd 512 + Gram partials: lane-per-pixel vs transposed (STX_FEW16T)",
          flush=True)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(1, 3, 512, 512, generator=g).to(dev)
    wraw = (torch.randn(64, 3, 3, 3, generator=g) * 0.2).to(dev)
    bias = (torch.randn(64, generator=g) * 0.1).to(dev)
    wt = ops.conv_weight_prep(wraw)
    nt = ops.conv_gram_tiles(3, 64, 512, 512)
    outs, ts = {}, {0: [], 1: []}
    for v in (0, 1):
        os.environ["STX_FEW16T"] = str(v)
        y = torch.empty(1, 64, 512, 512, device=dev)
        gp = torch.empty(nt * 4096, device=dev)
        am = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
        outs[v] = (y, gp, am)
    for _ in range(rounds):
        for v in (0, 1):
            os.environ["STX_FEW16T"] = str(v)
            y, gp, am = outs[v]
            ts[v].append(ev(lambda: ops.conv2d(x, wt, 3, 64, 3, bias=bias, out=y, gram_part=gp,
                                               out_amax=am), 10))
    G = [outs[v][1].view(nt, 64, 64).double().sum(0) for v in (0, 1)]
    zt = outs[1][0].double().view(64, -1)
    Gt = zt @ zt.t()
    print(f"conv1_1+gram  old {statistics.median(ts[0]) * 1e3:.1f} us  transposed "
          f"{statistics.median(ts[1]) * 1e3:.1f} us  y equal={torch.equal(outs[0][0], outs[1][0])}"
          f"  gram rel err old {float((G[0] - Gt).norm() / Gt.norm()):.2e} new "
          f"{float((G[1] - Gt).norm() / Gt.norm()):.2e}", flush=True)
    os.environ["STX_FEW16T"] = "1"

    print("== Gatys 512^2 iteration (graph replays)", flush=True)
    H = 512
    style = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H))).to(dev)
    content = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H))).to(dev)
    feat = V.VGGFeatures(V.load_vgg19_weights(), dev)
    engs = {}
    for v in (1, 2):
        setv(v - 1)
        engs[v] = V.GatysEngine(feat, style, content).capture(warmup=1)
    res = {1: [], 2: []}
    for _ in range(rounds):
        for v in (1, 2):
            res[v].append(ev(engs[v].step, 50))
    for v in (1, 2):
        torch.cuda.synchronize()
    same = torch.equal(engs[1].x, engs[2].x)
    m1, m2 = statistics.median(res[1]), statistics.median(res[2])
    print(f"gatys iteration: v1 {m1 * 1e3:.1f} us ({1e3 / m1:.0f} it/s)  v2 {m2 * 1e3:.1f} us "
          f"({1e3 / m2:.0f} it/s)  x{m1 / m2:.3f}  equal={same}", flush=True)

    print("== fast_st B=8 256^2 step (graph replays)", flush=True)
    from styletransfer_amd import network
    from styletransfer_amd.train import FastStTrainer
    st = torch.from_numpy(W.synthetic_image(3000, (1, 3, 256, 256))).to(dev)
    batch = torch.from_numpy(W.synthetic_image(4000, (8, 3, 256, 256))).to(dev)
    sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)}
    tr = {}
    for v in (1, 2):
        setv(v - 1)
        itn = network.ImageTransformNet(st, batch_size=8).to(dev)
        itn.load_state_dict(sd)
        t = FastStTrainer(itn, st)
        tr[v] = (t,) + t.capture(batch, warmup=1)
    res = {1: [], 2: []}
    for _ in range(rounds):
        for v in (1, 2):
            res[v].append(ev(tr[v][1], 10))
    same = torch.equal(tr[1][0].flat, tr[2][0].flat)
    m1, m2 = statistics.median(res[1]), statistics.median(res[2])
    print(f"fast_st step: v1 {m1 * 1e3:.1f} us ({8e3 / m1:.0f} img/s)  v2 {m2 * 1e3:.1f} us "
          f"({8e3 / m2:.0f} img/s)  x{m1 / m2:.3f}  equal={same}", flush=True)


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"done in {time.time() - t0:.1f} s")
