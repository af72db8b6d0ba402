"""Same-process A/B of whole-step settings: the Gatys 512^2 iteration and the fast_st B=8
256^2 training step, each built and hipGraph-captured once under every environment
variant, then replayed in interleaved rounds (median per variant) and compared bit for
bit against the first variant.

    python tools/ab_engine.py "STX_FIN_BATCH=0" "STX_FIN_BATCH=1" [--rounds 7] [--no-fast] [--no-gatys]

A variant is a comma-separated list of NAME=VALUE settings applied while that variant's
engine is built and captured (the library reads its switches at launch/capture time).
The process runs the A/B build of the library (`make AB=1`: libstx_ab.so, whose STX_KNOB
switches read the environment; the product build compiles them to their defaults) unless
STX_LIB names another."""
import os
import statistics
import sys

import torch

# the library's own switches (STX_KNOB) read the environment only in the A/B build
os.environ.setdefault("STX_LIB", os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "styletransfer_amd", "libstx_ab.so"))

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import vgg as V  # noqa: E402
from styletransfer_amd import weights as W  # noqa: E402


def ev(fn, reps):
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


class Env:
    def __init__(self, spec):
        # STX_AB=1: the host path's A/B switches read the environment only then (N.knob)
        self.kv = dict([("STX_AB", "1")] + [x.split("=", 1) for x in spec.split(",") if x])
        self.old = {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds = 7
    if "--rounds" in sys.argv:
        rounds = int(sys.argv[sys.argv.index("--rounds") + 1])
        args = [a for a in args if a != str(rounds)]
    dev = torch.device("cuda", 0)
    H = 512
    style = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H))).to(dev)
    content = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H))).to(dev)
    feat = V.VGGFeatures(V.load_vgg19_weights(), dev)
    engs = []
    for spec in ([] if "--no-gatys" in sys.argv else args):
        with Env(spec):
            engs.append(V.GatysEngine(feat, style, content).capture(warmup=1))
    res = [[] for _ in args]
    for _ in range(rounds):
        for i, e in enumerate(engs):
            res[i].append(ev(e.step, 50))
    for i, spec in enumerate(args[:len(engs)]):
        m = statistics.median(res[i])
        same = torch.equal(engs[i].x, engs[0].x)
        print(f"gatys  {spec:40s} {m * 1e3:8.1f} us  {1e3 / m:7.0f} it/s  min {min(res[i]) * 1e3:.1f}"
              f"  equal_to_first={same}", flush=True)
    if "--no-fast" in sys.argv:
        return
    from styletransfer_amd import network
    from styletransfer_amd.train import FastStTrainer
    st = torch.from_numpy(W.synthetic_image(3000, (1, 3, 256, 256))).to(dev)
    batch = torch.from_numpy(W.synthetic_image(4000, (8, 3, 256, 256))).to(dev)
    sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)}
    trs = []
    for spec in args:
        with Env(spec):
            itn = network.ImageTransformNet(st, batch_size=8).to(dev)
            itn.load_state_dict(sd)
            t = FastStTrainer(itn, st)
            trs.append((t,) + t.capture(batch, warmup=1))
    res = [[] for _ in args]
    for _ in range(rounds):
        for i, t in enumerate(trs):
            res[i].append(ev(t[1], 10))
    for i, spec in enumerate(args):
        m = statistics.median(res[i])
        same = torch.equal(trs[i][0].flat, trs[0][0].flat)
        print(f"fastst {spec:40s} {m * 1e3:8.1f} us  {8e3 / m:7.0f} img/s  min "
              f"{min(res[i]) * 1e3:.1f}  equal_to_first={same}", flush=True)


if __name__ == "__main__":
    main()
