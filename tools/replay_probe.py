"""Why does a 20-replay window of the Gatys graph run slower per iteration than a 500-replay
run?  Host time per graph.replay() call, GPU time per replay (events
between replays), and the timed() window at several lengths, back to back in one process."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from styletransfer_amd import vgg as V, weights as W  # noqa: E402


def window(eng, k, dev):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(k):
        eng.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    return (t2 - t0) / k * 1e3, (t1 - t0) / k * 1e3


def main():
    dev = torch.device("cuda", 0)
    H = 512
    s = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H))).to(dev)
    c = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H))).to(dev)
    eng = V.GatysEngine(V.VGGFeatures(V.load_vgg19_weights(), dev), s, c)
    eng.capture(warmup=1)
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize(dev)
    # per-replay GPU time (events after each replay) and host time per call
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
    host = []
    evs[0].record()
    for i in range(40):
        t0 = time.perf_counter()
        eng.step()
        host.append((time.perf_counter() - t0) * 1e3)
        evs[i + 1].record()
    torch.cuda.synchronize(dev)
    gpu = [evs[i].elapsed_time(evs[i + 1]) for i in range(40)]
    print("host ms per replay call:", " ".join(f"{h:.3f}" for h in host[:12]), "... median",
          f"{sorted(host)[20]:.3f}")
    print("gpu ms per replay      :", " ".join(f"{g:.3f}" for g in gpu[:12]), "... median",
          f"{sorted(gpu)[20]:.3f}")
    for k in (5, 20, 20, 20, 50, 100, 500, 20, 20):
        wall, enq = window(eng, k, dev)
        print(f"window {k:4d}: {wall:.4f} ms/iter wall ({1e3 / wall:.1f} it/s), host enqueue "
              f"{enq:.4f} ms/iter")


if __name__ == "__main__":
    main()
