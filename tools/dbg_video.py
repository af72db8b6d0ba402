import sys, torch
sys.path.insert(0, '.')
from styletransfer_amd import network, video
from styletransfer_amd import weights as W
dev = torch.device('cuda', 0)
sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(777, in_channels=6)}
frames = [torch.from_numpy(W.synthetic_image(900 + t, (1, 3, 64, 64))) for t in range(4)]
def rel(a, b): return float((a.cpu().double() - b.cpu().double()).norm() / b.cpu().double().norm())
def poison(sizes):
    ts = [torch.full((n,), float('nan'), device=dev) for n in sizes for _ in range(4)]
    torch.cuda.synchronize()
    del ts
ref = None
ALL = (1 << 10, 1 << 12, 12288, 1 << 14, 1 << 16, 1 << 18, 1 << 20, 1 << 22)
for name, sizes in [("none", ()), ("all", ALL)] + [(f"s{n}", (n,)) for n in ALL]:
    net = network.VideoTransformNet(torch.rand([3, 64, 64])); net.load_state_dict(sd)
    eng = video.FrameEngine(net, (1, 3, 64, 64), dev, graph=True)
    outs, info = [], []
    for t, f in enumerate(frames):
        if t >= 2: poison(sizes)
        outs.append(eng.step(f.to(dev)).clone().cpu())
        info.append((round(float(eng.scal[0]), 3), round(float(eng.scal[1]), 3)))
    if ref is None: ref = outs
    print(name, [round(rel(a, b), 4) for a, b in zip(outs, ref)], 'same-as-prev',
          [bool(torch.equal(outs[t], outs[t-1])) for t in range(1, 4)], info)
