import torch, sys
a = torch.load(sys.argv[1]); b = torch.load(sys.argv[2])
names = "y mean rstd am du ga gb am2".split()
for k in a:
    diffs = [n for n, x, y in zip(names, a[k], b[k]) if not torch.equal(x, y)]
    print(k, "identical" if not diffs else "DIFF " + " ".join(f"{n}:{float((x-y).abs().max()):.3g}" for n, x, y in zip(names, a[k], b[k]) if not torch.equal(x, y)))
