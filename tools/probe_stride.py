"""Probe: does a power-of-two channel-plane stride (NCHW at 512^2 / 256^2) slow the
channel-strided reads of the HBM-bound kernels?  torch's dim-0 reduction of a [C, HW]
tensor reads C rows at the plane stride per output element -- the access pattern of
conv_fewout16 / gram_bwd16; the same reduction over a padded plane stride (HW + pad)
and a plain contiguous read are timed beside it."""
import torch


def ev(fn, reps=50):
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


dev = torch.device("cuda", 0)
for C, HW in ((64, 512 * 512), (64, 256 * 256 * 8), (128, 256 * 256)):
    for pad in (0, 64, 256, 1024, 4096):
        base = torch.randn(C, HW + pad, device=dev)
        x = base[:, :HW]
        out = torch.empty(HW, device=dev)
        ms = ev(lambda: torch.sum(x, 0, out=out))
        print(f"C={C} HW={HW} pad={pad:5d}: dim-0 sum {ms * 1e3:7.1f} us  "
              f"{C * HW * 4 / ms / 1e9:6.2f} TB/s", flush=True)
    y = torch.randn(C * HW, device=dev)
    ms = ev(lambda: y.sum())
    print(f"C={C} HW={HW}: contiguous sum {ms * 1e3:7.1f} us  {C * HW * 4 / ms / 1e9:6.2f} TB/s")
    z = torch.empty_like(y)
    ms = ev(lambda: z.copy_(y))
    print(f"C={C} HW={HW}: copy {ms * 1e3:7.1f} us  {2 * C * HW * 4 / ms / 1e9:6.2f} TB/s", flush=True)
