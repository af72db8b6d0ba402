"""Time the streaming split Gram backward (gbwd16.hip) over shapes: HBM rate vs
plane geometry (power-of-two plane strides vs not)."""
import sys
import torch
sys.path.insert(0, ".")
from styletransfer_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)


def ev(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


for c, h, w in ((64, 512, 512), (64, 496, 512), (64, 512, 496), (64, 496, 496), (64, 480, 480),
                (128, 256, 256), (128, 240, 256), (128, 256, 240), (128, 240, 240)):
    z = torch.randn(1, c, h, w, device=dev)
    t = torch.randn(c, c, device=dev) * 0.01
    _, coef = ops.style_loss(z, t)
    dp = torch.randn(1, c, h // 2, w // 2, device=dev)
    dz = torch.empty_like(z)
    zam = ops.amax(z)
    ms = ev(lambda: ops.gram_bwd_fused(coef, z, out=dz, up_dp=dp, z_amax=zam))
    aux = torch.randn_like(z)
    msa = ev(lambda: ops.gram_bwd_fused(coef, z, out=dz, up_dp=dp, aux=aux, aux_scale=-0.5,
                                        z_amax=zam))
    cp = ev(lambda: dz.copy_(z))
    mb = 2.25 * c * h * w * 4 / 1e6
    mba = 3.25 * c * h * w * 4 / 1e6
    print(f"C{c} {h}x{w}: {ms * 1e3:7.1f} us {mb / (ms * 1e3):5.2f} TB/s | +aux {msa * 1e3:7.1f} us "
          f"{mba / (msa * 1e3):5.2f} TB/s | copy "
          f"{2 * c * h * w * 4 / 1e6 / (cp * 1e3):5.2f} TB/s", flush=True)
