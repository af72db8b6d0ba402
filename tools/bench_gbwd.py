"""Time the streaming split Gram backward (gbwd16.hip) at the Gatys shapes: the two loop
schedules (STX_GB_V1=1: run-time branches; 0: compile-time variants with ordered loads)
in one process, interleaved, with a bitwise comparison of their outputs."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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


for c, h, w, dp_on, aux_on in ((64, 512, 512, True, False), (128, 256, 256, True, True),
                               (256, 128, 128, False, False), (64, 256, 256, True, False),
                               (64, 496, 512, True, False)):
    z = torch.randn(1, c, h, w, device=dev)
    t = torch.randn(c, c, device=dev) * 0.01
    _, coef = ops.style_loss(z, t)
    dp = torch.randn(1, c, h // 2, w // 2, device=dev) if dp_on else None
    aux = torch.randn_like(z) if aux_on else None
    zam = ops.amax(z)
    outs, ts = {}, {0: [], 1: []}
    for v in (0, 1):
        os.environ["STX_GB_V1"] = str(v)
        outs[v] = torch.empty_like(z)
        ops.gram_bwd_fused(coef, z, out=outs[v], up_dp=dp, aux=aux, aux_scale=-0.5, z_amax=zam)
    for _ in range(5):
        for v in (0, 1):
            os.environ["STX_GB_V1"] = str(v)
            ts[v].append(ev(lambda: ops.gram_bwd_fused(coef, z, out=outs[v], up_dp=dp, aux=aux,
                                                       aux_scale=-0.5, z_amax=zam)))
    os.environ.pop("STX_GB_V1")
    nbytes = (2 + (0.25 if dp_on else 0) + (1 if aux_on else 0)) * c * h * w * 4
    m0, m1 = statistics.median(ts[0]) * 1e3, statistics.median(ts[1]) * 1e3
    print(f"C{c} {h}x{w} dp={int(dp_on)} aux={int(aux_on)}: v1 {m1:6.1f} us "
          f"{nbytes / m1 / 1e6:5.2f} TB/s | v2 {m0:6.1f} us {nbytes / m0 / 1e6:5.2f} TB/s"
          f"  equal={torch.equal(outs[0], outs[1])}", flush=True)
