"""Kernel-level numerics: every libstx kernel vs a plain PyTorch fp32 reference of
the same op (computed by torch on the same device).  Tolerances are stated per
test: rel = ||a-b|| / ||b|| over the whole tensor (fp32 MFMA is an exact fp32
fmaf chain; differences are summation-order rounding only)."""
import pytest
import torch
import torch.nn.functional as F

from styletransfer_amd import _native as N
from styletransfer_amd import ops

pytestmark = pytest.mark.gpu
TOL = 2e-5


def rel(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def rnd(*shape, dev, seed=0, scale=1.0, shift=0.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g) * scale + shift).to(dev)


def vinput(x, mode):
    if mode == N.STX_IN_RELU:
        return F.relu(x)
    if mode == N.STX_IN_RELU_POOL2:
        return F.max_pool2d(F.relu(x), 2, 2)
    if mode == N.STX_IN_UPSAMPLE2:
        return F.interpolate(x, scale_factor=2, mode="nearest")
    return x


CONV_CASES = [
    # n, cin, cout, h, w, ks, stride, mode
    (1, 3, 64, 37, 41, 3, 1, N.STX_IN_RAW),
    (2, 64, 64, 34, 70, 3, 1, N.STX_IN_RELU),
    (2, 64, 128, 34, 36, 3, 1, N.STX_IN_RELU_POOL2),
    (1, 128, 256, 40, 40, 3, 1, N.STX_IN_RELU_POOL2),
    (2, 128, 64, 12, 10, 3, 1, N.STX_IN_UPSAMPLE2),
    (2, 3, 32, 24, 20, 9, 1, N.STX_IN_RAW),
    (2, 32, 3, 24, 20, 9, 1, N.STX_IN_RAW),
    (2, 32, 64, 33, 30, 3, 2, N.STX_IN_RAW),
    (2, 64, 128, 64, 64, 3, 2, N.STX_IN_RAW),
    (2, 128, 128, 16, 16, 3, 1, N.STX_IN_RAW),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd(dev, case):
    n, cin, cout, h, w, ks, s, mode = case
    x = rnd(n, cin, h, w, dev=dev, seed=1, scale=2, shift=-1)
    wgt = rnd(cout, cin, ks, ks, dev=dev, seed=2, scale=0.2, shift=-0.1)
    b = rnd(cout, dev=dev, seed=3)
    wt = ops.conv_weight_prep(wgt)
    y = ops.conv2d(x, wt, cin, cout, ks, stride=s, in_mode=mode, bias=b)
    ref = F.conv2d(vinput(x, mode), wgt, b, stride=s, padding=ks // 2)
    torch.cuda.synchronize()
    assert y.shape == ref.shape
    assert rel(y, ref) < TOL


def test_conv_epilogue(dev):
    n, cin, cout, h, w = 2, 64, 64, 20, 36
    x = rnd(n, cin, h, w, dev=dev, seed=4, scale=2, shift=-1)
    wgt = rnd(cout, cin, 3, 3, dev=dev, seed=5, scale=0.2, shift=-0.1)
    mask = rnd(n, cout, h, w, dev=dev, seed=6, scale=2, shift=-1)
    aux = rnd(n, cout, h, w, dev=dev, seed=7)
    old = rnd(n, cout, h, w, dev=dev, seed=8)
    sc = torch.tensor(0.75, device=dev)
    wt = ops.conv_weight_prep(wgt)
    out = old.clone()
    ops.conv2d(x, wt, cin, cout, 3, mask=mask, aux=aux, aux_scale=-0.5, acc_scale=sc,
               accumulate=True, relu_out=True, out=out)
    ref = F.conv2d(x, wgt, padding=1) * 0.75
    ref = torch.where(mask > 0, ref, torch.zeros_like(ref)) - 0.5 * aux + old
    ref = F.relu(ref)
    assert rel(out, ref) < TOL


@pytest.mark.parametrize("case", [
    (2, 64, 64, 20, 36, 3, 1),
    (1, 128, 256, 16, 16, 3, 1),
    (2, 32, 64, 33, 30, 3, 2),
    (2, 64, 128, 32, 32, 3, 2),
    (2, 32, 3, 24, 20, 9, 1),
])
def test_conv_dgrad(dev, case):
    n, cin, cout, h, w, ks, s = case
    x = rnd(n, cin, h, w, dev=dev, seed=11, scale=2, shift=-1).requires_grad_()
    wgt = rnd(cout, cin, ks, ks, dev=dev, seed=12, scale=0.2, shift=-0.1)
    y = F.conv2d(x, wgt, stride=s, padding=ks // 2)
    dy = rnd(*y.shape, dev=dev, seed=13, scale=2, shift=-1)
    (ref,) = torch.autograd.grad(y, x, dy)
    wtT = ops.conv_weight_prep(wgt, transpose=True)
    if s == 1:
        dx = ops.conv2d(dy, wtT, cout, cin, ks)
    else:
        dx = ops.conv2d(dy, wtT, cout, cin, ks, in_mode=N.STX_IN_DILATE2, hv=h, wv=w)
    assert dx.shape == ref.shape
    assert rel(dx, ref) < TOL


@pytest.mark.parametrize("case", [
    (2, 64, 64, 20, 36, 3, 1, N.STX_IN_RAW),
    (2, 128, 128, 16, 16, 3, 1, N.STX_IN_RAW),
    (2, 32, 64, 33, 30, 3, 2, N.STX_IN_RAW),
    (2, 128, 64, 12, 10, 3, 1, N.STX_IN_UPSAMPLE2),
    (2, 3, 32, 24, 20, 9, 1, N.STX_IN_RAW),
    (2, 32, 3, 24, 20, 9, 1, N.STX_IN_RAW),
])
def test_conv_wgrad_bias(dev, case):
    n, cin, cout, h, w, ks, s, mode = case
    x = rnd(n, cin, h, w, dev=dev, seed=21, scale=2, shift=-1)
    wgt = rnd(cout, cin, ks, ks, dev=dev, seed=22, scale=0.2, shift=-0.1).requires_grad_()
    b = torch.zeros(cout, device=dev, requires_grad=True)
    y = F.conv2d(vinput(x, mode), wgt, b, stride=s, padding=ks // 2)
    dy = rnd(*y.shape, dev=dev, seed=23, scale=2, shift=-1)
    rw, rb = torch.autograd.grad(y, (wgt, b), dy)
    dw = ops.conv2d_wgrad(x, dy, cin, cout, ks, stride=s, in_mode=mode)
    db = ops.bias_grad(dy)
    assert rel(dw, rw) < TOL
    assert rel(db, rb) < TOL


@pytest.mark.parametrize("shape", [(1, 64, 32, 32), (2, 128, 16, 24), (1, 256, 8, 8),
                                   (1, 64, 512, 512), (3, 96, 7, 9)])
def test_gram_and_style_loss(dev, shape):
    b, c, h, w = shape
    z = rnd(*shape, dev=dev, seed=31, scale=2, shift=-0.5)
    t = rnd(1, c, h, w, dev=dev, seed=32)
    f = z.view(b, c, h * w)
    G = torch.bmm(f, f.transpose(1, 2)) / (c * h * w)
    ft = t.view(1, c, h * w)
    T = torch.bmm(ft, ft.transpose(1, 2)) / (c * h * w)
    g = ops.gram(z)
    assert rel(g, G) < TOL
    zr = z.clone().requires_grad_()
    fr = zr.view(b, c, h * w)
    loss_ref = F.mse_loss(torch.bmm(fr, fr.transpose(1, 2)) / (c * h * w), T.expand(b, c, c))
    (dz_ref,) = torch.autograd.grad(loss_ref * 3.0, zr)
    loss, coef = ops.style_loss(z, T[0].contiguous(), weight=3.0)
    assert rel(loss, loss_ref) < 1e-4
    dz = ops.gram_bwd(coef, z)
    assert rel(dz, dz_ref) < 1e-4


def test_mse_feature_content(dev):
    a = rnd(2, 128, 16, 16, dev=dev, seed=41, scale=2, shift=-1)
    b = rnd(2, 128, 16, 16, dev=dev, seed=42, scale=2, shift=-1)
    out = ops.mse(a, b)
    assert rel(out[0], F.mse_loss(a, b)) < 1e-5
    out = ops.mse(a, b, relu=True, mode=1)
    m = F.mse_loss(F.relu(a), F.relu(b))
    assert rel(out[0], m.pow(2) / a.numel()) < 1e-5
    assert rel(out[1], m) < 1e-5
    g = ops.diff_scale(a, b, 2.0 / a.numel())
    ar = a.clone().requires_grad_()
    (gr,) = torch.autograd.grad(F.mse_loss(ar, b), ar)
    assert rel(g, gr) < 1e-6


def test_maxpool_relu(dev):
    x = rnd(2, 8, 10, 14, dev=dev, seed=51, scale=2, shift=-1)
    x[0, 0, 0, :2] = 0.25  # ties
    x[0, 1, :2, :2] = -1.0  # all negative -> relu ties at 0
    y, idx = ops.maxpool2x2(x, relu_input=True)
    ry, ridx = F.max_pool2d(F.relu(x).cpu(), 2, 2, return_indices=True)
    assert torch.equal(y.cpu(), ry)
    assert torch.equal(idx.cpu(), ridx)
    dy = rnd(*y.shape, dev=dev, seed=52)
    dx = ops.maxpool2x2_bwd(dy, idx, 10, 14)
    xr = F.relu(x).cpu().requires_grad_()
    (rdx,) = torch.autograd.grad(F.max_pool2d(xr, 2, 2), xr, dy.cpu())
    assert torch.equal(dx.cpu(), rdx)
    # fused relu+pool backward from the pre-relu tensor
    dz = ops.relupool_bwd(dy, x)
    xr2 = x.cpu().requires_grad_()
    (rdz,) = torch.autograd.grad(F.max_pool2d(F.relu(xr2), 2, 2), xr2, dy.cpu())
    assert torch.equal(dz.cpu(), rdz)
    r = ops.relu(x)
    assert torch.equal(r, F.relu(x))
    assert torch.equal(ops.relu_bwd(x, r), torch.where(r > 0, x, torch.zeros_like(x)))


def test_adam(dev):
    n = 1001
    p = rnd(n, dev=dev, seed=61)
    g = rnd(n, dev=dev, seed=62, scale=2, shift=-1)
    pr = p.clone().cpu().requires_grad_()
    opt = torch.optim.Adam([pr])
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.zeros(16, dtype=torch.float32, device=dev)
    for it in range(3):
        gi = g * (it + 1)
        pr.grad = gi.cpu()
        opt.step()
        ops.adam_step(p, gi, m, v, step, ws)
    assert int(step.item()) == 3
    assert rel(p, pr.detach().to(dev)) < 1e-6


@pytest.mark.parametrize("n", [4096 * 1024 + 5, 3 * 512 * 512])
def test_adam_multiblock_graph(dev, n):
    """stx_adam_step_clear with many blocks and a grid-stride tail (n above the 4096-block
    cap, and not a multiple of 4), replayed from a captured hipGraph: torch.optim.Adam's
    update on every step, the device counter after each, the clear buffer zeroed."""
    p = rnd(n, dev=dev, seed=65)
    g = rnd(n, dev=dev, seed=66, scale=2, shift=-1)
    pr = p.clone().cpu().requires_grad_()
    opt = torch.optim.Adam([pr], lr=0.01)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.zeros(16, dtype=torch.float32, device=dev)
    clear = torch.full((300,), 2.0, device=dev)
    ops.adam_step(p, g, m, v, step, ws, lr=0.01, clear=clear)  # eager first step
    pr.grad = g.cpu()
    opt.step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with ops.graph_capture(graph, stream=s):
        ops.adam_step(p, g, m, v, step, ws, lr=0.01, clear=clear)
    for it in range(4):
        clear.fill_(1.0)
        graph.replay()
        pr.grad = g.cpu()
        opt.step()
        torch.cuda.synchronize()
        assert int(step.item()) == it + 2
        assert float(clear.abs().max()) == 0.0
    assert rel(p, pr.detach().to(dev)) < 1e-6


def test_graph_capture_with_cyclic_garbage(dev):
    """ops.graph_capture: a CUDAGraph left in a reference cycle (a finished engine) must not
    be collected while another stream captures -- HIP refuses the destruction mid-capture
    (hipErrorStreamCaptureUnsupported, an abort).  The capture body here allocates enough
    Python objects to cross the collector's thresholds; the helper collected before and
    holds the collector off until the capture ends."""
    import gc

    class Engine:
        pass

    x = torch.ones(1024, device=dev)  # (captured work runs only on replay)
    for _ in range(3):
        e = Engine()
        e.me = e  # a cycle: only the cyclic collector frees it
        e.graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with ops.graph_capture(e.graph):
                x.add_(1.0)
        torch.cuda.current_stream().wait_stream(s)
        del e
    assert gc.isenabled()
    g2 = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with ops.graph_capture(g2):
            junk = []
            for i in range(20000):  # well past gc's generation-0 threshold
                d = {"i": i}
                d["self"] = d
                junk.append(d)
            x.mul_(2.0)
    torch.cuda.current_stream().wait_stream(s)
    assert gc.isenabled()
    g2.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 2.0  # only g2 replayed


def test_adam_step_clear(dev):
    """stx_adam_step_clear (the Gatys engine's Adam launch that also zeroes its amax
    groups for the next iteration): the same update bits as stx_adam_step, and the clear
    buffer zeroed (sizes below, at and above one 256-thread pass)."""
    for nclear in (7, 256, 512, 1000):
        n = 4099
        p = rnd(n, dev=dev, seed=63)
        g = rnd(n, dev=dev, seed=64, scale=2, shift=-1)
        st = [(p.clone(), torch.zeros_like(p), torch.zeros_like(p),
               torch.zeros(1, dtype=torch.int32, device=dev),
               torch.zeros(16, dtype=torch.float32, device=dev)) for _ in range(2)]
        clear = torch.full((nclear,), 3.0, device=dev)
        for it in range(2):
            ops.adam_step(st[0][0], g * (it + 1), *st[0][1:])
            ops.adam_step(st[1][0], g * (it + 1), *st[1][1:], clear=clear)
            assert float(clear.abs().max()) == 0.0
            clear.fill_(5.0)
        assert torch.equal(st[0][0], st[1][0]) and int(st[1][3].item()) == 2


@pytest.mark.parametrize("relu,res,hw,nc", [(False, False, (12, 20), None),
                                            (True, False, (12, 20), None),
                                            (False, True, (12, 20), None),
                                            (True, True, (64, 64), None),
                                            (True, False, (128, 128), None),
                                            (False, True, (256, 256), None),
                                            (True, False, (7, 9), None),
                                            # the 256^2 ReLU backward (greg kernel), and the
                                            # pipelined 64^2 kernels (>= 1024 planes, B = 8)
                                            (True, False, (256, 256), None),
                                            (True, False, (64, 64), (8, 128)),
                                            (True, True, (64, 64), (8, 128))])
def test_instnorm(dev, relu, res, hw, nc):
    """InstanceNorm (+res, +ReLU) forward/backward on every kernel variant (register-
    resident planes up to 64^2 / 128^2 / 256^2, the loop kernels otherwise) and the
    max|.| annotations of y and du.  The backward recomputes the ReLU decision from x
    (+ res) and the saved statistics (stx_instnorm_bwd takes beta, not y): du must equal
    the fp64 backward through the mask of the HIP forward's own y (a decision that differs
    from y > 0 anywhere would be an O(1) error there)."""
    n, c = nc if nc else (2, 32 if hw == (12, 20) else 4)
    x = rnd(n, c, *hw, dev=dev, seed=71, scale=3, shift=-1).requires_grad_()
    r = rnd(n, c, *hw, dev=dev, seed=72).requires_grad_() if res else None
    gamma = rnd(c, dev=dev, seed=73, shift=0.5).requires_grad_()
    beta = rnd(c, dev=dev, seed=74).requires_grad_()
    u = x + r if res else x
    ref = F.instance_norm(u, weight=gamma, bias=beta, eps=1e-5)
    if relu:
        ref = F.relu(ref)
    ya = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
    y, mean, rstd = ops.instnorm_fwd(x.detach(), gamma.detach(), beta.detach(),
                                     res=r.detach() if res else None, relu=relu, out_amax=ya)
    assert rel(y, ref) < 1e-5
    assert float(ya.max()) == float(y.abs().max())
    dy = rnd(*y.shape, dev=dev, seed=75, scale=2, shift=-1)
    grads = torch.autograd.grad(ref, [x, gamma, beta], dy)
    dg = torch.empty(c, device=dev)
    db = torch.empty(c, device=dev)
    da = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
    du = ops.instnorm_bwd(dy, beta.detach(), x.detach(), r.detach() if res else None,
                          gamma.detach(), mean, rstd, relu=relu, dgamma=dg, dbeta=db, out_amax=da)
    assert rel(du, grads[0]) < 1e-4
    assert rel(dg, grads[1]) < 1e-5
    assert rel(db, grads[2]) < 1e-5
    assert float(da.max()) == float(du.abs().max())
    # the same backward in fp64 through the HIP forward's own ReLU decisions (y > 0)
    u64 = (x + r if res else x).detach().double().cpu()
    hw_ = u64[0, 0].numel()
    mu64 = u64.mean(dim=(2, 3), keepdim=True)
    rs64 = 1.0 / torch.sqrt(u64.var(dim=(2, 3), unbiased=False, keepdim=True) + 1e-5)
    xh = (u64 - mu64) * rs64
    g64 = dy.double().cpu() * ((y.cpu() > 0).double() if relu else 1.0)
    gm = gamma.detach().double().cpu().view(1, -1, 1, 1)
    du64 = gm * rs64 / hw_ * (hw_ * g64 - g64.sum(dim=(2, 3), keepdim=True)
                              - xh * (g64 * xh).sum(dim=(2, 3), keepdim=True))
    assert rel(du.cpu(), du64) < 1e-5, rel(du.cpu(), du64)


def test_upsample_tv(dev):
    x = rnd(2, 3, 5, 7, dev=dev, seed=81)
    assert torch.equal(ops.upsample2x(x), F.interpolate(x, scale_factor=2, mode="nearest"))
    dy = rnd(2, 3, 10, 14, dev=dev, seed=82)
    xr = x.clone().requires_grad_()
    (rdx,) = torch.autograd.grad(F.interpolate(xr, scale_factor=2, mode="nearest"), xr, dy)
    assert rel(ops.upsample2x_bwd(dy), rdx) < 1e-6
    y = rnd(2, 3, 20, 24, dev=dev, seed=83, scale=3, shift=-1)
    yr = y.clone().requires_grad_()
    ref = 1e-6 * (torch.sum(torch.abs(yr[:, :, :, :-1] - yr[:, :, :, 1:]))
                  + torch.sum(torch.abs(yr[:, :, :-1, :] - yr[:, :, 1:, :])))
    (rg,) = torch.autograd.grad(ref, yr)
    g = torch.empty_like(y)
    loss = ops.tv_loss(y, 1e-6, grad=g)
    assert rel(loss, ref) < 1e-5
    assert rel(g, rg) < 1e-6


def test_conv_fused_gram_phase_and_unpool(dev):
    """dgrad conv with fused ReLU mask + Gram-backward phase, and the 1x1 Gram-backward
    conv with the fused ReLU+MaxPool backward epilogue, vs unfused torch."""
    n, c, h, w = 2, 64, 20, 36
    z = rnd(n, c, h, w, dev=dev, seed=91, scale=2, shift=-1)
    dy = rnd(n, c, h, w, dev=dev, seed=92, scale=2, shift=-1)
    wgt = rnd(c, c, 3, 3, dev=dev, seed=93, scale=0.2, shift=-0.1)
    t = rnd(c, c, dev=dev, seed=94)
    loss, coef = ops.style_loss(z, t, weight=2.0)
    s2 = torch.tensor(0.5, device=dev)
    wtT = ops.conv_weight_prep(wgt, transpose=True)
    out = ops.conv2d(dy, wtT, c, c, 3, mask=z, p2_z=z, p2_coef=coef, p2_scale=s2)
    xr = z.clone().requires_grad_()
    (ref_d,) = torch.autograd.grad(F.conv2d(xr, wgt, padding=1), xr, dy)
    ref = torch.where(z > 0, ref_d, torch.zeros_like(ref_d)) + 0.5 * ops.gram_bwd(coef, z)
    assert rel(out, ref) < TOL
    # unpool epilogue: out = s*A.z + unpool(dp)*(z>0)
    dp = rnd(n, c, h // 2, w // 2, dev=dev, seed=95, scale=2, shift=-1)
    aux = rnd(n, c, h, w, dev=dev, seed=96)
    out2 = ops.gram_bwd_fused(coef, z, acc_scale=s2, up_dp=dp, aux=aux, aux_scale=-0.25)
    ref2 = 0.5 * ops.gram_bwd(coef, z) + ops.relupool_bwd(dp, z) - 0.25 * aux
    assert rel(out2, ref2) < TOL


@pytest.mark.parametrize("case", [(1, 64, 3, 37, 70), (2, 64, 3, 16, 64), (2, 32, 9, 24, 20),
                                  (1, 32, 9, 9, 130), (3, 32, 3, 8, 8)])
def test_conv_fewin(dev, case):
    """3-input-channel convs (convfew.hip: VGG conv1_1, ITN conv0 / conv22 dgrad) vs
    fp64, ragged tiles, bias + relu_out + out_amax epilogue.  They run on the fp16
    hi/lo split MFMA with block-local scales (fp32-class: 2e-6 of fp64, as every
    split kernel in test_conv_split_gpu.py)."""
    n, cout, ks, h, w = case
    x = rnd(n, 3, h, w, dev=dev, seed=21, scale=2, shift=-1)
    wgt = rnd(cout, 3, ks, ks, dev=dev, seed=22, scale=0.2, shift=-0.1)
    b = rnd(cout, dev=dev, seed=23)
    wt = ops.conv_weight_prep(wgt)
    am = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
    y = ops.conv2d(x, wt, 3, cout, ks, bias=b, out_amax=am)
    ref = F.conv2d(x.double(), wgt.double(), b.double(), padding=ks // 2)
    assert rel(y, ref) < 2e-6
    assert float(am.max()) == float(y.abs().max())
    yr = ops.conv2d(x, wt, 3, cout, ks, bias=b, relu_out=True)
    assert rel(yr, F.relu(ref)) < 2e-6
    # an input tile of zeros next to a large one (block-local scales) stays exact
    x2 = x.clone()
    x2[..., : x.shape[-1] // 2] = 0
    x2[..., x.shape[-1] // 2:] *= 1e4
    y2 = ops.conv2d(x2, wt, 3, cout, ks, bias=b)
    assert rel(y2, F.conv2d(x2.double(), wgt.double(), b.double(), padding=ks // 2)) < 2e-6


@pytest.mark.parametrize("case", [(1, 3, 37, 70, N.STX_IN_RAW), (2, 3, 16, 64, N.STX_IN_RELU),
                                  (2, 1, 9, 130, N.STX_IN_RAW), (1, 2, 64, 64, N.STX_IN_RAW)])
def test_conv_fewout(dev, case):
    """<= 3-output-channel 3x3 convs (convfew.hip GEMM + col2im: VGG conv1_1's data
    gradient to the image) vs fp64, ragged tiles, bias/accumulate/relu_out."""
    n, cout, h, w, mode = case
    x = rnd(n, 64, h, w, dev=dev, seed=31, scale=2, shift=-1)
    wgt = rnd(cout, 64, 3, 3, dev=dev, seed=32, scale=0.2, shift=-0.1)
    b = rnd(cout, dev=dev, seed=33)
    old = rnd(n, cout, h, w, dev=dev, seed=34)
    wt = ops.conv_weight_prep(wgt)
    ref = F.conv2d(vinput(x, mode).double(), wgt.double(), b.double(), padding=1)
    y = ops.conv2d(x, wt, 64, cout, 3, in_mode=mode, bias=b)
    assert rel(y, ref) < 1e-6
    out = old.clone()
    ops.conv2d(x, wt, 64, cout, 3, in_mode=mode, bias=b, out=out, accumulate=True,
               relu_out=True)
    assert rel(out, F.relu(ref + old.double())) < 1e-6
    # with a bound on max|x| (the Gatys backward passes conv1_2's out_amax): the split
    # MFMA kernel, fp32-class (2e-6 of fp64)
    am = ops.amax(x)
    y16 = ops.conv2d(x, wt, 64, cout, 3, in_mode=mode, bias=b, in_amax=am)
    assert rel(y16, ref) < 2e-6
    out = old.clone()
    ops.conv2d(x, wt, 64, cout, 3, in_mode=mode, bias=b, out=out, accumulate=True,
               relu_out=True, in_amax=am)
    assert rel(out, F.relu(ref + old.double())) < 2e-6
