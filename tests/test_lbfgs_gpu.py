"""On-device L-BFGS (styletransfer_amd.optim.LBFGS) vs torch.optim.LBFGS.

StyleNetwork.train_gatys runs `optim.LBFGS` with its defaults
(stransfer/network.py:435); our LBFGS restates torch's algorithm on libstx vector
kernels.  Same closure, same inputs: trajectories must agree to reduction-order
rounding (dot products are summed in a different order)."""
import numpy as np
import pytest
import torch

from styletransfer_amd import network
from styletransfer_amd import optim as stx_optim
from styletransfer_amd import weights as W

pytestmark = pytest.mark.gpu


def quad_problem(dev, n=4096, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    m = (torch.randn(n, generator=g).abs() + 0.5).to(dev)     # diagonal curvature
    b = torch.randn(n, generator=g).to(dev)
    x0 = torch.randn(n, generator=g).to(dev)
    return m, b, x0


@pytest.mark.parametrize("history,n", [(100, 4096), (3, 4096), (1, 4096), (100, 4093),
                                       (5, 2500)])
def test_lbfgs_matches_torch_on_quadratic(dev, history, n):
    """history 1 / 3 / 5 evict from the ring within the 4 steps; n = 4093 / 2500 are not
    multiples of the 1024-element history chunk (padded slots, ragged tail).
    The compact form and torch's two-loop recursion agree in exact arithmetic; in fp32
    their roundings differ and 4 steps x 20 iterations amplify them (the CPU restatement
    of the compact form lands 1e-7 .. 3e-5 from torch's CPU run; on the GPU both fp32 runs
    land 1e-6 .. 2e-4 from fp64, case by case either one nearer), so the end point is held
    against torch's fp64 run: within 5x torch fp32's own distance from it (floor 1e-4)."""
    m, b, x0 = quad_problem(dev, n)
    xs = []
    runs = ((torch.optim.LBFGS, dev, torch.float32), (stx_optim.LBFGS, dev, torch.float32),
            (torch.optim.LBFGS, "cpu", torch.float64))
    for cls, where, dt in runs:
        mm, bb = m.to(where, dt), b.to(where, dt)
        x = x0.clone().to(where, dt).view(1, -1).requires_grad_()
        opt = cls([x], history_size=history)

        def closure():
            opt.zero_grad()
            f = 0.5 * ((mm * x.view(-1) - bb) ** 2).sum() + 0.1 * (x ** 4).sum()
            f.backward()
            return f

        for _ in range(4):
            opt.step(closure)
        xs.append(x.detach().double().cpu().clone())
    ref32, ours, ref64 = xs
    rel = lambda a, c: float((a - c).norm() / c.norm())  # noqa: E731
    e_ours, e_ref = rel(ours, ref64), rel(ref32, ref64)
    print(f"history {history} n {n}: ours vs fp64 {e_ours:.2e}, torch fp32 vs fp64 {e_ref:.2e}, "
          f"ours vs torch fp32 {rel(ours, ref32):.2e}")
    assert e_ours <= max(5 * e_ref, 1e-4), (e_ours, e_ref)
    assert rel(ours, ref32) < 1e-3


def test_lbfgs_gatys(dev):
    """train_gatys (L-BFGS) on the HIP closure: the native optimiser and torch's give
    the same losses after two outer steps."""
    s = torch.from_numpy(W.synthetic_image(21, (1, 3, 64, 64))).to(dev)
    c = torch.from_numpy(W.synthetic_image(22, (1, 3, 64, 64))).to(dev)
    finals = []
    for cls in (torch.optim.LBFGS, stx_optim.LBFGS):
        net = network.StyleNetwork(s, c)
        x = c.clone()
        opt = cls([x.requires_grad_()])

        def closure():
            opt.zero_grad()
            net(x, c)
            tot = net.get_total_current_style_loss(100_000) + net.get_total_current_content_loss(1)
            tot.backward()
            return tot

        def value():
            with torch.no_grad():
                net(x, c)
                return float(net.get_total_current_style_loss(100_000)
                             + net.get_total_current_content_loss(1))

        first = value()
        for _ in range(2):
            opt.step(closure)
        finals.append(value())
    assert finals[1] < 0.5 * first
    # 40 closure evaluations of a non-convex loss amplify fp32 reassociation between
    # torch's and our dot products (0.1-0.6 % end-point spread observed as the loss
    # reductions' summation order changed between builds).  This is a smoke check of
    # the optimiser on the real closure: the step-for-step equivalence is pinned at 1e-4
    # by test_lbfgs_matches_torch_on_quadratic, and train_gatys against the reference's
    # own L-BFGS run in fp64 three-way form by test_train_gatys_lbfgs_reference.
    assert abs(finals[0] - finals[1]) <= 1e-2 * abs(finals[0]), finals


def _gatys_lbfgs_fp64_losses(feat, s, c, n_evals, sw=100_000, cw=1):
    """Losses of torch.optim.LBFGS (reference defaults) in float64 on the Gatys closure
    sw * sum_l mse(gram(Z_l), gram(Z_l(style))) + cw * mse(Z_4, Z_4(content)) from the
    content image (stransfer/network.py:411-458), the first n_evals evaluations."""
    import forced_ref as R
    vw = [(w.double(), bb.double()) for w, bb in zip(feat.w, feat.b)]
    s64, c64 = s.double(), c.double()
    with torch.no_grad():
        targets = [R.gram(z) for z in R.vgg_forward(vw, s64)]
        c4 = R.vgg_forward(vw, c64)[3]
    x = c64.clone().requires_grad_()
    opt = torch.optim.LBFGS([x])
    out = []

    def closure():
        opt.zero_grad()
        zs = R.vgg_forward(vw, x)
        style = sum(torch.nn.functional.mse_loss(R.gram(z), t) for z, t in zip(zs, targets))
        total = sw * style + cw * torch.nn.functional.mse_loss(zs[3], c4)
        total.backward()
        out.append(float(total))
        return total
    while len(out) < n_evals:
        opt.step(closure)
    return np.array(out[:n_evals])


def test_gatys_lbfgs_engine_matches_torch_control_flow(dev):
    """vgg.GatysLBFGS (graph replays, one host read per iteration, the opening
    evaluation of a step reused from the previous iteration's graph) against
    torch.optim.LBFGS driving the SAME closure (the engine's eager loss evaluation):
    identical evaluation counts per outer step and the same losses up to the
    direction's rounding (compact form vs torch's two-loop recursion)."""
    from styletransfer_amd import vgg as V
    H = 64
    s = torch.from_numpy(W.synthetic_image(31, (1, 3, H, H))).to(dev)
    c = torch.from_numpy(W.synthetic_image(32, (1, 3, H, H))).to(dev)
    feat = V.VGGFeatures(V.load_vgg19_weights(), dev)
    # torch's optimiser over the engine's eager closure
    ref = V.GatysLBFGS(feat, s, c)
    x = ref.x
    opt = torch.optim.LBFGS([x])
    ref_losses, ref_evals = [], []

    def closure():
        ref._closure()
        x.grad = ref.grad
        ref_losses.append(float(ref.total))
        return ref.total.clone()

    for _ in range(4):
        opt.step(closure)
        ref_evals.append(opt.state[x]["func_evals"])
    eng = V.GatysLBFGS(feat, s, c)
    losses, evals = [], []
    for _ in range(4):
        eng.step(on_eval=losses.append)
        evals.append(eng.func_evals)
    assert evals == ref_evals, (evals, ref_evals)
    assert len(losses) == len(ref_losses)
    got, want = np.array(losses), np.array(ref_losses)
    err = np.abs(got - want) / np.abs(want)
    assert err[:6].max() < 1e-4, err[:6]
    # the whole trajectory three-way: torch.optim.LBFGS in fp64 over an fp64 restatement
    # of the same closure (tests/forced_ref.py: VGG prefix + Gram / content MSE, pinned to
    # the reference by test_forced_ref_pin.py); per evaluation, the engine's loss error
    # against it is held to 3x the error of torch's fp32 optimiser on the engine closure
    # (fp32 rounding, amplified the same way along the trajectory), floor 1e-5
    l64 = _gatys_lbfgs_fp64_losses(feat, s, c, len(losses))
    e_ours = np.abs(got - l64) / np.abs(l64)
    e_t32 = np.abs(want - l64) / np.abs(l64)
    print(f"engine vs fp64 max {e_ours.max():.2e}, torch fp32 vs fp64 max {e_t32.max():.2e}")
    assert e_ours.max() <= max(3 * e_t32.max(), 1e-5), (e_ours.max(), e_t32.max())
    # every graph evaluation is one torch makes (the last step's closing evaluation is the
    # next step's opening one), but for stops on g.d (none expected here)
    assert eng.closure_runs <= eng.func_evals + 1, (eng.closure_runs, eng.func_evals)
    pairs, n_iter = eng.history()
    assert n_iter == opt.state[x]["n_iter"] and 0 < pairs <= 100


def _lb_hdr(opt):
    """(count, n_iter, cand, accepted, H_diag, t, order) of the device state block
    (lbfgs.hip LbHdr: 8 ints, 8 floats, order[257])."""
    st = opt._buf["state"]
    iv = st[:32].view(torch.int32).cpu()
    fv = st[32:64].view(torch.float32).cpu()
    count = int(iv[0])
    order = st[64:64 + 4 * 257].view(torch.int32).cpu()[:count].tolist()
    return dict(count=count, n_iter=int(iv[1]), cand=int(iv[2]), accepted=int(iv[4]),
                H_diag=float(fv[0]), t=float(fv[1]), order=order)


def _two_loop(S, Y, g, H_diag):
    """torch.optim.LBFGS's two-loop recursion (torch/optim/lbfgs.py, the direction of
    StyleNetwork.train_gatys' optimiser) over pairs oldest first, in the dtype given."""
    ro = [1.0 / torch.dot(y, s) for s, y in zip(S, Y)]
    q = -g.clone()
    al = [None] * len(S)
    for i in range(len(S) - 1, -1, -1):
        al[i] = torch.dot(S[i], q) * ro[i]
        q.add_(Y[i] * -al[i])
    r = q * H_diag
    for i in range(len(S)):
        be = torch.dot(Y[i], r) * ro[i]
        r.add_(S[i] * (al[i] - be))
    return r


def test_gatys_lbfgs_512_history100_direction_vs_fp64(dev):
    """The benched L-BFGS configuration (vgg.GatysLBFGS at 512^2, history 100, from a
    noise image as bench.py's gatys_lbfgs leg) run until the ring is full and has evicted
    (> 100 accepted pairs), then ONE more direction (stx_lbfgs_direction: pair update with
    eviction, compact-form solve, combine) from that state, three-way: its t*d against
    torch's two-loop recursion in fp64 over the same (fp32-stored) pairs, held to 3x the
    error of the same two-loop in fp32 on the GPU (torch's own arithmetic).  The call is
    repeated from a restored copy of the state: x, the history slabs, the state block and
    the scalars must come out bit-identical (the solve has no data race)."""
    from styletransfer_amd import vgg as V
    H = 512
    s = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H))).to(dev)
    c = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H))).to(dev)
    gen = torch.Generator().manual_seed(3000)
    noise = torch.rand((1, 3, H, H), generator=gen).to(dev)
    eng = V.GatysLBFGS(V.VGGFeatures(V.load_vgg19_weights(), dev), s, c, init=noise).capture()
    opt = eng.opt
    steps = 0
    while steps < 16:  # until the full ring has evicted (slot 100 in use)
        eng.step()
        steps += 1
        if opt.state[eng.x]["n_iter"] > 115 and eng.history()[0] == 100 and \
                sorted(_lb_hdr(opt)["order"]) != list(range(100)):
            break
    hdr0 = _lb_hdr(opt)
    assert hdr0["count"] == 100 and hdr0["n_iter"] > 101, hdr0
    assert sorted(hdr0["order"]) != list(range(100)), "ring has not wrapped"
    b = opt._buf
    n, m1 = b["n"], 101
    npad = b["hist"].numel() // (2 * m1)
    saved = {k: b[k].clone() for k in ("hist", "state", "prev_g", "scal", "ws")}
    x0, g = eng.x.clone(), eng.grad.view(-1).clone()

    def run_once():
        for k, v in saved.items():
            b[k].copy_(v)
        eng.x.copy_(x0)
        opt.direction(g)
        torch.cuda.synchronize()
        return (eng.x.clone(), b["hist"].clone(), b["state"].clone(), b["scal"].clone())

    out1 = run_once()
    out2 = run_once()
    for a, c2, what in zip(out1, out2, ("x", "hist", "state", "scal")):
        assert torch.equal(a, c2), f"direction not reproducible: {what}"
    hdr = _lb_hdr(opt)
    hist = b["hist"]
    # the reference's pair update from the saved state (torch: y = g - prev_g,
    # s = t_prev d_prev, accepted when y.s > 1e-10, the oldest pair evicted when full)
    sv = saved["hist"][hdr0["cand"] * npad:hdr0["cand"] * npad + n]
    yv = g - saved["prev_g"][:n]
    assert hdr["accepted"] == int(float(torch.dot(yv.double(), sv.double())) > 1e-10)
    assert hdr["n_iter"] == hdr0["n_iter"] + 1 and hdr["count"] == 100
    Ss = [hist[k * npad:k * npad + n] for k in hdr["order"]]
    Ys = [hist[(m1 + k) * npad:(m1 + k) * npad + n] for k in hdr["order"]]
    if hdr["accepted"]:  # the new pair is the last in order and equals (s_prev, g - prev_g)
        assert torch.equal(Ss[-1], sv)
        assert float((Ys[-1] - yv).abs().max()) == 0.0
        assert hdr["order"][:-1] == hdr0["order"][1:]
    t = hdr["t"]
    td_ours = hist[hdr["cand"] * npad:hdr["cand"] * npad + n].double()
    assert torch.equal((x0.view(-1) + td_ours.float()), eng.x.view(-1)) or \
        float((x0.view(-1) + td_ours.float() - eng.x.view(-1)).abs().max()) == 0.0
    Hd = float(torch.dot(Ys[-1].double(), Ss[-1].double()) / torch.dot(Ys[-1].double(),
                                                                        Ys[-1].double()))
    d64 = _two_loop([v.double() for v in Ss], [v.double() for v in Ys], g.double(), Hd)
    d32 = _two_loop(Ss, Ys, g, torch.tensor(hdr["H_diag"], device=dev))
    rel = lambda a, c3: float((a - c3).norm() / c3.norm())  # noqa: E731
    e_ours, e_t32 = rel(td_ours, t * d64), rel(t * d32.double(), t * d64)
    print(f"512^2 history 100 (n_iter {hdr['n_iter']}): ours vs fp64 {e_ours:.2e}, "
          f"torch-fp32 two-loop vs fp64 {e_t32:.2e}, H_diag {hdr['H_diag']:.4g} vs {Hd:.4g}")
    assert e_ours <= max(3 * e_t32, 1e-6), (e_ours, e_t32)
