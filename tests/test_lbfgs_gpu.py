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
    assert err.max() < 5e-2, err.max()
    # every graph evaluation is one torch makes (the last step's closing evaluation is the
    # next step's opening one), but for stops on g.d (none expected here)
    assert eng.closure_runs <= eng.func_evals + 1, (eng.closure_runs, eng.func_evals)
    pairs, n_iter = eng.history()
    assert n_iter == opt.state[x]["n_iter"] and 0 < pairs <= 100
