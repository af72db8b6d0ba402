"""Parity of the HIP path (through the reference-style API and the C-ABI) with the
golden vectors generated from the real reference (oracle/gen_golden.py).

Tolerances (BASELINE.json north star: Gram and loss tensors within 1e-4 relative
fp32; integer/index results bit-exact):
  * losses, Gram matrices, outputs: relative error <= 1e-4
  * gradients: relative norm error <= 1e-4 (whole tensor)
  * Adam-updated images: relative error of the update (x - x0) <= 1e-3, because the
    first Adam step is ~lr*sign(g) and sign flips of |g|~1e-12 entries are
    reassociation noise (SURVEY.md §7 "Adam step-1 sign sensitivity").
"""
import os

import numpy as np
import pytest
import torch

import forced_ref as R
from conftest import GOLDEN
from styletransfer_amd import network, ops
from styletransfer_amd import vgg as V
from styletransfer_amd import weights as W

pytestmark = pytest.mark.gpu


def g(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


def rel(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def proj(a, seed=99):
    a = np.asarray(a, np.float64).ravel()
    r = W.hash_normal(seed, a.size * 8).astype(np.float64).reshape(8, a.size)
    return r @ a


def update_close(x, x0, ref, lr=1e-3, max_flip_frac=1e-3, tol=1e-3):
    """Adam-updated image vs reference: the update (x - x0) may differ by a sign
    flip (~2*lr per step) on pixels whose gradient is ~0; those must be rare, the
    rest must agree to `tol` relative."""
    du = np.asarray(x, np.float64) - x0
    dr = np.asarray(ref, np.float64) - x0
    flip = np.abs(du - dr) > 0.5 * lr
    assert flip.mean() <= max_flip_frac, flip.mean()
    keep = ~flip
    assert rel(du[keep], dr[keep]) < tol


def test_gram_style_golden(dev):
    d = g("gram")
    for i in range(int(d["n"])):
        x, t = T(d[f"x{i}"], dev), T(d[f"t{i}"], dev)
        assert rel(ops.gram(x), d[f"G{i}"]) < 1e-4
        sl = network.StyleLoss(t)
        assert rel(sl.target, d[f"T{i}"]) < 1e-4
        xr = x.clone().requires_grad_()
        sl(xr)
        sl.loss.backward()
        assert rel(sl.loss, d[f"loss{i}"]) < 1e-4
        assert rel(xr.grad, d[f"dx{i}"]) < 1e-4
        # gram_matrix API (differentiable)
        xg = x.clone().requires_grad_()
        G = sl.gram_matrix(xg)
        G.sum().backward()
        xt = x.detach().cpu().double().requires_grad_()
        f = xt.view(xt.shape[0], xt.shape[1], -1)
        (torch.bmm(f, f.transpose(1, 2)) / f[0].numel()).sum().backward()
        assert rel(xg.grad, xt.grad) < 1e-4


def test_content_feature_golden(dev):
    d = g("content_feature")
    x, t = T(d["x"], dev), T(d["target"], dev)
    for name, cls in (("content", network.ContentLoss),
                      ("feature", network.FeatureReconstructionLoss)):
        m = cls(t)
        xr = x.clone().requires_grad_()
        m(xr)
        m.loss.backward()
        assert rel(m.loss, d[f"{name}_loss"]) < 1e-4
        assert rel(xr.grad, d[f"{name}_dx"]) < 1e-4


def test_tv_golden(dev):
    d = g("tv")
    y = T(d["y"], dev).requires_grad_()
    net = network.ImageTransformNet(y.detach()[:1], 2)
    loss = net.get_total_variation_regularization_loss(y)
    loss.backward()
    assert rel(loss, d["loss"]) < 1e-5
    assert rel(y.grad, d["dy"]) < 1e-5


@pytest.fixture(scope="module")
def stylenet(dev):
    d = g("stylenet")
    net = network.StyleNetwork(T(d["style"], dev), T(d["content"], dev))
    return d, net


def test_stylenet_structure(stylenet):
    d, net = stylenet
    assert [len(list(p.children())) for p in net.net_pieces] == list(d["piece_layer_counts"])
    assert [i for _, i in net.style_losses] == list(d["style_piece_idx"])
    assert [i for _, i in net.content_losses] == list(d["content_piece_idx"])
    assert [i for _, i in net.feature_losses] == list(d["feature_piece_idx"])
    names = [n for p in net.net_pieces for n, _ in p.named_children()]
    assert names[:5] == ["Conv2d_1", "ReLU_1", "Conv2d_2", "ReLU_2", "MaxPool2d_2"]
    for (l, _), pr in zip(net.style_losses, d["ref_style_targets_proj"]):
        assert rel(proj(l.target.cpu().numpy()), pr) < 1e-4


def test_stylenet_forward_backward(stylenet, dev):
    d, net = stylenet
    x = T(d["x0"], dev).requires_grad_()
    content = T(d["content"], dev)
    net(x, content)
    s = net.get_total_current_style_loss(100_000)
    c = net.get_total_current_content_loss(1)
    f = net.get_total_current_feature_loss(1)
    (s + c).backward()
    assert rel([float(l.loss) for l, _ in net.style_losses], d["ref_style_losses"]) < 1e-4
    assert rel(net.content_losses[0][0].loss, d["ref_content_loss"]) < 1e-4
    assert rel(net.feature_losses[0][0].loss, d["ref_feature_loss"]) < 1e-4
    assert rel(s, d["ref_total_style"]) < 1e-4
    assert rel(c, d["ref_total_content"]) < 1e-4
    assert rel(f, d["ref_total_feature"]) < 1e-4
    assert rel(x.grad, d["dx"]) < 1e-4


def test_stylenet_generic_path_matches(stylenet, dev):
    """Non-fused per-piece autograd path (any tap layout) == fused engine."""
    d, net = stylenet
    x = T(d["x0"], dev).requires_grad_()
    content = T(d["content"], dev)
    net._forward_generic(x, content, None)
    (net.get_total_current_style_loss(100_000) + net.get_total_current_content_loss()).backward()
    assert rel([float(l.loss) for l, _ in net.style_losses], d["ref_style_losses"]) < 1e-4
    assert rel(net.feature_losses[0][0].loss, d["ref_feature_loss"]) < 1e-4
    assert rel(x.grad, d["dx"]) < 1e-4


def test_gatys_adam_api_and_engine(stylenet, dev):
    d, net = stylenet
    content = T(d["content"], dev)
    c0 = d["content"].astype(np.float64)
    # reference-API loop with get_content_optimizer (HIP Adam)
    x = content.clone()
    opt = net.get_content_optimizer(x)
    losses = []
    for it in range(3):
        opt.zero_grad()
        net(x, content)
        tot = net.get_total_current_style_loss(100_000) + net.get_total_current_content_loss(1)
        tot.backward()
        opt.step()
        losses.append(float(tot))
        if it == 0:
            update_close(x.detach().cpu().numpy(), c0, d["ref_adam1"])
    assert rel(losses, d["ref_adam_losses"]) < 1e-4
    update_close(x.detach().cpu().numpy(), c0, d["ref_adam3"])
    # fused engine (graph-captured iteration)
    eng = V.GatysEngine(net.features(), None, content,
                        targets=[l.target for l, _ in net.style_losses])
    elosses = []
    for it in range(3):
        elosses.append(float(eng.step()))
    assert rel(elosses, d["ref_adam_losses"]) < 1e-4
    update_close(eng.x.cpu().numpy(), c0, d["ref_adam3"])
    eng2 = V.GatysEngine(net.features(), None, content,
                         targets=[l.target for l, _ in net.style_losses])
    eng2.run(3, graph=True)
    update_close(eng2.x.cpu().numpy(), c0, d["ref_adam3"])
    assert rel(eng2.total, d["ref_adam_losses"][2]) < 1e-4


def test_gatys_config2_512_engine_golden(dev):
    """BASELINE config 2 at full size: GatysEngine at 512^2 (the bench's rank-0 inputs and
    its exact launches: the fused Gram partials of 1024 tiles, 256x2 grids, the data
    gradients of 1024 blocks; one eager iteration, then hipGraph replays) against the
    reference's own StyleNetwork (gatys512.npz, 3 Adam iterations).  Losses within 1e-4;
    the first update ~lr*sign(g) agrees in sign except on a negligible fraction of
    pixels (|g| ~ rounding).  At this size the fp32 reference's image gradient is itself
    ~1.1e-3 from the fp64 run's (elements within rounding of a ReLU / argmax kink), so
    gradients are compared three-way: HIP's distance from the fp64 run <= 2.5x (4x after
    two steps) the fp32 reference's (32 projections + norm); the image after 3 steps
    pixel by pixel, its sign-flipped pixels bounded separately (flip-aware)."""
    d = g("gatys512")
    H = int(d["size"])
    style = T(W.synthetic_image(int(d["style_seed"]), (1, 3, H, H)), dev)
    content = T(W.synthetic_image(int(d["content_seed"]), (1, 3, H, H)), dev)
    eng = V.GatysEngine(V.VGGFeatures(V.load_vgg19_weights(), dev), style, content)
    eng.capture(warmup=1)                       # iteration 1 (eager), then capture
    torch.cuda.synchronize()
    tot = [float(eng.total)]
    per = eng.losses().detach().cpu().numpy().copy()
    dx1 = eng.grad.detach().cpu().numpy().astype(np.float64)
    x1 = eng.x.detach().cpu().numpy().astype(np.float64)
    for _ in range(2):                          # iterations 2, 3: graph replays
        eng.step()
        tot.append(float(eng.total))
    dx3 = eng.grad.detach().cpu().numpy().astype(np.float64)
    x3 = eng.x.detach().cpu().numpy().astype(np.float64)
    c0 = W.synthetic_image(int(d["content_seed"]), (1, 3, H, H)).astype(np.float64)
    nproj = lambda a: np.concatenate([[np.linalg.norm(a)], proj32(a)])  # noqa: E731
    assert rel(tot, d["losses"]) < 1e-4, (tot, d["losses"])
    # style x5 (unweighted), content; the feature loss is computed but not optimised
    assert rel(per, d["losses_it1"]) < 1e-4, (per, d["losses_it1"])
    errs = {}
    # iteration 1's gradient: 2.5x; after two Adam steps (~lr*sign(g) per pixel, so a pixel
    # whose |g| is at rounding level steps either way in any fp32 run) the trajectories of
    # fp32 runs fan out from the fp64 one by their own sign flips: the gradient 4x.  The
    # loss trajectory above is held to 1e-4.
    for k, v, f in (("dx1", dx1, 2.5), ("dx3", dx3, 4.0)):
        e, r = rel(nproj(v), d[f"{k}_proj_64"]), rel(d[f"{k}_proj"], d[f"{k}_proj_64"])
        errs[k] = (e, r)
        assert e <= max(f * r, 1e-5), (k, e, r)
    # the image after 3 steps, flip-aware against the fp64 run's full update: pixels that
    # stepped the other way (|du - du64| > lr / 2: a whole +-lr step where |g| is at rounding
    # level) are counted and bounded on their own; every other pixel's update is held to
    # 2.5x the fp32 reference's own error on its non-flipped pixels (gatys512.npz)
    lr = 1e-3
    u, u64 = x3 - c0, d["upd3_64"].astype(np.float64)
    flip = np.abs(u - u64) > 0.5 * lr
    keep_rel = rel(u[~flip], u64[~flip])
    ref_flip, ref_keep = float(d["upd3_ref_flip_frac"]), float(d["upd3_ref_keep_rel"])
    errs["upd3"] = dict(flip_frac=float(flip.mean()), ref_flip_frac=ref_flip,
                        keep_rel=keep_rel, ref_keep_rel=ref_keep)
    assert flip.mean() <= 1e-4, errs["upd3"]
    assert keep_rel <= 2.5 * ref_keep, errs["upd3"]
    s_hip = (x1 - c0).ravel() > 0
    s_ref = np.unpackbits(d["upd1_sign"])[:s_hip.size].astype(bool)
    flips = float(np.mean(s_hip != s_ref))
    assert flips <= 1e-3, flips
    print(f"gatys512: losses {tot}; vs fp64 (hip, fp32 reference): {errs}; "
          f"step-1 sign flips {flips:.2e}")


@pytest.fixture(scope="module")
def itn_case(dev):
    d = g("itn")
    net = network.ImageTransformNet(T(d["style"], dev), batch_size=2)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
    return d, net


def test_itn_state_dict_keys(itn_case):
    d, net = itn_case
    keys = list(net.state_dict().keys())
    assert len(keys) == int(d["n_params"]) == 62
    assert keys == [k for k, _ in W.itn_synthetic(4321)]


def test_itn_forward_backward_golden(itn_case, dev, monkeypatch):
    d, net = itn_case
    batch = T(d["batch"], dev)
    ln = network.StyleNetwork(T(d["style"], dev),
                              T(W.synthetic_image(23, (1, 3, 64, 64)), dev))
    net.zero_grad()
    with R.HipBranchSpy(net, V, monkeypatch) as spy:
        y = net(batch)
        assert rel(y, d["y"]) < 1e-4
        ln(y, content_image=batch)
    hip_branches = (spy.itn, spy.vgg)
    sl = ln.get_total_current_style_loss(100_000)
    cl = ln.get_total_current_content_loss(1)
    tv = net.get_total_variation_regularization_loss(y)
    total = sl + cl + tv
    total.backward()
    assert rel(sl, d["style_loss"]) < 1e-4
    assert rel(cl, d["content_loss"]) < 1e-4
    assert rel(tv, d["tv_loss"]) < 1e-4
    assert rel(total, d["total"]) < 1e-4
    # parameter gradients vs fp64 truth (itn_fp64.npz: the pinned oracle in float64 on
    # the same inputs).  A ReLU / argmax branch decided differently from fp64 (an
    # element within rounding of a kink) moves every parameter gradient upstream of it;
    # which parameters those are is read from the branch records themselves (HIP's, and
    # an fp32 oracle run's standing in for the fp32 reference), never inferred from the
    # size of an error.  Downstream of every flip: HIP within 2.5x the fp32 reference's
    # error.  All parameters, flips included, are held to fp32-class error against fp64
    # with the branches forced in tests/test_itn_masks_gpu.py.
    f64 = g("itn_fp64")
    norms = f64["grad64_proj"][:, 0]
    params = list(net.parameters())
    flipped = itn_flipped_params(hip_branches)
    errs = []
    for i in range(len(params)):
        gp = params[i].grad.detach().cpu().numpy()
        if norms[i] < 1e-7 * norms.max():
            # conv bias followed by InstanceNorm: exactly 0 in exact arithmetic (fp64
            # |g| ~ 1e-14; fp32 rounding noise ~1e-5 in the reference)
            assert np.linalg.norm(gp) < 1e-6 * norms.max(), i
            continue
        e64 = rel(proj32(gp), f64["grad64_proj"][i, 1:])
        r32 = float(f64["ref32_err"][i])
        if i in flipped:
            # upstream of a flip: a loose bound only (the forced-branch tests hold these
            # parameters to fp32-class error)
            assert e64 <= max(2.5 * r32, 3e-2), (i, e64, r32)
            continue
        errs.append((e64, r32, i))
        assert e64 <= max(2.5 * r32, 1e-5), (i, e64, r32)
    # At this size every parameter is flip-affected: the fp32 reference's own run decides
    # one loss-network branch differently from fp64 (pinned on CPU by
    # tests/test_forced_ref_pin.py::test_golden_flip_sites), and a VGG flip moves every
    # ITN gradient.  The tight fp32-class check of all 62 gradients is therefore the
    # forced-branch one (test_itn_masks_gpu.py), whose fp64 ground truth (forced_ref.py)
    # is itself pinned to itn_fp64.npz / itn.npz by test_forced_ref_pin.py.
    print("ITN grad error vs fp64 downstream of every flip (hip, fp32-ref, param):",
          sorted(errs)[-3:], "flip-affected params:", len(flipped),
          "HIP flips (ITN, VGG) vs fp64:", itn_flip_counts(hip_branches))

    with torch.no_grad():
        assert rel(net(batch[:1]), d["y_single"]) < 1e-4


def proj32(a, seed=77):
    a = np.asarray(a, np.float64).ravel()
    r = W.hash_normal(seed, a.size * 32).astype(np.float64).reshape(32, a.size)
    return r @ a


def itn_flipped_params(hip_branches):
    """Parameters (indices) whose gradient a branch flip can move: upstream of any
    element where HIP's decision or the fp32 reference's (an fp32 oracle run on the
    golden inputs) differs from the fp64 run's."""
    d = g("itn")
    sd = W.itn_synthetic(4321)
    keys = [k for k, _ in sd]
    vgg = W.vgg19_synthetic(1234, 5)
    n64 = R.natural_branches(sd, vgg, d["batch"], torch.float64)
    n32 = R.natural_branches(sd, vgg, d["batch"], torch.float32)
    return (R.flip_upstream(keys, hip_branches[0], n64[0], hip_branches[1], n64[1])
            | R.flip_upstream(keys, n32[0], n64[0], n32[1], n64[1]))


def itn_flip_counts(hip_branches):
    d = g("itn")
    n64 = R.natural_branches(W.itn_synthetic(4321), W.vgg19_synthetic(1234, 5), d["batch"],
                             torch.float64)
    return R.count_flips(hip_branches[0], n64[0]), R.count_flips(hip_branches[1], n64[1])


def test_itn_adam_step_golden(itn_case, dev, monkeypatch):
    """itn.npz["adam1_proj"]: the reference's ImageTransformNet.get_optimizer() Adam
    step (stransfer/network.py:643-649) after the golden forward/backward."""
    d, _ = itn_case
    net = network.ImageTransformNet(T(d["style"], dev), batch_size=2)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
    batch = T(d["batch"], dev)
    ln = network.StyleNetwork(T(d["style"], dev), T(W.synthetic_image(23, (1, 3, 64, 64)), dev))
    opt = net.get_optimizer()
    opt.zero_grad()
    with R.HipBranchSpy(net, V, monkeypatch) as spy:
        y = net(batch)
        ln(y, content_image=batch)
    (ln.get_total_current_style_loss(100_000) + ln.get_total_current_content_loss(1)
     + net.get_total_variation_regularization_loss(y)).backward()
    gnorm = [float(p.grad.norm()) for p in net.parameters()]
    grads = [p.grad.detach().clone() for p in net.parameters()]
    flipped = itn_flipped_params((spy.itn, spy.vgg))
    p0 = [p.detach().clone() for p in net.parameters()]
    opt.step()
    errs = []
    for i, p in enumerate(net.parameters()):
        assert float((p.detach() - p0[i]).abs().max()) <= 1.001e-3  # |step 1| <= lr
        if gnorm[i] < 1e-6 * max(gnorm):
            # zero-gradient biases: step 1 is lr*sign(rounding noise) on both sides
            continue
        # Adam step 1 moves every element by ~lr*sign(g).  Downstream of the backward's
        # ReLU-boundary flip the gradients match the reference to ~1e-3 and so do the
        # steps; upstream, elements whose gradient sign the flip changes step the other
        # way (2e-3 each; measured <= 9e-3 of the parameter norm).  A missing or
        # doubled step or a wrong lr moves a parameter by ~1e-2 of its norm.
        e = rel(proj(p.detach().cpu().numpy()), d["adam1_proj"][i])
        errs.append((e, i))
        assert e < (2e-2 if i in flipped else 2e-3), (i, e)
    print("ITN Adam step vs reference (rel err, param):", sorted(errs)[-3:],
          "flip-affected params:", len(flipped))
    # the optimizer itself, flips aside: torch.optim.Adam on the same gradients
    for p0i, gi, p in zip(p0, grads, net.parameters()):
        q = p0i.clone().requires_grad_()
        q.grad = gi.clone()
        torch.optim.Adam([q]).step()
        assert float((q.detach() - p.detach()).abs().max()) <= 1e-6 * max(
            1.0, float(p0i.abs().max())), "Adam step 1 vs torch.optim.Adam"


def test_fast_st_trainer_matches_api(itn_case, dev):
    """FastStTrainer (fused loss net, flat params, flat Adam) == API closure + Adam."""
    from styletransfer_amd.train import FastStTrainer
    d, _ = itn_case
    style = T(d["style"], dev)
    batch = T(d["batch"], dev)
    sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)}
    a = network.ImageTransformNet(style, 2)
    a.load_state_dict(sd)
    b = network.ImageTransformNet(style, 2)
    b.load_state_dict(sd)
    ln = network.StyleNetwork(style, torch.rand([1, 3, 64, 64]))
    opt = a.get_optimizer()
    opt.zero_grad()
    y = a(batch)
    ln(y, content_image=batch)
    total = (ln.get_total_current_style_loss(100_000) + ln.get_total_current_content_loss(1)
             + a.get_total_variation_regularization_loss(y))
    total.backward()
    ga = [p.grad.clone() for p in a.parameters()]
    opt.step()
    p0 = [q.detach().clone() for q in b.parameters()]
    tr = FastStTrainer(b, style)
    tb = tr.step(batch)
    assert rel(tb, total) < 1e-5
    gmax = max(float(g.norm()) for g in ga)
    for p, q, gq, q0 in zip(a.parameters(), b.parameters(), ga, p0):
        if float(gq.norm()) < 1e-6 * gmax:
            # conv biases feeding InstanceNorm: the exact gradient is 0 and both sides
            # hold fp32 rounding noise (see test_itn_forward_backward_params)
            assert float(q.grad.norm()) < 1e-6 * gmax
            continue
        assert rel(q.grad, gq) < 1e-5
        # Adam step 1 moves each element by ~lr*sign(g): elements whose gradient is
        # at rounding-noise level (|g| < 1e-4 max|g|) may step either way; the rest
        # must take the same step
        da, db = (p.detach() - q0), (q.detach() - q0)
        big = gq.abs() >= 1e-4 * gq.abs().max()
        assert rel(db[big], da[big]) < 1e-4
        assert float((db - da).abs().max()) <= 2.0001e-3


def test_determinism(itn_case, dev):
    """Bit-reproducible runs: no float atomics, fixed reduction orders (the split
    convs' per-tensor scales come from atomicMax, which is order-independent)."""
    from styletransfer_amd.train import FastStTrainer
    d, _ = itn_case
    style = T(d["style"], dev)
    batch = T(d["batch"], dev)
    sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)}
    outs = []
    for _ in range(2):
        net = network.ImageTransformNet(style, 2)
        net.load_state_dict(sd)
        tr = FastStTrainer(net, style)
        tr.step(batch)
        tr.step(batch)
        outs.append(tr.flat.detach().clone())
    assert torch.equal(outs[0], outs[1])
    xs = []
    feat = V.VGGFeatures(V.load_vgg19_weights(), dev)
    s = torch.from_numpy(W.synthetic_image(5, (1, 3, 96, 96))).to(dev)
    c = torch.from_numpy(W.synthetic_image(6, (1, 3, 96, 96))).to(dev)
    for _ in range(2):
        eng = V.GatysEngine(feat, s, c)
        for _ in range(3):
            eng.step()
        xs.append(eng.x.clone())
    assert torch.equal(xs[0], xs[1])


def test_fast_st_graph_replay_equals_eager(itn_case, dev):
    """FastStTrainer.capture: hipGraph replays of the training step (forward/backward
    graph + Adam graph) train bit-identically to eager steps, on fresh batches copied
    into the static input."""
    from styletransfer_amd.train import FastStTrainer
    d, _ = itn_case
    style = T(d["style"], dev)
    batch = T(d["batch"], dev)
    batches = [batch, batch.flip(3).contiguous(), batch.flip(2).contiguous()]
    sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)}
    na, nb = network.ImageTransformNet(style, 2), network.ImageTransformNet(style, 2)
    na.load_state_dict(sd)
    nb.load_state_dict(sd)
    ta, tb = FastStTrainer(na, style), FastStTrainer(nb, style)
    ta.step(batch)  # = tb's capture warm-up step
    la = [ta.step(x) for x in batches]
    replay, static, loss = tb.capture(batch, warmup=1)
    lb = []
    for x in batches:
        static.copy_(x)
        replay()
        lb.append(loss.clone())
    torch.cuda.synchronize()
    assert torch.equal(ta.flat, tb.flat)
    for u, v in zip(la, lb):
        assert torch.equal(u, v)


def test_dp_gradient_equivalence(itn_case, dev):
    """W shards with the (mean/W + sum) scaling, summed, == the full-batch gradient."""
    from styletransfer_amd.train import FastStTrainer
    d, _ = itn_case
    style = T(d["style"], dev)
    batch = torch.cat([T(d["batch"], dev)] * 2)  # B=4
    sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)}

    def grads(world, shard):
        net = network.ImageTransformNet(style, 2)
        net.load_state_dict(sd)
        tr = FastStTrainer(net, style, world_size=1)
        tr.world = world  # scaling only; the all-reduce is summed by hand below
        tr.flat_grad.zero_()
        y = net(shard)
        tr._total(shard, y).backward()
        return tr.flat_grad.clone()

    full = grads(1, batch)
    summed = grads(2, batch[:2].contiguous()) + grads(2, batch[2:].contiguous())
    assert rel(summed, full) < 1e-5


def test_images_golden(dev):
    from styletransfer_amd import img_utils
    d = g("images")
    root = os.path.dirname(GOLDEN)
    data = os.path.join(os.path.dirname(root), "data")
    x = img_utils.image_loader(os.path.join(data, "dancing.jpg"))
    assert x.is_cuda
    assert torch.equal(x.cpu(), torch.from_numpy(d["dancing_256"]))
