"""The CPU oracle (oracle/reference_cpu.py) against the golden vectors produced by
the real reference (oracle/gen_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import reference_cpu as O
from styletransfer_amd import weights as W


def g(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


def proj(a, seed=99):
    a = np.asarray(a, np.float64).ravel()
    r = W.hash_normal(seed, a.size * 8).astype(np.float64).reshape(8, a.size)
    return r @ a


def test_weight_generator_pinned():
    d = g("weights_pin")
    for (w, _), p in zip(W.vgg19_synthetic(1234, 5), d["vgg_proj"]):
        assert rel(proj(w), p) < 1e-12
    for (_, v), p in zip(W.itn_synthetic(4321), d["itn_proj"]):
        assert rel(proj(v), p) < 1e-12


def test_gram_style():
    d = g("gram")
    for i in range(int(d["n"])):
        x = torch.from_numpy(d[f"x{i}"]).requires_grad_()
        sl = O.StyleLoss(torch.from_numpy(d[f"t{i}"]))
        sl(x)
        sl.loss.backward()
        assert rel(O.gram_matrix(x.detach()), d[f"G{i}"]) < 1e-6
        assert rel(sl.loss.detach(), d[f"loss{i}"]) < 1e-6
        assert rel(x.grad, d[f"dx{i}"]) < 1e-6


def test_content_feature():
    d = g("content_feature")
    for name, cls in (("content", O.ContentLoss), ("feature", O.FeatureReconstructionLoss)):
        x = torch.from_numpy(d["x"]).requires_grad_()
        m = cls(torch.from_numpy(d["target"]))
        m(x)
        m.loss.backward()
        assert rel(m.loss.detach(), d[f"{name}_loss"]) < 1e-6
        assert rel(x.grad, d[f"{name}_dx"]) < 1e-6


def test_tv():
    d = g("tv")
    y = torch.from_numpy(d["y"]).requires_grad_()
    loss = O.total_variation(y)
    loss.backward()
    assert rel(loss.detach(), d["loss"]) < 1e-6
    assert rel(y.grad, d["dy"]) < 1e-6


def test_stylenet_and_adam():
    d = g("stylenet")
    net = O.StyleNetwork(torch.from_numpy(d["style"]), torch.from_numpy(d["content"]))
    assert [len(list(p.children())) for p in net.net_pieces] == list(d["piece_layer_counts"])
    x = torch.from_numpy(d["x0"]).requires_grad_()
    content = torch.from_numpy(d["content"])
    net(x, content)
    (net.get_total_current_style_loss(100_000) + net.get_total_current_content_loss()).backward()
    assert rel([float(l.loss) for l, _ in net.style_losses], d["ref_style_losses"]) < 2e-5
    assert rel(x.grad, d["dx"]) < 2e-5
    x = content.clone()
    opt = net.get_content_optimizer(x)
    losses = [float(O.gatys_adam_iter(net, x, content, opt)) for _ in range(3)]
    assert rel(losses, d["ref_adam_losses"]) < 1e-5
    assert rel(x.detach(), d["ref_adam3"]) < 1e-5


@pytest.mark.slow
def test_itn():
    d = g("itn")
    net = O.image_transform_net(4321)
    batch = torch.from_numpy(d["batch"])
    ln = O.StyleNetwork(torch.from_numpy(d["style"]),
                        torch.from_numpy(W.synthetic_image(23, (1, 3, 64, 64))))
    total, y = O.fast_st_closure(net, ln, batch)
    assert rel(y.detach(), d["y"]) < 1e-5
    assert rel(float(total), d["total"]) < 1e-5
    for i, p in enumerate(net.parameters()):
        ref = d["grad_proj"][i]
        assert rel(proj(p.grad.numpy()), ref[1:]) < 1e-3


def test_adam_restatement_matches_torch():
    p = torch.randn(100, generator=torch.Generator().manual_seed(0))
    g_ = torch.randn(100, generator=torch.Generator().manual_seed(1))
    pr = p.clone().requires_grad_()
    opt = torch.optim.Adam([pr])
    m, v, q = torch.zeros(100), torch.zeros(100), p.clone()
    for step in range(1, 4):
        pr.grad = g_ * step
        opt.step()
        O.adam_reference_step(q, g_ * step, m, v, step)
    assert rel(q, pr.detach()) < 1e-6
