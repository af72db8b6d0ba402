"""End-to-end workflows against fixtures of the real reference (oracle/gen_golden.py)
and against the pinned oracle, through the reference's API and CLI:

  * `StyleNetwork.train_gatys` (L-BFGS, stransfer/network.py:411-458) vs the
    reference's own train_gatys run (lbfgs.npz);
  * BASELINE config 1: `python -m stransfer gatys_st data/dancing.jpg
    data/styles/picasso.jpg -s 50 --optimizer adam` vs the reference's Adam loop on
    the same images (config1.npz);
  * `ImageTransformNet.static_train` (stransfer/network.py:651-770) vs the oracle's
    closure + torch.optim.Adam on the same batches;
  * `fast_st train --synthetic` -> checkpoint -> `fast_st convert-image`
    (stransfer/clis/fast_st.py:26-63, network.py:798-832) vs the oracle's forward
    of the written checkpoint.
"""
import logging
import os
import shutil

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import GOLDEN, REPO
from styletransfer_amd import constants, network
from styletransfer_amd import weights as W

pytestmark = pytest.mark.gpu


def g(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


def rel(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


def proj32(a, seed=77):
    a = np.asarray(a, np.float64).ravel()
    r = W.hash_normal(seed, a.size * 32).astype(np.float64).reshape(32, a.size)
    return r @ a


class LossTrace(logging.Handler):
    """The closure losses train_gatys logs at DEBUG ("Loss: %s")."""

    def __init__(self):
        super().__init__()
        self.vals = []

    def emit(self, rec):
        if isinstance(rec.msg, str) and rec.msg.startswith("Loss:") and rec.args:
            self.vals.append(float(rec.args[0]))

    def __enter__(self):
        lg = logging.getLogger("StyleTransfer")
        self._saved = lg.level
        lg.setLevel(logging.DEBUG)
        lg.addHandler(self)
        return self

    def __exit__(self, *a):
        lg = logging.getLogger("StyleTransfer")
        lg.removeHandler(self)
        lg.setLevel(self._saved)


def test_train_gatys_lbfgs_reference(dev):
    """The reference's own train_gatys (lbfgs.npz): 2 outer L-BFGS steps at 64^2, 40
    closure evaluations, loss 9288 -> 641.  L-BFGS amplifies rounding chaotically:
    the fp32 reference itself drifts from its fp64 evaluation by up to ~5e-2 in the
    later losses and 2.8e-2 in the image.  So: the first evaluations (before the
    amplification) match the reference to 1e-5, the evaluation count matches, and
    against the fp64 run the HIP trajectory is no further than 2x the fp32
    reference's distance, per evaluation and for the image."""
    d = g("lbfgs")
    s, c = torch.from_numpy(d["style"]).to(dev), torch.from_numpy(d["content"]).to(dev)
    net = network.StyleNetwork(s, c)
    with LossTrace() as tr:
        out = net.train_gatys(s, c, steps=int(d["steps"]), style_weight=float(d["style_weight"]))
    ref, r64 = d["losses"], d["losses64"]
    got = np.array(tr.vals)
    assert len(got) == len(ref), (len(got), len(ref))
    e_ref = np.abs(got - ref) / np.abs(ref)
    assert e_ref[:4].max() < 1e-5, e_ref[:4]
    e64 = np.abs(got - r64) / np.abs(r64)
    e32 = np.abs(ref - r64) / np.abs(r64)
    i64, i32 = rel(out, d["image64"]), rel(d["image"], d["image64"])
    print(f"L-BFGS: vs reference max {e_ref.max():.2e}; vs fp64 max {e64.max():.2e} "
          f"(fp32 reference {e32.max():.2e}); image vs fp64 {i64:.2e} (reference {i32:.2e})")
    assert e64.max() <= 2.0 * e32.max()
    assert i64 <= 2.0 * i32


@pytest.fixture
def project_root(tmp_path, monkeypatch):
    """A scratch PROJECT_ROOT with the reference's data layout (data/dancing.jpg,
    data/styles/picasso.jpg) and the CWD there (checkpoints are CWD-relative)."""
    for rel_path in ("data/dancing.jpg", "data/styles/picasso.jpg"):
        dst = tmp_path / rel_path
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(REPO, rel_path), dst)
    monkeypatch.setattr(constants, "PROJECT_ROOT_PATH", str(tmp_path))
    monkeypatch.chdir(tmp_path)
    return tmp_path


def test_config1_gatys_cli_adam(dev, project_root):
    """BASELINE config 1 through the CLI (Adam, 50 iterations at 256^2 on the
    reference's images): the saved PNG vs the reference's `imshow` bytes, and the
    per-iteration losses of the same loop (GatysEngine) vs the reference's."""
    from click.testing import CliRunner
    from styletransfer_amd import img_utils
    from styletransfer_amd import vgg as V
    from styletransfer_amd.clis import cli
    d = g("config1")
    r = CliRunner().invoke(cli, ["gatys_st", "data/dancing.jpg", "data/styles/picasso.jpg",
                                 "-s", "50", "--optimizer", "adam", "-n", "cfg1.png"])
    assert r.exit_code == 0, r.output + repr(r.exception)
    got = np.asarray(Image.open(project_root / "results" / "cfg1.png")).astype(np.int32)
    want = d["image_u8"].astype(np.int32)
    diff = np.abs(got - want)
    print(f"config1 PNG: max |diff| {diff.max()}, mean {diff.mean():.4f}, "
          f"> 1: {(diff > 1).mean():.2e}")
    # Adam steps are ~lr*sign(g): pixels whose gradient is at rounding level may step
    # the other way; in bytes that is at most a couple of units on rare pixels
    assert diff.mean() < 0.05 and (diff > 2).mean() < 1e-3
    content = img_utils.image_loader(str(project_root / "data/dancing.jpg"))
    style = img_utils.image_loader(str(project_root / "data/styles/picasso.jpg"))
    net = network.StyleNetwork(style, content)
    eng = V.GatysEngine(net.features(), None, content,
                        targets=[l.target for l, _ in net.style_losses])
    losses = [float(eng.step()) for _ in range(int(d["iters"]))]
    lerr = np.abs(np.array(losses) - d["losses"]) / d["losses"]
    print(f"config1 losses: max rel err {lerr.max():.2e}")
    assert lerr.max() < 1e-4
    assert rel(proj32(eng.x.cpu().numpy()), d["image_proj"][1:]) < 1e-3


def test_static_train_matches_oracle(dev, project_root):
    """static_train (graph-replayed steps, evaluation / static_test / image logging at
    iteration 0 interleaved, checkpoint with the reference's name and keys) trains
    bit-identically to plain FastStTrainer.step() calls on the same 4 synthetic
    batches, and matches the oracle's closure + torch.optim.Adam within the fp32
    sensitivity of the computation: against the oracle evaluated in fp64, the HIP
    run's update error is at most 5x the fp32 oracle's.  (4 Adam steps amplify
    gradient rounding: each step is ~lr*sign(g), so tiny-gradient elements flip; the
    fp32 oracle is itself 3.6e-2 from fp64 here.)"""
    from oracle import reference_cpu as O
    from styletransfer_amd import dataset
    from styletransfer_amd.train import FastStTrainer
    H, B = 64, 4
    style = torch.from_numpy(W.synthetic_image(61, (1, 3, H, H)))
    sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)}
    net = network.ImageTransformNet(style.to(dev), batch_size=B)
    net.load_state_dict(sd)
    loaders = dataset.get_synthetic_loader(B, n_train=16, n_test=4, size=H, seed=5)
    net.static_train(style_name="synth", epochs=1, loaders=loaders)
    ck = project_root / "data" / "models" / "fast_st_synth_epoch0.pth"
    assert ck.is_file()
    saved = torch.load(ck, weights_only=True)
    assert list(saved) == list(sd)
    ph = torch.cat([saved[k].reshape(-1).cpu() for k in sd]).double()
    # the same steps through the trainer directly (eager): bit-identical
    net2 = network.ImageTransformNet(style.to(dev), batch_size=B)
    net2.load_state_dict(sd)
    tr = FastStTrainer(net2, style.to(dev))
    for batch in loaders[1]:
        tr.step(batch.squeeze(1).to(dev))
    assert torch.equal(tr.flat.cpu().double(), ph)
    # oracle, fp32 and fp64, same batches in order
    p0 = torch.cat([v.reshape(-1) for v in sd.values()]).double()
    upd = {}
    for dt in (torch.float32, torch.float64):
        itn = O.image_transform_net(4321).to(dt)
        ln = O.StyleNetwork(style.to(dt), torch.rand([1, 3, 256, 256]).to(dt),
                            vgg=O.vgg19_features(1234).to(dt))
        opt = torch.optim.Adam(itn.parameters())
        for batch in loaders[1]:
            opt.zero_grad()
            O.fast_st_closure(itn, ln, batch.squeeze(1).to(dt))
            opt.step()
        upd[dt] = torch.cat([p.detach().reshape(-1) for p in itn.parameters()]).double() - p0
    u64 = upd[torch.float64]
    e_hip = float((ph - p0 - u64).norm() / u64.norm())
    e_32 = float((upd[torch.float32] - u64).norm() / u64.norm())
    print(f"static_train update vs fp64 oracle: hip {e_hip:.2e}, fp32 oracle {e_32:.2e}")
    assert e_hip <= 5.0 * e_32


def test_fast_st_cli_train_then_convert(dev, project_root):
    """`fast_st train STYLE --synthetic 8 -e 1 -b 4` then `fast_st convert-image IMG
    STYLE`: the converted PNG == the oracle's forward of the written checkpoint on the
    same loaded image, byte for byte up to one unit of rounding."""
    from click.testing import CliRunner
    from oracle import reference_cpu as O
    from styletransfer_amd import img_utils
    from styletransfer_amd.clis import cli
    r = CliRunner().invoke(cli, ["fast_st", "train", "data/styles/picasso.jpg", "--synthetic",
                                 "8", "-e", "1", "-b", "4"])
    assert r.exit_code == 0, r.output + repr(r.exception)
    ck = project_root / "data" / "models" / "fast_st_picasso.jpg_epoch0.pth"
    assert ck.is_file()
    r = CliRunner().invoke(cli, ["fast_st", "convert-image", "data/dancing.jpg", "picasso.jpg"])
    assert r.exit_code == 0, r.output + repr(r.exception)
    got = np.asarray(Image.open(project_root / "results" / "converted_fast_st_picasso.jpg.png"))
    itn = O.image_transform_net(4321)
    itn.load_state_dict({k: v.cpu() for k, v in torch.load(ck, weights_only=True).items()})
    x = img_utils.image_loader(str(project_root / "data/dancing.jpg")).cpu()
    with torch.no_grad():
        want = np.asarray(img_utils.to_pil(itn(x)))
    diff = np.abs(got.astype(np.int32) - want.astype(np.int32))
    # the reference's byte conversion clamps to [0, 255] before * 255 (img_utils.imshow,
    # stransfer/img_utils.py:104-110), so values just above 1 wrap modulo 256: a one-unit
    # rounding difference there reads as 255 -- compare on the byte circle
    diff = np.minimum(diff, 256 - diff)
    print(f"convert-image vs oracle: max |diff| {diff.max()}, > 0: {(diff > 0).mean():.2e}")
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-2


def test_convert_config3_b32_256_forward_vs_oracle(dev):
    """BASELINE config 3 at full size: the ImageTransformNet forward of `fast_st
    convert-image` batched 32 x 256^2 (stransfer/network.py:520-611, :798-832) vs the
    oracle's fp32 forward on the same inputs and weights, 1e-4 relative (whole batch
    and every image)."""
    from oracle import reference_cpu as O
    x = torch.from_numpy(W.synthetic_image(6000, (32, 3, 256, 256)))
    net = network.ImageTransformNet(torch.rand([3, 256, 256]), batch_size=32)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
    with torch.no_grad():
        y = net(x.to(dev)).cpu()
        yr = O.image_transform_net(4321)(x)
    assert rel(y, yr) < 1e-4, rel(y, yr)
    worst = max(rel(y[i], yr[i]) for i in range(32))
    assert worst < 1e-4, worst
