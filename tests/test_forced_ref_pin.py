"""Pin tests/forced_ref.py -- the fp64 ground truth of the forced-branch ITN gradient
tests (tests/test_itn_masks_gpu.py) -- to the reference's own fixtures (VERDICT r4,
weak #1): with its branch decisions left to itself (the natural ones of an unforced
run), forced_ref's loss and parameter gradients must be exactly those of the pinned
oracle, whose fp32 run oracle/gen_golden.py checked against the reference's
`stransfer/network.py` (ImageTransformNet :461-611, static_train closure :690-731,
loss network :204-401) on the same inputs:

  * float64: every parameter's 32 projections equal itn_fp64.npz["grad64_proj"] (the
    oracle in float64) to 1e-9 relative -- a term dropped or changed in forced_ref
    alone cannot pass this;
  * float32: every parameter's [norm, 8 projections] equal itn.npz["grad_proj"] (the
    REFERENCE's own fp32 gradients) to 1e-5 relative, and the loss its "total".

CPU only (torch CPU, ~10 s)."""
import numpy as np
import pytest
import torch

import forced_ref as R
from conftest import GOLDEN
from styletransfer_amd import weights as W

ITN_SEED, VGG_SEED = 4321, 1234


def _proj(a, seed, k):
    a = np.asarray(a, np.float64).ravel()
    r = W.hash_normal(seed, a.size * k).astype(np.float64).reshape(k, a.size)
    return r @ a


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.fixture(scope="module")
def case():
    d = np.load(f"{GOLDEN}/itn.npz")
    f64 = np.load(f"{GOLDEN}/itn_fp64.npz")
    sd = W.itn_synthetic(ITN_SEED)
    vgg = W.vgg19_synthetic(VGG_SEED, 5)
    return d, f64, sd, vgg


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32], ids=["fp64", "fp32"])
def test_forced_ref_natural_branches_equal_golden(case, dtype):
    d, f64, sd, vgg = case
    ni, nv = R.natural_branches(sd, vgg, d["batch"], dtype)
    grads, total = R.forced_grads(sd, vgg, d["style"], d["batch"], ni, nv, dtype)
    keys = [k for k, _ in sd]
    assert list(grads) == keys
    gmax = max(float(g.norm()) for g in grads.values())
    worst = []
    for i, k in enumerate(keys):
        g = grads[k].double().numpy()
        if dtype == torch.float64:
            want = f64["grad64_proj"][i]
            got = np.concatenate([[np.linalg.norm(g)], _proj(g, 77, 32)])
            tol = 1e-9
        else:
            want = d["grad_proj"][i]
            got = np.concatenate([[np.linalg.norm(g)], _proj(g, 99, 8)])
            tol = 1e-5
        if want[0] < 1e-7 * gmax:
            # a conv bias that feeds an InstanceNorm: 0 in exact arithmetic, rounding
            # noise in both runs -- compare magnitudes only
            assert got[0] < 1e-5 * gmax and want[0] < 1e-5 * gmax, k
            continue
        e = _rel(got, want)
        worst.append((e, k))
        assert e <= tol, f"{k}: forced_ref {dtype} vs golden {e:.2e}"
    if dtype == torch.float32:
        assert abs(total - float(d["total"])) <= 1e-5 * abs(float(d["total"]))
    print(f"{dtype}: worst {sorted(worst)[-3:]}")


def test_golden_flip_sites():
    """Why test_itn_forward_backward_golden holds no parameter to the tight bound at the
    golden size: the fp32 reference's own run already decides loss-network branches
    differently from fp64 (a flip in the VGG prefix moves every ITN parameter's
    gradient), so all 62 parameters are flip-affected there; the forced-branch tests
    carry the tight check.  This pins that count so a change in it is seen."""
    d = np.load(f"{GOLDEN}/itn.npz")
    sd = W.itn_synthetic(ITN_SEED)
    vgg = W.vgg19_synthetic(VGG_SEED, 5)
    ni64, nv64 = R.natural_branches(sd, vgg, d["batch"], torch.float64)
    ni32, nv32 = R.natural_branches(sd, vgg, d["batch"], torch.float32)
    fi, fv = R.count_flips(ni32, ni64), R.count_flips(nv32, nv64)
    keys = [k for k, _ in sd]
    up = R.flip_upstream(keys, ni32, ni64, nv32, nv64)
    print(f"fp32-vs-fp64 flips: ITN {fi}, VGG {fv}; flip-affected params {len(up)}")
    assert fv > 0 and len(up) == 62
