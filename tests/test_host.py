"""Host-side logic that needs no GPU: the C-ABI library loads and exports every
declared symbol; image I/O parity with the reference; checkpoint helpers; module
structure / state_dict keys; the product path fails loudly without a GPU."""
import os
import re
import subprocess

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO


def test_library_exports_header_symbols():
    from styletransfer_amd import _native as N
    L = N.lib()
    assert L.stx_version() == 1
    out = subprocess.check_output(["nm", "-D", "--defined-only", N.LIB_PATH]).decode()
    syms = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    hdr = open(os.path.join(REPO, "include", "stx.h")).read()
    decl = set(re.findall(r"\b(stx_[a-z0-9_]+)\s*\(", hdr))
    assert len(decl) >= 30
    assert decl <= syms, decl - syms
    assert decl == set(N.SIGNATURES), decl ^ set(N.SIGNATURES)
    # the ABI revision the binding checks at load (a library of another revision is
    # refused, never driven with arguments whose meaning changed)
    rev = re.search(r"#define STX_ABI_VERSION (\d+)", hdr).group(1)
    assert L.stx_abi_version() == N.STX_ABI_VERSION == int(rev)


def test_struct_mirrors_match_the_library():
    """Every ctypes mirror has the size and last-member offset the compiled library has
    (stx_abi_layout): a member added to include/stx.h but not to _native.py, or the other
    way round, fails here instead of shifting fields on the GPU."""
    import ctypes as C
    from styletransfer_amd import _native as N
    out = (C.c_longlong * 12)()
    assert N.lib().stx_abi_layout(C.cast(out, C.c_void_p), 12) == 12
    mirrors = [(N.ConvParams, "unpool_out"), (N.WprepJob, "pad_"), (N.LossParts, "k"),
               (N.GramFinJob, "coef_amax"), (N.PGradJob, "pad_"), (N.ImageMeta, "tmp_offset")]
    for i, (S, last) in enumerate(mirrors):
        assert S._fields_[-1][0] == last, S
        assert (C.sizeof(S), getattr(S, last).offset) == (out[2 * i], out[2 * i + 1]), S


def test_host_queries_without_gpu():
    from styletransfer_amd import ops
    assert ops.conv_weight_dims(3, 64, 3) == (4, 64)
    assert ops.conv_weight_dims(128, 256, 3) == (128, 256)
    assert ops.coef_pitch(64) == 64 and ops.coef_pitch(96) == 128
    from styletransfer_amd import _native as N
    assert N.lib().stx_gram_ws(1, 64, 262144) > 0
    assert N.lib().stx_conv2d_wgrad_ws(8, 128, 128, 3, 1, 64, 64) > 0


def test_invalid_args_rejected():
    from styletransfer_amd import _native as N
    import ctypes as C
    p = N.ConvParams()  # all zero: must be rejected before any launch
    rc = N.lib().stx_conv2d(C.byref(p), None)
    assert rc == 1001
    assert b"unsupported" in N.lib().stx_last_error_string()


def test_pool_sum_contract_rejected():
    """stx_conv_params.pool_sum (the fused nearest-x2 upsampling backward) is refused
    before any launch unless it comes with pool_out on the split path's plain epilogue."""
    from styletransfer_amd import _native as N
    import ctypes as C
    cp, op = N.lib(), None
    # a well-formed split-path data gradient geometry (64 -> 128 at 64x64), fake pointers
    p = N.ConvParams(x=16, y=32, n=1, cin=64, h=64, w=64, cout=128, ks=3, stride=1, pad=1,
                     in_mode=0, hv=64, wv=64, ho=64, wo=64, cin_pad=64, cout_pad=128,
                     wt16=48, w_amax=64, in_amax=80, pool_sum=1)
    rc = cp.stx_conv2d(C.byref(p), op)  # no pool_out
    assert rc == 1001 and b"pool_sum" in cp.stx_last_error_string()
    p.pool_out, p.relu_out = 96, 1      # pool_out given, but a ReLU epilogue
    rc = cp.stx_conv2d(C.byref(p), op)
    assert rc == 1001 and b"pool_sum" in cp.stx_last_error_string()
    p.relu_out, p.ho, p.wo, p.hv, p.wv, p.h, p.w = 0, 63, 63, 63, 63, 63, 63  # odd output
    rc = cp.stx_conv2d(C.byref(p), op)
    assert rc == 1001 and b"pool_sum" in cp.stx_last_error_string()


def test_phase2_contract_rejected():
    """The fused Gram-backward phase (p2_z) on the split path needs a raw-input data
    gradient; any other loader mode is refused before a launch, not dropped."""
    from styletransfer_amd import _native as N
    import ctypes as C
    L = N.lib()
    for mode, (hv, wv) in ((N.STX_IN_RELU, (64, 64)), (N.STX_IN_RELU_POOL2, (32, 32)),
                           (N.STX_IN_UPSAMPLE2, (128, 128))):
        p = N.ConvParams(x=16, y=32, n=1, cin=64, h=64, w=64, cout=64, ks=3, stride=1, pad=1,
                         in_mode=mode, hv=hv, wv=wv, ho=hv, wo=wv, cin_pad=64, cout_pad=64,
                         wt16=48, w_amax=64, in_amax=80, p2_z=96, p2_wt=112, p2_c=64,
                         p2_amax=128)
        rc = L.stx_conv2d(C.byref(p), None)
        assert rc == 1001 and b"raw-input" in L.stx_last_error_string(), mode


def test_grayscale_frames_expand_to_rgb():
    """iterate_raw_frames: 2-D (grayscale) frames become HxWx3 like PIL's L -> RGB."""
    from PIL import Image
    from styletransfer_amd import video
    arr = (np.arange(2 * 5 * 7) % 251).astype(np.uint8).reshape(2, 5, 7)
    out = list(video.iterate_raw_frames(arr))
    assert len(out) == 2
    for f, g in zip(out, arr):
        assert f.shape == (5, 7, 3)
        assert np.array_equal(f, np.asarray(Image.fromarray(g).convert("RGB")))


def test_image_loader_matches_reference():
    from styletransfer_amd import img_utils
    d = np.load(os.path.join(GOLDEN, "images.npz"))
    x = img_utils.image_loader(os.path.join(REPO, "data", "dancing.jpg"))
    assert torch.equal(x.cpu(), torch.from_numpy(d["dancing_256"]))
    y = img_utils.image_loader(os.path.join(REPO, "data", "styles", "picasso.jpg"))
    assert torch.equal(y.cpu(), torch.from_numpy(d["picasso_256"]))


def test_imshow_bytes_match_reference(tmp_path):
    from PIL import Image
    from styletransfer_amd import img_utils
    d = np.load(os.path.join(GOLDEN, "images.npz"))
    p = tmp_path / "o.png"
    img_utils.imshow(torch.from_numpy(d["imshow_in"]), path=str(p))
    assert np.array_equal(np.asarray(Image.open(p)), d["imshow_out"])


def test_latest_weights_lexicographic(tmp_path, monkeypatch):
    from styletransfer_amd import constants, network
    mdir = tmp_path / "data" / "models"
    mdir.mkdir(parents=True)
    for e in (1, 9, 10):
        torch.save({"w": torch.tensor([float(e)])}, mdir / f"fast_st_wave_epoch{e}.pth")
    monkeypatch.setattr(constants, "PROJECT_ROOT_PATH", str(tmp_path))
    sd = network._load_latest_model_weigths("fast_st", "wave")
    assert float(sd["w"]) == 9.0  # reference quirk: 'epoch9' sorts after 'epoch10'
    with pytest.raises(AssertionError):
        network._load_latest_model_weigths("fast_st", "nope")


def test_itn_structure_cpu():
    from styletransfer_amd import network
    from styletransfer_amd import weights as W
    net = network.ImageTransformNet(torch.rand(3, 8, 8), batch_size=2)
    keys = list(net.state_dict().keys())
    assert keys == [k for k, _ in W.itn_synthetic(4321)]
    assert sum(p.numel() for p in net.parameters()) == 1_679_235
    assert isinstance(net[0], torch.nn.Conv2d) and net[0].padding_mode == "zeros"
    vnet = network.VideoTransformNet(torch.rand(3, 8, 8))
    assert vnet[0].in_channels == 6 and not vnet.has_external_weights


@pytest.mark.skipif(torch.cuda.device_count() > 0, reason="checks the no-GPU failure mode")
def test_product_path_fails_loudly_without_gpu():
    from styletransfer_amd import _native as N
    from styletransfer_amd import network
    net = network.ImageTransformNet(torch.rand(3, 8, 8), batch_size=1)
    with pytest.raises(N.NativeError, match="no CPU fallback"):
        net(torch.rand(1, 3, 16, 16))


def test_vgg_weights_from_local_state_dict(tmp_path):
    from styletransfer_amd import vgg as V
    sd = {}
    for idx, (co, ci) in zip((0, 2, 5, 7, 10), V.VGG_CONV_SHAPES):
        sd[f"features.{idx}.weight"] = torch.full((co, ci, 3, 3), float(idx))
        sd[f"features.{idx}.bias"] = torch.zeros(co)
    p = tmp_path / "vgg19.pth"
    torch.save(sd, p)
    ws = V.load_vgg19_weights(str(p))
    assert [float(w.flat[0]) for w, _ in ws] == [0.0, 2.0, 5.0, 7.0, 10.0]


def test_cli_help():
    from click.testing import CliRunner
    from styletransfer_amd.clis import cli
    r = CliRunner().invoke(cli, ["gatys_st", "--help"])
    assert r.exit_code == 0 and "--steps" in r.output and "-cw" in r.output
    r = CliRunner().invoke(cli, ["fast_st", "train", "--help"])
    assert r.exit_code == 0 and "--batch-size" in r.output
    r = CliRunner().invoke(cli, ["fast_st", "convert-image", "--help"])
    assert r.exit_code == 0 and "--out-dir" in r.output


def test_loader_workers_per_rank(monkeypatch):
    """The GPU-conditioned COCO loader's decode workers are sized per rank: the usable
    CPUs (affinity, cgroup quota) split over the node's ranks (LOCAL_WORLD_SIZE), minus one
    for the rank's training loop, at most 16 (stransfer/dataset.py:141-197's loader, fed
    at the data-parallel step rate)."""
    from styletransfer_amd import dataset as D
    n = D.usable_cpus()
    assert n >= 1
    for lw in (1, 2, 8):
        assert D.default_workers(lw) == max(0, min(16, n // lw - 1))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert D.default_workers() == max(0, min(16, n // 4 - 1))


def test_parity_and_gram128_host_contracts():
    """Round-5 host logic without a GPU: the 128-channel fused Gram's slab geometry and its
    single-round gate, the parity-class upsampling slab size, the trained network's slab
    jobs (the two up convs get a parity-class job), and the new stx_conv2d contracts
    (wt16_up only on an upsampled-input split conv; mse_ref only with a 128-channel
    fused Gram) refused before any launch."""
    import ctypes as C
    import torch
    from styletransfer_amd import _native as N
    from styletransfer_amd import network, ops
    assert [ops.gram_tile_units(c) for c in (3, 64, 128, 256)] == [1, 1, 3, 10]
    # conv2_2 at Gatys 512^2 (256 tiles: one round) vs fast_st's B = 8 (512 blocks)
    assert ops.conv_gram_tiles(128, 128, 256, 256, n=1, in_mode=N.STX_IN_RELU) == 256
    assert ops.conv_gram_tiles(64, 128, 256, 256, n=1, in_mode=N.STX_IN_RAW) == 256
    assert ops.conv_gram_tiles(128, 128, 128, 128, n=8, in_mode=N.STX_IN_RELU) == 0
    assert ops.conv_gram_tiles(128, 128, 256, 256, n=1, in_mode=N.STX_IN_UPSAMPLE2) == 0
    L = N.lib()
    # [a][cin16][ry][b, rx][hi, lo][cout64] fp16
    assert L.stx_conv_weight16up_bytes(64, 32) == 2 * 64 * 2 * 4 * 2 * 64 * 2
    assert L.stx_conv_weight16up_bytes(20, 40) == 2 * 32 * 2 * 4 * 2 * 64 * 2
    net = network.ImageTransformNet(torch.rand(3, 8, 8), batch_size=1).to("cpu")
    convs = [m for m in net.modules() if isinstance(m, network.Conv2d)]
    ups = [c for c in convs if c._up_input]
    assert [tuple(c.weight.shape[:2]) for c in ups] == [(64, 128), (32, 64)]
    slabs = ops.TrainedSlabs(convs)
    kinds = [slabs._jobs[i].kind for i in range(slabs._njobs)]
    assert kinds.count(N.STX_WPREP_F16UP) == 2
    assert sum(s[5] is not None for s in slabs.slabs) == 2
    base = dict(x=16, y=32, n=1, cin=64, h=32, w=32, cout=64, ks=3, stride=1, pad=1,
                cin_pad=64, cout_pad=64, wt16=48, w_amax=64, in_amax=80)
    p = N.ConvParams(in_mode=N.STX_IN_RAW, hv=32, wv=32, ho=32, wo=32, wt16_up=96, **base)
    assert L.stx_conv2d(C.byref(p), None) == 1001 and b"wt16_up" in L.stx_last_error_string()
    # the parity-class taps assume the full x2 image: a truncated virtual size (hv < 2h or
    # wv < 2w, which UPSAMPLE2 otherwise accepts) is refused, not computed with the wrong
    # border
    for hv, wv in ((64, 63), (63, 64), (62, 64)):
        p = N.ConvParams(in_mode=N.STX_IN_UPSAMPLE2, hv=hv, wv=wv, ho=hv, wo=wv, wt16_up=96,
                         **base)
        assert L.stx_conv2d(C.byref(p), None) == 1001 and b"wt16_up" in L.stx_last_error_string()
    # unpool_out: only a raw-input split data gradient with cout 64 and its operands
    p = N.ConvParams(in_mode=N.STX_IN_RAW, hv=32, wv=32, ho=32, wo=32, unpool_out=1, **base)
    assert L.stx_conv2d(C.byref(p), None) == 1001 and b"unpool_out" in L.stx_last_error_string()
    p = N.ConvParams(in_mode=N.STX_IN_RAW, hv=32, wv=64, ho=32, wo=64, gram_part=112,
                     mse_ref=128, mse_parts=144, **dict(base, w=64))
    assert L.stx_conv2d(C.byref(p), None) == 1001 and b"mse_ref" in L.stx_last_error_string()
