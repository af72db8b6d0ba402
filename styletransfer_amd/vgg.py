"""VGG-19 loss network on libstx: the fused forward/backward of the StyleNetwork
losses (Gatys hot loop and the fast_st loss network).

Reference semantics (stransfer/network.py:204-401): the VGG-19 `.features`
stack is sliced into pieces at the loss taps

    [conv1_1] [relu, conv1_2] [relu, pool, conv2_1] [relu, conv2_2] [relu] [pool, conv3_1]

with StyleLoss on the outputs of Conv2d_1..Conv2d_5 (pre-ReLU), ContentLoss on
Conv2d_4 (pre-ReLU) and FeatureReconstructionLoss on ReLU_4.  The reference
re-runs the prefix from the image for every loss (7x for the input, 2x for the
content image) and also computes VGG weight gradients; both are redundant work,
so this engine runs each layer once:

  forward   Z1 = conv1_1(x)            Z2 = conv1_2(relu Z1)
            Z3 = conv2_1(pool relu Z2) Z4 = conv2_2(relu Z3)   Z5 = conv3_1(pool relu Z4)
            (ReLU and ReLU+MaxPool are fused into the next conv's LDS halo load)
            style_l = mean((gram(Z_l) - T_l)^2)   content = mse(Z4, C4)
            feature = mse(relu Z4, relu C4)^2 / numel(Z4)
  backward  dZ5 = g_s5 A5 Z5 ; dP2 = conv3_1ᵀ(dZ5) ; dZ4 = unpool(dP2)·[Z4>0] + g_s4 A4 Z4
            + content/feature terms ; dZ3 = conv2_2ᵀ(dZ4)·[Z3>0] + g_s3 A3 Z3 ; ...
            dx = conv1_1ᵀ(dZ1)
where g is the vector of upstream gradients of the 7 losses (device tensor),
so the same code serves `total.backward()` for any loss combination.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as N
from . import ops
from . import weights as W

# tap layout of the reference StyleNetwork (stransfer/network.py:214-232)
STYLE_CONVS = (0, 1, 2, 3, 4)   # Conv2d_1..Conv2d_5
CONTENT_CONV = 3                # Conv2d_4
N_LOSSES = 7                    # style x5, content, feature
VGG_CONV_SHAPES = [(64, 3), (64, 64), (128, 64), (128, 128), (256, 128)]
# how each conv's input is formed from the previous conv's output
IN_MODES = [N.STX_IN_RAW, N.STX_IN_RELU, N.STX_IN_RELU_POOL2, N.STX_IN_RELU,
            N.STX_IN_RELU_POOL2]


def load_vgg19_weights(path: str | None = None, seed: int = 1234):
    """The first five VGG-19 convs as [(w, b)] numpy arrays.

    `torchvision.models.vgg19(pretrained=True)` (stransfer/network.py:246) needs a
    download.  A local torchvision state_dict (keys `features.{0,2,5,7,10}.*` or
    `{0,2,5,7,10}.*`) is used when `path` or $STX_VGG19_WEIGHTS names one (loaded
    with weights_only=True); otherwise deterministic synthetic weights."""
    path = path or os.environ.get("STX_VGG19_WEIGHTS")
    if path and os.path.exists(path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        out = []
        for idx in (0, 2, 5, 7, 10):
            for pre in ("features.", ""):
                if f"{pre}{idx}.weight" in sd:
                    out.append((sd[f"{pre}{idx}.weight"].float().numpy(),
                                sd[f"{pre}{idx}.bias"].float().numpy()))
                    break
            else:
                raise KeyError(f"VGG-19 weights file {path} lacks conv index {idx}")
        return out
    return W.vgg19_synthetic(seed, 5)


class VGGFeatures:
    """Frozen conv1_1..conv3_1 with prepped forward and data-gradient slabs."""

    def __init__(self, convs, device):
        self.device = torch.device(device)
        self.w, self.b, self.wt, self.wtT = [], [], [], []
        # fp16 hi/lo split slabs (conv16.hip) where the shape is eligible, else None
        self.wt16, self.wtT16 = [], []
        for (w, b), (cout, cin) in zip(convs, VGG_CONV_SHAPES):
            wt = torch.as_tensor(np.ascontiguousarray(w), dtype=torch.float32).to(self.device)
            bt = torch.as_tensor(np.ascontiguousarray(b), dtype=torch.float32).to(self.device)
            assert tuple(wt.shape) == (cout, cin, 3, 3), wt.shape
            self.w.append(wt)
            self.b.append(bt)
            self.wt.append(ops.conv_weight_prep(wt))
            self.wtT.append(ops.conv_weight_prep(wt, transpose=True))
            split = N.knob("STX_CONV_SPLIT", "1") != "0"
            self.wt16.append(ops.conv_weight_prep16(wt) if split and
                             ops.split_eligible(cin, cout, 3) else None)
            self.wtT16.append(ops.conv_weight_prep16(wt, transpose=True) if split and
                              ops.split_eligible(cout, cin, 3) else None)

    @classmethod
    def from_modules(cls, convs, device):
        """From five nn.Conv2d modules (the layers of a StyleNetwork)."""
        return cls([(c.weight.detach().cpu().numpy(), c.bias.detach().cpu().numpy())
                    for c in convs], device)

    def conv(self, l, x, out=None, in_amax=None, out_amax=None):
        cout, cin = VGG_CONV_SHAPES[l]
        return ops.conv2d(x, self.wt[l], cin, cout, 3, in_mode=IN_MODES[l], bias=self.b[l],
                          out=out, wt16=self.wt16[l], in_amax=in_amax, out_amax=out_amax)

    def dgrad(self, l, dz, out, **kw):
        """d/d(conv_l input, after its loader transform) of dz = d/dZ_l."""
        cout, cin = VGG_CONV_SHAPES[l]
        return ops.conv2d(dz, self.wtT[l], cout, cin, 3, out=out, wt16=self.wtT16[l], **kw)

    def fuses_pool(self, l, wo):
        """conv l can write relu+maxpool of its output for conv l+1 (split path)."""
        return (l + 1 < len(IN_MODES) and IN_MODES[l + 1] == N.STX_IN_RELU_POOL2
                and self.wt16[l] is not None and self.wt16[l + 1] is not None and wo > 32)

    def gram_tiles(self, l, ho, wo, n=1):
        """Fused Gram partials per image conv l emits in a batch of n (0: not fusable)."""
        cout, cin = VGG_CONV_SHAPES[l]
        # conv1_1 (3 input channels) runs on convfew.hip's split kernel without a slab
        if (cin >= 16 and self.wt16[l] is None) or N.knob("STX_GRAM_FUSE", "1") == "0":
            return 0
        return ops.conv_gram_tiles(cin, cout, ho, wo, n=n, in_mode=self._run_mode(l, wo))

    def _run_mode(self, l, wo):
        """The loader mode conv l runs with (forward): raw where conv l-1 writes the
        pooled input for it."""
        mode = IN_MODES[l]
        if mode == N.STX_IN_RELU_POOL2 and l > 0 and self.fuses_pool(l - 1, 2 * wo):
            return N.STX_IN_RAW
        return mode

    def gram_groups(self, l, ho, wo, n=1):
        """In-kernel group sums per image of conv l's fused Gram (0: not grouped).  Off
        unless STX_GRAM_GROUPED=1: the in-launch reduction (ticket counter + sc1 hand-off)
        adds ~4.6 us to each producing conv, more than the smaller finalize saves (same-
        process A/B: Gatys 512^2 695 -> 703 us, fast_st B8 4478 -> 4469 us)."""
        if N.knob("STX_GRAM_GROUPED", "0") != "1" or not self.gram_tiles(l, ho, wo, n):
            return 0
        cout, cin = VGG_CONV_SHAPES[l]
        return ops.conv_gram_groups(cin, cout, ho, wo, n=n, in_mode=self._run_mode(l, wo))

    def forward(self, x, upto=5, outs=None, amax=None, pools=None, on_layer=None, grams=None,
                content=None, keep=None):
        """[Z1..Z_upto] (pre-ReLU conv outputs).  amax: device [>=5] slots, zeroed by
        the caller; slot l+1 receives max|Z_l| (the next split conv's input scale);
        each slot is an amax group of N.STX_AMAX_SLOTS floats (slot(amax, k)).
        Where fuses_pool holds, conv l also writes P = maxpool(relu(Z_l)) (into
        pools[l] if given) and conv l+1 reads P directly.  grams[l] (if given and not
        None): conv l writes its fused Gram partials there (gram_tiles); a (slab,
        counters) pair instead: the in-kernel group sums (gram_groups) after the per-tile
        scratch.  content=(c4, parts): the content tap's conv (fused Gram, 128 channels)
        also writes its content / feature MSE sums against c4 into parts.  keep (a set of
        layer indices, or None = all): the layers whose full output is needed; a layer
        outside it that writes a fused pooled output writes that alone (its entry in the
        returned list is the pooled tensor)."""
        zs, cur, pin = [], x, None
        for l in range(upto):
            cout, cin = VGG_CONV_SHAPES[l]
            src, mode = cur, IN_MODES[l]
            if mode == N.STX_IN_RELU_POOL2 and pin is not None:
                src, mode = pin, N.STX_IN_RAW
            kw = {}
            if amax is not None:
                kw = dict(in_amax=slot(amax, l) if l > 0 else None,
                          out_amax=slot(amax, l + 1))
            pin = None
            if l + 1 < upto and self.fuses_pool(l, src.shape[3]):
                shp = (src.shape[0], cout, src.shape[2] // 2, src.shape[3] // 2)
                pin = pools[l] if pools is not None and pools[l] is not None else \
                    torch.empty(shp, device=src.device, dtype=torch.float32)
                if pools is not None:
                    pools[l] = pin
                kw["pool_out"] = pin
                if keep is not None and l not in keep and outs is None and grams is None \
                        and on_layer is None and self.wt16[l] is not None:
                    kw["pool_only"] = True
            if grams is not None and grams[l] is not None:
                if isinstance(grams[l], tuple):
                    kw["gram_part"], kw["gram_cnt"] = grams[l]
                else:
                    kw["gram_part"] = grams[l]
                if content is not None and l == CONTENT_CONV:
                    kw["mse_ref"], kw["mse_parts"] = content
            cur = ops.conv2d(src, self.wt[l], cin, cout, 3, in_mode=mode, bias=self.b[l],
                             out=None if outs is None else outs[l], wt16=self.wt16[l], **kw)
            zs.append(cur)
            if on_layer is not None:
                on_layer(l, cur)
        return zs

    def style_targets(self, style_image):
        """T_l = gram(Z_l(style)) [C][C] (StyleLoss.set_target, :125-131)."""
        zs = self.forward(style_image.contiguous())
        return [ops.gram(z) for z in zs]


@dataclass
class LossState:
    """Activations + scratch of one loss evaluation (kept for the backward)."""
    z: list = field(default_factory=list)       # Z1..Z5
    coef: list = field(default_factory=list)    # A_l per style layer
    c4: torch.Tensor = None                     # content target (pre-ReLU conv2_2)
    losses: torch.Tensor = None                 # [8] style x5, content, feature, f-mse
    fmean: torch.Tensor = None                  # [2] feature loss, its mse
    folded: bool = False                        # loss weights baked into coef
    alpha: float = 0.0
    amax: torch.Tensor = None                   # [16] max|.| slots of split-conv inputs
    amax_cleared: bool = False                  # amax already zeroed (by the engine's Adam)
    coef_amax: list = None                      # per tap: amax group >= max|A| (or None)
    pools: list = field(default_factory=lambda: [None] * 5)  # fused relu+pool outputs
    lws: list = field(default_factory=lambda: [None] * 5)    # per-layer style-loss scratch
    parts: list = field(default_factory=lambda: [None] * 5)  # deferred loss partials
    grams: list = field(default_factory=lambda: [None] * 5)  # fused Gram partial slabs
    fin_jobs: list = None                       # the last batched finalize's jobs (bench)
    mse_parts: torch.Tensor = None              # content tap's fused MSE sums (2 per tile)


def loss_forward(feat: VGGFeatures, targets, x, c4, st: LossState | None = None,
                 folded_weights=None, total=None, extra_slot=False):
    """Forward of all 7 losses for input batch x [B,3,H,W] given style targets and
    the content target c4 (= Z4 of the content image, pre-ReLU).

    folded_weights=(style_weight, content_weight): constant loss weights are baked
    into the backward operators (A_l scaled by style_weight; the content term's
    alpha*Z4 on A_4's diagonal) so the backward needs no device scalars — the
    Gatys engine's case.  None: operators for weight 1; the backward scales by the
    upstream gradient vector (autograd case).

    The five style-loss reductions are deferred (partials kept in per-layer
    workspaces) and done in one launch after the forward, together with the
    weighted total (into `total`, if given, with the folded weights)."""
    if st is None:
        st = LossState()
    dev = x.device
    if st.amax is None:
        st.amax = torch.zeros(LOSS_AMAX_GROUPS * N.STX_AMAX_SLOTS, device=dev,
                              dtype=torch.float32)
    elif not st.amax_cleared:
        st.amax.zero_()
    st.amax_cleared = False  # (the Gatys engine's Adam launch clears it for the next pass)
    if st.losses is None:
        # [style x5, content, feature, feature-mse]
        st.losses = torch.empty(N_LOSSES + 1, device=dev, dtype=torch.float32)
        st.fmean = st.losses[6:8]
    if not st.coef:
        st.coef = [None] * 5
    B, _, H, W = x.shape
    z4_shape = (B, 128, H // 2, W // 2)
    assert tuple(c4.shape) == z4_shape, (c4.shape, z4_shape)
    sw, alpha = 1.0, 0.0
    st.folded = folded_weights is not None
    if st.folded:
        sw = float(folded_weights[0])
        alpha = float(folded_weights[1]) * 2.0 / (B * 128 * (H // 2) * (W // 2))
    st.alpha = alpha
    st.c4 = c4
    split = N.knob("STX_GRAM_SPLIT", "1") != "0"
    overlap = N.knob("STX_LOSS_STREAM", "0") != "0"  # measured slower (A/B)
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev) if overlap else main
    capturing = False
    if overlap:
        # the side stream never grows the shared scratch buffer: size it here, on main
        L = N.lib()
        hw = [(64, H * W), (64, H * W), (128, (H // 2) * (W // 2)),
              (128, (H // 2) * (W // 2)), (256, (H // 4) * (W // 4))]
        need = max([L.stx_gram_ws(B, c, n) for c, n in hw] +
                   [L.stx_mse_ws(B * 128 * (H // 2) * (W // 2))])
        ops.WS.get(need, dev)
        side.wait_stream(main)
        capturing = torch.cuda.is_current_stream_capturing()
        if not capturing:
            for t in [st.losses, st.amax, c4] + [c for c in st.coef if c is not None]:
                t.record_stream(side)

    # conv layers whose Gram partials come out of the conv epilogue (no re-read of Z)
    hs = [H, H, H // 2, H // 2, H // 4]
    for l in range(5):
        nt = feat.gram_tiles(l, hs[l], hs[l] * W // H, n=B) if split else 0
        ng = feat.gram_groups(l, hs[l], hs[l] * W // H, n=B) if nt else 0
        if nt == 0:
            st.grams[l] = None
        elif ng:  # per-tile scratch + group sums, and the group arrival counters
            if not isinstance(st.grams[l], tuple) or st.grams[l][0].numel() != B * (nt + ng) * 4096:
                st.grams[l] = (torch.empty(B * (nt + ng) * 4096, device=dev, dtype=torch.float32),
                               torch.zeros(B * ng, device=dev, dtype=torch.int32))
        elif st.grams[l] is None or isinstance(st.grams[l], tuple) or \
                st.grams[l].numel() != B * ops.gram_tile_units(VGG_CONV_SHAPES[l][0]) * nt * 4096:
            st.grams[l] = torch.empty(B * ops.gram_tile_units(VGG_CONV_SHAPES[l][0]) * nt * 4096,
                                      device=dev, dtype=torch.float32)

    fuse_content = N.knob("STX_CONTENT_FUSE", "1") != "0"
    # the content tap's Gram in its conv epilogue: the content / feature MSE sums too
    content = None
    if st.grams[CONTENT_CONV] is not None and fuse_content:
        nt4 = feat.gram_tiles(CONTENT_CONV, hs[CONTENT_CONV], hs[CONTENT_CONV] * W // H, n=B)
        if st.mse_parts is None or st.mse_parts.numel() != 2 * B * nt4:
            st.mse_parts = torch.empty(2 * B * nt4, device=dev, dtype=torch.float32)
        content = (c4, st.mse_parts)
    # the five taps' Gram finalizes in one launch after the forward (STX_FIN_BATCH=0: one
    # finalize launch per tap, right after its partials)
    # (with the loss stream the jobs are recorded on the side stream's calls and the one
    # finalize launch runs on main after the join)
    fin = ops.FinalizeBatch() if N.knob("STX_FIN_BATCH", "1") != "0" else None

    def tap_loss(i, l, z, b_, c_, fuse_mse):
        if fuse_mse:  # style loss + content/feature/feature-mse in one pass over z
            st.parts[i], st.coef[i] = ops.style_content_loss(
                z, targets[i], c4, st.losses[5:8], weight=sw, diag_alpha=alpha,
                coef=st.coef[i], z_amax=slot(st.amax, l + 1), defer_ws=st.lws[i], fin=fin)
            return
        fused_mse = False
        if st.grams[l] is not None:
            gp = st.grams[l]
            if isinstance(gp, tuple):  # the group sums after the B * nt tile slots
                ng = gp[1].numel() // b_
                gp = gp[0][gp[0].numel() - b_ * ng * 4096:]
            fused_mse = l == CONTENT_CONV and content is not None
            st.parts[i], st.coef[i] = ops.style_loss_from_parts(
                gp, gp.numel() // (b_ * ops.gram_tile_units(c_) * 4096), b_, c_, z[0, 0].numel(),
                targets[i], weight=sw, diag_alpha=alpha if l == CONTENT_CONV else 0.0,
                coef=st.coef[i], defer_ws=st.lws[i], fin=fin,
                mse_parts=st.mse_parts if fused_mse else None,
                mse_out=st.losses[5:8] if fused_mse else None)
        else:
            st.parts[i], st.coef[i] = ops.style_loss(
                z, targets[i], weight=sw, diag_alpha=alpha if l == CONTENT_CONV else 0.0,
                coef=st.coef[i], z_amax=slot(st.amax, l + 1) if split else None,
                defer_ws=st.lws[i], fin=fin)
        if l == CONTENT_CONV and not fused_mse:  # content, feature, feature-mse: one pass
            ops.mse(z, c4, mode=2, out=st.losses[5:8])

    st.coef_amax = [None] * 5  # (per style tap)

    def on_layer(l, z):
        # the style loss of layer l (and the content/feature losses at conv2_2) run on
        # the side stream while the next conv runs: memory-bound reductions under
        # compute-bound convs, joined before the backward
        if overlap:
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            if not capturing:
                z.record_stream(side)
        with torch.cuda.stream(side):
            i = STYLE_CONVS.index(l)
            b_, c_ = z.shape[:2]
            fuse_mse = l == CONTENT_CONV and st.grams[l] is None and split and fuse_content
            L = N.lib()
            need = (L.stx_style_content_ws if fuse_mse else L.stx_gram_ws)(b_, c_,
                                                                             z[0, 0].numel())
            if st.lws[i] is None or st.lws[i].numel() < need:
                st.lws[i] = torch.empty(need, device=dev, dtype=torch.uint8)
            njobs = len(fin.jobs) if fin is not None else 0
            tap_loss(i, l, z, b_, c_, fuse_mse)
            if i in COEF_AMAX_SLOT and fin is not None and len(fin.jobs) == njobs + 1:
                # the batched finalize also writes max|A| of the taps whose Gram backward
                # runs inside a data-gradient conv: that phase's split-MFMA A scale
                st.coef_amax[i] = slot(st.amax, COEF_AMAX_SLOT[i])
                fin.jobs[-1].coef_amax = st.coef_amax[i].data_ptr()

    st.z = feat.forward(x, 5, st.z if st.z else None, amax=st.amax, pools=st.pools,
                        on_layer=on_layer, grams=st.grams, content=content)
    if overlap:
        main.wait_stream(side)
        if not capturing:
            for c in st.coef:
                c.record_stream(main)
    if fin is not None:
        # (the jobs stay on the state for bench.py's per-tap cost of the batched launch)
        st.fin_jobs = list(fin.jobs)
        fin.flush()  # every tap's G, backward operator A and loss partials: one launch
    # the 5 style losses (+ the weighted total) in one launch
    w = None
    extra = None
    if total is not None:
        fw = folded_weights if folded_weights is not None else (1.0, 1.0)
        w = [float(fw[0])] * 5 + [float(fw[1])]
        extra = st.losses[5:6]
        if extra_slot:  # st.losses[8] (written by the caller, e.g. TV) joins the total
            w += [0.0, 0.0, 1.0]
            extra = st.losses[5:9]
    ops.loss_finalize(st.parts, st.losses[0:5], extra=extra, weights=w, total=total)
    return st


_SIDE = {}


# amax groups of LossState.amax: 0..5 forward, 6..10 backward split-conv inputs, 11 / 12
# max|A| of the taps whose Gram backward is a data-gradient conv's second phase
LOSS_AMAX_GROUPS = 17  # LossState.amax: the groups below
COEF_AMAX_SLOT = {0: 11, 1: 15, 2: 12, 3: 16, 4: 14}  # max|A| per tap (split phase /
# composed weights / the unpool epilogues of conv2_1^T and conv3_1^T)
COMPOSE_AMAX_SLOT = 13  # max|A5 W| of the composed conv3_1 data-gradient weights


def slot(amax, k):
    """The k-th amax group of a slot vector (include/stx.h STX_AMAX_SLOTS)."""
    return amax[k * N.STX_AMAX_SLOTS:(k + 1) * N.STX_AMAX_SLOTS]


def _side_stream(dev):
    """Per-device secondary stream for the loss reductions (loss_forward)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _SIDE.get(key)
    if s is None:
        s = _SIDE[key] = torch.cuda.Stream(torch.device("cuda", key))
    return s


def loss_values(st: LossState):
    """[style1..5, content, feature] (a view of the device loss vector)."""
    return st.losses[:N_LOSSES]


def loss_backward(feat: VGGFeatures, st: LossState, g=None, dx=None, feature_grad=True,
                  scratch=None):
    """dx = sum_i g[i] * d loss_i / dx (g: device [7]: style x5, content, feature), or,
    for a folded forward, the gradient of the folded weighted total (g ignored).

    Six launches: the Gram backward of the pooled layers runs as a 1x1 MFMA conv with
    the ReLU+MaxPool backward fused into its epilogue; the Gram backward of the
    other layers is a second GEMM phase inside the data-gradient conv, after its
    ReLU mask."""
    z = st.z
    B = z[0].shape[0]
    sc = scratch if scratch is not None else {}

    def buf(name, shape):
        t = sc.get(name)
        if t is None or tuple(t.shape) != tuple(shape):
            t = torch.empty(shape, device=z[0].device, dtype=torch.float32)
            sc[name] = t
        return t

    folded = st.folded
    s = (lambda i: None) if folded else (lambda i: g[i:i + 1])
    am = st.amax  # slots 0..5: forward; 6..10: backward split-conv inputs; COEF_AMAX_SLOT;
    # COMPOSE_AMAX_SLOT
    sp = feat.wt16[1] is not None  # split kernels in use
    n4 = (B, 128, z[3].shape[2] // 2, z[3].shape[3] // 2)
    ca = st.coef_amax if st.coef_amax else [None] * 5
    # dZ4 = unpool(dP2)[Z4 > 0] + A4 Z4 (+ the folded content term) in the epilogue of the
    # conv that produces dP2 (stx_conv_params.unpool_out): dP2 never reaches HBM
    dz4 = None
    up4 = None
    if sp and ca[3] is not None and n4[3] % 32 == 0 and n4[2] % 4 == 0 and \
            N.knob("STX_UNPOOL_FUSE", "1") != "0":
        up4 = dict(unpool_out=(z[3], st.coef[3], ca[3], slot(am, 4), s(3)),
                   aux=st.c4 if folded else None, aux_scale=-st.alpha,
                   out_amax=slot(am, 7) if folded else None)
    # (STX_COMPOSE=0: the Gram backward of conv3_1 as its own 1x1 pass, dZ5 = A5 Z5; A/B)
    if sp and B == 1 and feat.wtT16[4] is not None and ca[4] is not None and \
            N.knob("STX_COMPOSE", "1") != "0":
        # conv3_1's output feeds only its style loss, so dP2 = conv3_1^T(A5 Z5) =
        # conv^T_{A5 W}(Z5): A5 folded into the data-gradient weights (one small GEMM
        # launch that writes the split slab), dZ5 never formed.  One operator per image:
        # B == 1.
        sc["compose5"] = ops.conv_weight_compose16(
            st.coef[4], ca[4], feat.w[4], feat.wtT16[4][1], slot(am, COMPOSE_AMAX_SLOT),
            scale=s(4), out=sc.get("compose5"))
        cout, cin = VGG_CONV_SHAPES[4]
        if up4:
            dz4 = ops.conv2d(z[4], None, cout, cin, 3, out=buf("dz4", z[3].shape),
                             wt16=(sc["compose5"], slot(am, COMPOSE_AMAX_SLOT)),
                             in_amax=slot(am, 5), **up4)
        else:
            dp2 = ops.conv2d(z[4], None, cout, cin, 3, out=buf("dp2", n4),
                             wt16=(sc["compose5"], slot(am, COMPOSE_AMAX_SLOT)),
                             in_amax=slot(am, 5))
    else:
        # conv3_1 output: dZ5 = A5 Z5
        dz5 = ops.gram_bwd_fused(st.coef[4], z[4], out=buf("dz5", z[4].shape), acc_scale=s(4),
                                 out_amax=slot(am, 6), z_amax=slot(am, 5) if sp else None)
        # -> grad wrt pool(relu Z4)
        if up4:
            dz4 = feat.dgrad(4, dz5, buf("dz4", z[3].shape), in_amax=slot(am, 6), **up4)
        else:
            dp2 = feat.dgrad(4, dz5, buf("dp2", n4), in_amax=slot(am, 6))
    # dZ4 = unpool(dP2)*[Z4>0] + A4 Z4 (+ content)
    if dz4 is None:
        dz4 = ops.gram_bwd_fused(st.coef[3], z[3], out=buf("dz4", z[3].shape), acc_scale=s(3),
                                 up_dp=dp2, aux=st.c4 if folded else None, aux_scale=-st.alpha,
                                 out_amax=slot(am, 7) if folded else None,
                                 z_amax=slot(am, 4) if sp else None)
    n = z[3].numel()
    dz4_amax = slot(am, 7) if folded else None
    if not folded:
        ops.diff_scale(z[3], st.c4, 2.0 / n, s1=g[5:6], out=dz4, accumulate=True)
        if feature_grad:
            ops.diff_scale(z[3], st.c4, 4.0 / (float(n) * float(n)), s1=g[6:7],
                           s2=st.fmean[1:2], relu=True, out=dz4, accumulate=True)
    # dZ3 = conv2_2^T(dZ4)*[Z3>0] + A3 Z3
    dz3 = feat.dgrad(3, dz4, buf("dz3", z[2].shape), mask=z[2], p2_z=z[2],
                     p2_coef=st.coef[2], p2_scale=s(2), in_amax=dz4_amax, out_amax=slot(am, 8),
                     p2_amax=slot(am, 3), p2_wt_amax=ca[2])
    # -> grad wrt pool(relu Z2)
    n2 = (B, 64, z[1].shape[2] // 2, z[1].shape[3] // 2)
    if sp and ca[1] is not None and n2[3] % 32 == 0 and n2[2] % 4 == 0 and \
            N.knob("STX_UNPOOL_FUSE", "1") != "0":
        # dZ2 = unpool(dP1) [Z2 > 0] + A2 Z2 in conv2_1^T's epilogue: dP1 never reaches HBM
        dz2 = feat.dgrad(2, dz3, buf("dz2", z[1].shape), in_amax=slot(am, 8),
                         out_amax=slot(am, 9),
                         unpool_out=(z[1], st.coef[1], ca[1], slot(am, 2), s(1)))
    else:
        dp1 = feat.dgrad(2, dz3, buf("dp1", n2), in_amax=slot(am, 8))
        dz2 = ops.gram_bwd_fused(st.coef[1], z[1], out=buf("dz2", z[1].shape), acc_scale=s(1),
                                 up_dp=dp1, out_amax=slot(am, 9),
                                 z_amax=slot(am, 2) if sp else None)
    # dZ1 = conv1_2^T(dZ2)*[Z1>0] + A1 Z1
    dz1 = feat.dgrad(1, dz2, buf("dz1", z[0].shape), mask=z[0], p2_z=z[0],
                     p2_coef=st.coef[0], p2_scale=s(0), in_amax=slot(am, 9), p2_amax=slot(am, 1),
                     out_amax=slot(am, 10) if sp else None, p2_wt_amax=ca[0])
    # conv1_1 dgrad -> image (64 -> 3 GEMM + col2im; on the split MFMA given max|dZ1|)
    xs = (B, 3, z[0].shape[2], z[0].shape[3])
    if dx is None:
        dx = torch.empty(xs, device=z[0].device, dtype=torch.float32)
    return feat.dgrad(0, dz1, dx, in_amax=slot(am, 10) if sp else None)


def content_target(feat: VGGFeatures, content, out=None, amax=None):
    """C4 = conv2_2 output of the content image (ContentLoss target, pre-ReLU).
    amax: optional zeroed slot vector (>= 5 groups): each conv then emits its output's
    max|.| for the next split conv instead of that conv re-reading its input."""
    # (conv1_2's Z2 is read by nothing here: only its pooled output is written)
    return feat.forward(content.contiguous(), 4, amax=amax, keep={3})[3] if out is None else \
        feat.forward(content.contiguous(), 4, [None, None, None, out], amax=amax)[3]


class GatysEngine:
    """One Gatys iteration = forward + backward + Adam on the image, as a single
    hipGraph replay (BASELINE.json config 2):

        opt.zero_grad(); net(x, content)
        (style_weight*sum(style) + content_weight*content).backward(); opt.step()

    All buffers are static so the iteration can be captured once and replayed.
    """

    def __init__(self, feat: VGGFeatures, style_image, content_image, style_weight=100_000,
                 content_weight=1, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, init=None,
                 targets=None):
        dev = feat.device
        self.feat = feat
        if targets is None:
            targets = feat.style_targets(style_image.to(dev, torch.float32))
        self.targets = [t.reshape(t.shape[-2:]).contiguous() for t in targets]
        self.content = content_image.to(dev, torch.float32).contiguous()
        self.c4 = content_target(feat, self.content).clone()
        src = self.content if init is None else init.to(dev, torch.float32)
        self.x = src.clone().contiguous()
        self.grad = torch.zeros_like(self.x)
        self.m = torch.zeros_like(self.x)
        self.v = torch.zeros_like(self.x)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.adam_ws = torch.zeros(16, dtype=torch.float32, device=dev)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.sw, self.cw = float(style_weight), float(content_weight)
        self.g = torch.tensor([self.sw] * 5 + [self.cw, 0.0], device=dev, dtype=torch.float32)
        self.total = torch.zeros((), device=dev, dtype=torch.float32)
        self.st = LossState()
        self.scratch = {}
        self.graph = None

    def _iteration(self):
        loss_forward(self.feat, self.targets, self.x, self.c4, self.st,
                     folded_weights=(self.sw, self.cw), total=self.total)
        loss_backward(self.feat, self.st, dx=self.grad, feature_grad=False,
                      scratch=self.scratch)
        # the Adam launch also zeroes the amax groups for the next iteration's forward
        ops.adam_step(self.x, self.grad, self.m, self.v, self.step_dev, self.adam_ws, self.lr,
                      self.betas[0], self.betas[1], self.eps, clear=self.st.amax)
        self.st.amax_cleared = True

    def capture(self, warmup=2):
        """Capture one iteration into a hipGraph (after `warmup` eager iterations,
        which also allocate every buffer)."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._iteration()
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with ops.graph_capture(self.graph):
            self._iteration()
        return self

    def step(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self._iteration()
        return self.total

    def run(self, steps, graph=True):
        """`steps` iterations; with graph=True the first one runs eagerly (it
        allocates every buffer) and the rest replay a captured hipGraph."""
        if steps <= 0:
            return self.x
        if not graph:
            for _ in range(steps):
                self._iteration()
            return self.x
        self.capture(warmup=1)
        for _ in range(steps - 1):
            self.graph.replay()
        return self.x

    def losses(self):
        """[style x5, content, feature] of the last forward (device tensor)."""
        return loss_values(self.st)


class GatysLBFGS:
    """StyleNetwork.train_gatys (stransfer/network.py:411-458) as hipGraph replays:
    torch.optim.LBFGS (lr 1, max_iter 20, max_eval 25, tolerance_grad 1e-7,
    tolerance_change 1e-9, history 100) over the image with the closure

        zero_grad; net(x, content); (style_weight*style + content_weight*content).backward()

    Two graphs: `eval` (closure + gradient statistics) for the evaluation that opens an
    outer step, and `iter` (stx_lbfgs_direction -- pair update, compact two-loop
    direction, x += t d -- then the closure and the statistics) for every loop
    iteration; optim.LBFGS.run drives them with torch's control flow and one host read
    per iteration.  Every closure evaluation the graphs make is one torch makes too:
    torch's last iteration of an outer step (n_iter == max_iter) moves x without
    evaluating, and the next step opens with a closure at that point -- the `iter`
    graph's evaluation, reused.  The one exception is an iteration that stops on
    g.d > -tolerance_change: x does not move and its (identical) re-evaluation is
    discarded."""

    def __init__(self, feat: VGGFeatures, style_image, content_image, style_weight=100_000,
                 content_weight=1, targets=None, init=None, **lbfgs_kw):
        from .optim import LBFGS
        dev = feat.device
        self.feat = feat
        if targets is None:
            targets = feat.style_targets(style_image.to(dev, torch.float32))
        self.targets = [t.reshape(t.shape[-2:]).contiguous() for t in targets]
        self.content = content_image.to(dev, torch.float32).contiguous()
        self.c4 = content_target(feat, self.content).clone()
        src = self.content if init is None else init.to(dev, torch.float32)
        self.x = src.clone().contiguous()
        self.grad = torch.zeros_like(self.x)
        self.sw, self.cw = float(style_weight), float(content_weight)
        self.total = torch.zeros((), device=dev, dtype=torch.float32)
        self.st = LossState()
        self.scratch = {}
        self.opt = LBFGS([self.x], **lbfgs_kw)
        self.opt._buffers(self.x.numel(), dev)
        self.g_eval = self.g_iter = None
        self._at_x = None  # the latest evaluation, made at the current x
        self.closure_runs = 0  # closure evaluations actually executed (graph replays)

    def _closure(self):
        loss_forward(self.feat, self.targets, self.x, self.c4, self.st,
                     folded_weights=(self.sw, self.cw), total=self.total)
        loss_backward(self.feat, self.st, dx=self.grad, feature_grad=False,
                      scratch=self.scratch)
        # the statistics launch also zeroes the amax groups for the next forward
        self.opt.grad_stats(self.grad.view(-1), self.total.view(1), clear=self.st.amax)
        self.st.amax_cleared = True

    def capture(self):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._closure()  # allocates every buffer (x unchanged: no optimiser state)
        torch.cuda.current_stream().wait_stream(s)
        b = self.opt._buf
        self.g_eval = torch.cuda.CUDAGraph()
        with ops.graph_capture(self.g_eval):
            self._closure()
            b["host"].copy_(b["scal"], non_blocking=True)  # the scalars torch tests
        self.g_iter = torch.cuda.CUDAGraph()
        with ops.graph_capture(self.g_iter, pool=self.g_eval.pool()):
            self.opt.direction(self.grad.view(-1))
            self._closure()
            b["host"].copy_(b["scal"], non_blocking=True)
        return self

    def _read(self):
        # the graph's last node copied scal into the pinned mirror
        loss, gmax, gtd, t, smax, flag = self.opt._scal_host(0, 1, 3, 4, 5, 6)
        return loss, gmax, gtd, t, smax, flag

    def step(self, on_eval=None):
        """One outer optimizer.step(closure); returns its opening loss (host float).
        on_eval(loss): called with the loss of every evaluation torch counts."""
        if self.g_iter is None:
            self.capture()

        def evaluate():
            self.g_eval.replay()
            self.closure_runs += 1
            loss, gmax = self.opt._scal_host(0, 1)
            self._at_x = (loss, loss, gmax, self.grad.view(-1))
            return self._at_x

        pending = []

        def move(g):
            self.g_iter.replay()
            self.closure_runs += 1
            loss, gmax, gtd, t, smax, flag = self._read()
            self._at_x = (loss, loss, gmax, self.grad.view(-1))
            pending.append(self._at_x)
            return gtd, t, smax, bool(flag)

        def evaluate_after_move():
            return pending.pop() if pending else evaluate()

        first, self._at_x = self._at_x, None
        ret = self.opt.run(evaluate_after_move, move, first=first, on_eval=on_eval)
        if self._at_x is None:  # (no evaluation or move ran: gradient already tiny)
            self._at_x = first
        return ret

    @property
    def func_evals(self):
        return self.opt.state[self.x].get("func_evals", 0)

    def history(self):
        """(committed pairs, torch n_iter) from the device state."""
        pairs, n_iter = self.opt._scal(8, 9)
        return int(pairs), int(n_iter)

    def run(self, steps):
        for _ in range(steps):
            self.step()
        return self.x
