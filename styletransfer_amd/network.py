"""Networks and losses — the `stransfer.network` API (tupini07/StyleTransfer,
stransfer/network.py) on MI355X kernels.

Every class and method of the reference keeps its name, arguments, defaults,
attributes and side effects (`.loss` attributes set by forward, piece lists,
checkpoint naming).  Arithmetic runs on libstx (HIP/gfx950) through
`styletransfer_amd.autograd`; the StyleNetwork loss evaluation is one fused
forward/backward over the VGG prefix (styletransfer_amd/vgg.py) instead of the
reference's per-loss prefix re-runs — same loss values, ~5.8x less arithmetic.

Documented differences (all numerics-neutral):
  * pretrained VGG-19 weights are a remote download in the reference
    (:246); here `vgg_weights=` / $STX_VGG19_WEIGHTS (a local torchvision
    state_dict) or deterministic synthetic weights;
  * VGG parameters are frozen (the reference leaves requires_grad=True and
    computes VGG weight gradients nobody reads);
  * `padding_mode='reflection'` = zero padding (torch 1.1.0 semantics);
  * optim.Adam arguments map to the HIP Adam (`styletransfer_amd.optim.Adam`).
"""
from __future__ import annotations

import logging
import os
import shutil
import weakref

import numpy as np
import torch
import torch.nn as nn
import torch.optim as optim
from tqdm import tqdm

from . import _native as N
from . import autograd as A
from . import c_logging, constants, dataset, img_utils
from . import optim as stx_optim
from . import vgg as V
from . import weights as W
from .layers import Conv2d, InstanceNorm2d, MaxPool2d, ReLU, Upsample

LOGGER = c_logging.get_logger()


def _dev(t: torch.Tensor) -> torch.Tensor:
    return t.to(constants.DEVICE, torch.float32)


class _NullWriter:
    def __init__(self, *a, **k):
        pass

    def add_scalar(self, *a, **k):
        pass

    def add_image(self, *a, **k):
        pass


def get_tensorboard_writer(path: str):
    """stransfer/network.py:25-35 (tensorboardX when installed, else a no-op writer)."""
    shutil.rmtree(path, ignore_errors=True)
    try:
        from tensorboardX import SummaryWriter
    except ImportError:
        return _NullWriter(path)
    return SummaryWriter(path)


def adaptive_torch_load(weights_path: str):
    """stransfer/network.py:38-50; loads tensors only (weights_only=True)."""
    loc = "cuda" if constants.DEVICE.type == "cuda" else "cpu"
    return torch.load(weights_path, map_location=loc, weights_only=True)


def _load_latest_model_weigths(model_name: str, style_name: str, models_path="data/models/"):
    """Lexicographically last matching checkpoint (stransfer/network.py:53-76; the
    reference's sort puts epoch9 after epoch10 — kept)."""
    models_path = os.path.join(constants.PROJECT_ROOT_PATH, models_path)
    try:
        names = os.listdir(models_path)
    except FileNotFoundError:
        names = []
    try:
        latest = sorted(x for x in names if x.startswith(model_name) and style_name in x)[-1]
    except IndexError:
        LOGGER.critical("There are no weights for the specified model name (%s) and style "
                        "(%s). In the specified path: %s", model_name, style_name, models_path)
        raise AssertionError("There are no weights for the specified model name and style.")
    return adaptive_torch_load(os.path.join(models_path, latest))


# ============================================================== losses
class StyleLoss(nn.Module):
    """stransfer/network.py:79-131."""

    def __init__(self, target: torch.Tensor):
        super().__init__()
        self.set_target(target)

    def gram_matrix(self, input: torch.Tensor) -> torch.Tensor:
        return A.GramFn.apply(input)

    def forward(self, input: torch.Tensor) -> torch.Tensor:
        self.loss = A.StyleLossFn.apply(input, self.target)
        return input

    def set_target(self, target: torch.Tensor):
        with torch.no_grad():
            self.target = A.GramFn.apply(target.detach().contiguous()).detach()


class ContentLoss(nn.Module):
    """stransfer/network.py:134-164."""

    def __init__(self, target: torch.Tensor):
        super().__init__()
        self.set_target(target)

    def set_target(self, target: torch.Tensor):
        self.target = target.detach()

    def forward(self, input: torch.Tensor) -> torch.Tensor:
        self.loss = A.MSELossFn.apply(input, _expand(self.target, input))
        return input


class FeatureReconstructionLoss(nn.Module):
    """stransfer/network.py:167-201: mse(input, target)^2 / numel."""

    def __init__(self, target: torch.Tensor):
        super().__init__()
        self.set_target(target)

    def set_target(self, target: torch.Tensor):
        self.target = target.detach()

    def forward(self, input: torch.Tensor) -> torch.Tensor:
        self.loss = A.FeatureLossFn.apply(input, _expand(self.target, input))
        return input


def _expand(t, like):
    if t.shape == like.shape:
        return t
    return t.expand_as(like).contiguous()  # F.mse_loss broadcasting semantics


# ============================================================== VGG / StyleNetwork
def vgg19_features(weights=None, device=None) -> nn.Sequential:
    """VGG-19 `.features` (cfg E) built from libstx layers.  conv1_1..conv3_1 take
    `weights` (see vgg.load_vgg19_weights); deeper convs (never executed by the
    losses) get synthetic weights."""
    device = device or constants.DEVICE
    first = V.load_vgg19_weights(weights) if not isinstance(weights, list) else weights
    rest = W.vgg19_synthetic(1234, 16)[5:]
    params = list(first) + list(rest)
    layers, cin, k = [], 3, 0
    for v in W.VGG19_CFG:
        if v == "M":
            layers.append(MaxPool2d(kernel_size=2, stride=2))
            continue
        conv = Conv2d(cin, v, kernel_size=3, padding=1)
        with torch.no_grad():
            conv.weight.copy_(torch.as_tensor(np.ascontiguousarray(params[k][0])))
            conv.bias.copy_(torch.as_tensor(np.ascontiguousarray(params[k][1])))
        layers += [conv, ReLU(inplace=True)]
        cin, k = v, k + 1
    net = nn.Sequential(*layers).to(device).eval()
    for p in net.parameters():
        p.requires_grad_(False)
    return net


class StyleNetwork(nn.Module):
    """Gatys et al. loss network (stransfer/network.py:204-458)."""

    content_layers = ["Conv2d_4"]
    style_layers = ["Conv2d_1", "Conv2d_2", "Conv2d_3", "Conv2d_4", "Conv2d_5"]
    feature_loss_layers = ["ReLU_4"]

    def __init__(self, style_image: torch.Tensor, content_image: torch.Tensor = None,
                 vgg_weights=None):
        super().__init__()
        self.content_losses, self.style_losses, self.feature_losses = [], [], []
        if content_image is None:
            content_image = torch.zeros([1, 3, 256, 256])  # :241-243
        style_image, content_image = _dev(style_image), _dev(content_image)
        vgg = vgg19_features(vgg_weights)
        self.net_pieces = [nn.Sequential()]
        cur, i = 0, 0
        with torch.no_grad():
            for layer in vgg:  # piece slicing as :264-314
                if isinstance(layer, nn.Conv2d):
                    i += 1
                if isinstance(layer, nn.ReLU):
                    layer.inplace = False
                name = type(layer).__name__ + f"_{i}"
                self.net_pieces[cur].add_module(name, layer)
                tapped = False
                if name in self.content_layers:
                    self.content_losses.append(
                        [ContentLoss(self.run_through_pieces(content_image)), cur])
                    tapped = True
                if name in self.style_layers:
                    self.style_losses.append([StyleLoss(self.run_through_pieces(style_image)), cur])
                    tapped = True
                if name in self.feature_loss_layers:
                    self.feature_losses.append(
                        [FeatureReconstructionLoss(self.run_through_pieces(content_image)), cur])
                    tapped = True
                if tapped:
                    self.net_pieces.append(nn.Sequential())
                    cur += 1
        self._pieces = nn.ModuleList(self.net_pieces)
        self._feat = None
        self._feat_key = None
        self._content_key = None

    # ---------------------------------------------------------------- pieces
    def run_through_pieces(self, input_g: torch.Tensor, until=-1) -> torch.Tensor:
        """stransfer/network.py:316-340."""
        x = _dev(input_g) if not input_g.is_cuda else input_g
        pieces = self.net_pieces if until == -1 else self.net_pieces[:until + 1]
        for piece in pieces:
            x = piece(x)
        return x

    def get_total_current_content_loss(self, weight=1) -> torch.Tensor:
        return weight * torch.stack([x[0].loss for x in self.content_losses]).sum()

    def get_total_current_feature_loss(self, weight=1) -> torch.Tensor:
        return weight * torch.stack([x[0].loss for x in self.feature_losses]).sum()

    def get_total_current_style_loss(self, weight=1) -> torch.Tensor:
        return weight * torch.stack([x[0].loss for x in self.style_losses]).sum()

    # ---------------------------------------------------------------- fused engine
    def _standard_layout(self) -> bool:
        return (list(self.content_layers) == ["Conv2d_4"]
                and list(self.style_layers) == StyleNetwork.style_layers
                and list(self.feature_loss_layers) == ["ReLU_4"]
                and [i for _, i in self.style_losses] == [0, 1, 2, 3, 5]
                and [i for _, i in self.content_losses] == [3]
                and [i for _, i in self.feature_losses] == [4])

    def _convs(self):
        return [m for p in self.net_pieces for m in p if isinstance(m, nn.Conv2d)][:5]

    def features(self) -> V.VGGFeatures:
        convs = self._convs()
        key = tuple((c.weight.data_ptr(), c.weight._version) for c in convs)
        if self._feat is None or self._feat_key != key:
            self._feat = V.VGGFeatures.from_modules(convs, constants.DEVICE)
            self._feat_key = key
        return self._feat

    def _set_content_targets(self, content_image):
        # keyed on the tensor object itself (a weak reference) and its version: a new
        # tensor that lands in a recycled allocator block (same data_ptr, version 0)
        # is a different content image and must be re-targeted
        key = self._content_key
        if key is not None and key[0]() is content_image and key[1] == content_image._version:
            return
        feat = self.features()
        with torch.no_grad():
            c4 = V.content_target(feat, content_image).clone()
            self.content_losses[0][0].set_target(c4)
            self.feature_losses[0][0].set_target(A.ReLUFn.apply(c4))
        self._content_key = (weakref.ref(content_image), content_image._version)

    def forward(self, input_image: torch.Tensor, content_image=None, style_image=None) -> None:
        """stransfer/network.py:366-401.  Sets `.loss` on every loss module."""
        input_image = input_image if input_image.is_cuda else _dev(input_image)
        if content_image is not None and not content_image.is_cuda:
            content_image = _dev(content_image)
        if not self._standard_layout():
            return self._forward_generic(input_image, content_image, style_image)
        if content_image is not None:
            self._set_content_targets(content_image.contiguous())
        if style_image is not None:
            # reference quirk (:391-394): style targets are re-set from content_image
            with torch.no_grad():
                zs = self.features().forward(content_image.contiguous())
                for (loss, _), z in zip(self.style_losses, zs):
                    loss.target = A.GramFn.apply(z).detach()
        c4 = self.content_losses[0][0].target
        z4_shape = (input_image.shape[0], 128, input_image.shape[2] // 2,
                    input_image.shape[3] // 2)
        if tuple(c4.shape) != z4_shape:
            c4 = c4.expand(z4_shape).contiguous()
        targets = [loss.target for loss, _ in self.style_losses]
        losses = A.VGGLossFn.apply(input_image.contiguous(), c4, self.features(), targets)
        for k, (loss, _) in enumerate(self.style_losses):
            loss.loss = losses[k]
        self.content_losses[0][0].loss = losses[5]
        self.feature_losses[0][0].loss = losses[6]

    def _forward_generic(self, input_image, content_image, style_image):
        """Any tap layout: one pass over the pieces (no prefix re-runs)."""
        taps = {}
        for group in (self.content_losses, self.feature_losses, self.style_losses):
            for loss, idx in group:
                taps.setdefault(idx, []).append(loss)
        last = max(taps)
        if content_image is not None:
            with torch.no_grad():
                c = content_image
                for idx, piece in enumerate(self.net_pieces[:last + 1]):
                    c = piece(c)
                    for loss in taps.get(idx, []):
                        if any(loss is l for l, _ in self.content_losses + self.feature_losses):
                            loss.set_target(c)
                        elif style_image is not None:
                            loss.set_target(c)  # reference quirk (:391-394)
        x = input_image
        for idx, piece in enumerate(self.net_pieces[:last + 1]):
            x = piece(x)
            for loss in taps.get(idx, []):
                loss(x)

    # ---------------------------------------------------------------- optimisation
    def get_content_optimizer(self, input_img, optt=None):
        """stransfer/network.py:403-409 (optim.Adam -> the HIP Adam)."""
        if optt is None or optt is optim.Adam:
            optt = stx_optim.Adam
        elif optt is optim.LBFGS:
            optt = stx_optim.LBFGS
        return optt([input_img.requires_grad_()])

    def train_gatys(self, style_image: torch.Tensor, content_image: torch.Tensor, steps=550,
                    style_weight=100_000, content_weight=1) -> torch.Tensor:
        """L-BFGS Gatys optimisation from the content image (stransfer/network.py:411-458)."""
        assert isinstance(style_image, torch.Tensor), "Images need to be already loaded"
        assert isinstance(content_image, torch.Tensor), "Images need to be already loaded"
        content_image = _dev(content_image)
        if self._standard_layout() and content_image.is_cuda:
            # the fused loss engine: direction, closure and gradient statistics replayed
            # as one hipGraph per L-BFGS iteration (vgg.GatysLBFGS), torch's control flow
            targets = [l.target for l, _ in self.style_losses]
            eng = V.GatysLBFGS(self.features(), None, content_image.contiguous(),
                               style_weight, content_weight, targets=targets)

            def log(loss):  # a host float from the iteration's one read: no extra sync
                LOGGER.info("Loss: %s", loss)  # stransfer/network.py:453 logs at INFO
            for _ in tqdm(range(steps)):
                eng.step(on_eval=log)
            return eng.x.requires_grad_()
        image = content_image.clone()
        opt = self.get_content_optimizer(image, optt=optim.LBFGS)  # -> the HIP L-BFGS

        def closure():
            opt.zero_grad()
            self(image, content_image)
            total = (self.get_total_current_style_loss(weight=style_weight)
                     + self.get_total_current_content_loss(weight=content_weight))
            total.backward()
            if LOGGER.isEnabledFor(logging.INFO):  # formatting a device tensor syncs
                LOGGER.info("Loss: %s", total)  # stransfer/network.py:453
            return total

        for _ in tqdm(range(steps)):
            opt.step(closure)
        return image

    def train_gatys_adam(self, style_image, content_image, steps=500, style_weight=100_000,
                         content_weight=1, graph=True) -> torch.Tensor:
        """The Adam variant of the Gatys loop (get_content_optimizer's default
        optimiser; BASELINE.json's "Adam iters"): one hipGraph replay per iteration."""
        assert isinstance(style_image, torch.Tensor), "Images need to be already loaded"
        targets = [l.target for l, _ in self.style_losses]  # set in __init__, as the reference
        eng = V.GatysEngine(self.features(), None, _dev(content_image), style_weight,
                            content_weight, targets=targets)
        eng.run(steps, graph=graph)
        return eng.x


# ============================================================== ImageTransformNet
class ResidualBlock(nn.Module):
    """stransfer/network.py:461-506: conv-IN-ReLU-conv, + x, IN (no final ReLU)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1):
        super().__init__()
        self.conv1 = Conv2d(in_channels, out_channels, kernel_size, stride, kernel_size // 2,
                            padding_mode="reflection")
        self.insn1 = InstanceNorm2d(out_channels, affine=True)
        self.relu = ReLU()
        self.conv2 = Conv2d(out_channels, out_channels, kernel_size, stride, kernel_size // 2,
                            padding_mode="reflection")
        self.insn2 = InstanceNorm2d(out_channels, affine=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # IN + ReLU fused; (+ residual) + IN fused; each conv's bias gradient comes out of
        # the following IN's backward kernel (conv bias passed detached)
        # the skip gradient (insn2's du for x) is added inside conv1's data-gradient epilogue
        link = A.ResLink() if torch.is_grad_enabled() and x.requires_grad else None
        out = self.insn1(self.conv1(x, bias_grad=False, link=link), relu=True,
                         conv_bias=self.conv1.bias)
        return self.insn2(self.conv2(out, bias_grad=False), res=x, conv_bias=self.conv2.bias,
                          res_link=link)


def _itn_layers(in_channels=3):
    def conv(i, o, k, s, up=False):
        c = Conv2d(i, o, kernel_size=k, stride=s, padding=k // 2, padding_mode="reflection")
        c._up_input = up  # behind an Upsample (forward fuses it into the conv)
        return c

    return [
        conv(in_channels, 32, 9, 1), InstanceNorm2d(32, affine=True), ReLU(),
        conv(32, 64, 3, 2), InstanceNorm2d(64, affine=True), ReLU(),
        conv(64, 128, 3, 2), InstanceNorm2d(128, affine=True), ReLU(),
        ResidualBlock(128, 128, 3), ResidualBlock(128, 128, 3), ResidualBlock(128, 128, 3),
        ResidualBlock(128, 128, 3), ResidualBlock(128, 128, 3),
        Upsample(mode="nearest", scale_factor=2),
        conv(128, 64, 3, 1, up=True), InstanceNorm2d(64, affine=True), ReLU(),
        Upsample(mode="nearest", scale_factor=2),
        conv(64, 32, 3, 1, up=True), InstanceNorm2d(32, affine=True), ReLU(),
        conv(32, 3, 9, 1),
    ]


class ImageTransformNet(nn.Sequential):
    """Johnson et al. transform network (stransfer/network.py:509-832).  Same module
    indices / state_dict keys ('0.weight' ... '22.bias', 62 tensors).  forward fuses
    Upsample->Conv (upsampling inside the conv's halo load), Conv->IN->ReLU and the
    residual add."""

    def __init__(self, style_image: torch.Tensor, batch_size=4, in_channels=3):
        super().__init__(*_itn_layers(in_channels))
        assert isinstance(style_image, torch.Tensor), "Style image need to be already loaded"
        self.style_image = style_image
        self.batch_size = batch_size
        self.to(constants.DEVICE)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x if x.is_cuda else _dev(x)
        mods = list(self._modules.values())
        i, up = 0, False
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(m, Upsample) and isinstance(nxt, nn.Conv2d):
                up = True
                i += 1
                continue
            if isinstance(m, nn.Conv2d):
                mode = N.STX_IN_UPSAMPLE2 if up else N.STX_IN_RAW
                up = False
                if isinstance(nxt, nn.InstanceNorm2d):
                    # the IN backward produces the conv's bias gradient (sum du)
                    x = m(x, mode, bias_grad=False)
                    relu = i + 2 < len(mods) and isinstance(mods[i + 2], nn.ReLU)
                    x = nxt(x, relu=relu, conv_bias=m.bias)
                    i += 3 if relu else 2
                    continue
                x = m(x, mode)
            else:
                x = m(x)
            i += 1
        return x

    def get_total_variation_regularization_loss(self, transformed_image: torch.Tensor,
                                                regularization_factor=1e-6) -> torch.Tensor:
        """stransfer/network.py:621-641 (sum over the batch)."""
        return A.TVLossFn.apply(transformed_image, float(regularization_factor))

    def get_optimizer(self, optimizer=None):
        """stransfer/network.py:643-649."""
        if optimizer is None or optimizer is optim.Adam:
            optimizer = stx_optim.Adam
        return optimizer(self.parameters())

    # ---------------------------------------------------------------- workflows
    def static_train(self, style_name="nsp", epochs=50, style_weight=100_000, content_weight=1,
                     loaders=None, graph=True):
        """stransfer/network.py:651-770, data-parallel when launched with torchrun.

        One process per GPU (styletransfer_amd/distributed.py): `batch_size` is the
        global batch, each rank trains on its batch_size/world shard of it, the flat
        gradient is SUM-all-reduced once per step (train.FastStTrainer) and every rank
        applies the same Adam update.  Rank 0 alone logs, runs static_test and writes
        the per-epoch checkpoint.  `loaders=(test, train)` (or a callable taking the
        Shard and returning them) overrides COCO, e.g. dataset.get_synthetic_loader.
        graph=True replays each step as hipGraphs (FastStTrainer.train_step)."""
        from . import distributed as D
        from .train import FastStTrainer
        shard = D.from_env()
        dev = D.device_for(shard)
        if next(self.parameters()).device != dev:
            self.to(dev)
        main = shard.is_main
        tb_writer = (get_tensorboard_writer(f"runs/fast-image-style-transfer-still-image_{style_name}")
                     if main else _NullWriter())
        trainer = FastStTrainer(self, self.style_image.to(dev), style_weight=style_weight,
                                content_weight=content_weight, world_size=shard.world,
                                process_group=shard.group)
        loss_network = trainer.loss_network() if main else None
        if main:
            LOGGER.info('Training network with "%s" optimizer on %d data-parallel rank(s)',
                        type(trainer.opt), shard.world)
        if callable(loaders):
            loaders = loaders(shard)
        test_loader, train_loader = loaders or dataset.get_coco_loader(
            test_split=0.10, test_limit=20, batch_size=self.batch_size, shard=shard)
        iteration = 0
        if main:
            os.makedirs("data/models", exist_ok=True)
        for epoch in range(epochs):
            if main:
                LOGGER.info("Starting epoch %d", epoch)
            ckpt = f"data/models/fast_st_{style_name}_epoch{epoch}.pth"
            if os.path.isfile(ckpt):
                self.load_state_dict(adaptive_torch_load(ckpt))
                trainer.resync_params()
                continue
            sampler = getattr(train_loader, "batch_sampler", None)
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(epoch)
            for batch in tqdm(train_loader, disable=not main):
                batch = batch.squeeze(1).to(dev, torch.float32).contiguous()
                if iteration % 20 == 0:
                    # local (mean/W + TV-sum) losses summed over ranks = the global-batch loss
                    total = shard.sum_(trainer.evaluate(batch).reshape(1))[0]
                    if main:
                        tb_writer.add_scalar("data/fst_train_loss", total, iteration)
                        LOGGER.info("Batch Loss: %.8f", float(total))
                if main and iteration % 150 == 0:
                    avg = self.static_test(test_loader, loss_network)
                    tb_writer.add_scalar("data/fst_test_loss", avg, iteration)
                if main and iteration % 50 == 0:
                    with torch.no_grad():
                        img = torch.clamp(self(batch), min=0, max=255)[0]
                    tb_writer.add_image("data/fst_images",
                                        img_utils.concat_images(img.squeeze(), batch[0].squeeze()),
                                        iteration)
                iteration += 1
                trainer.train_step(batch, graph=graph)
            if main:
                torch.save(self.state_dict(), ckpt)
            shard.barrier()
        return trainer

    def static_test(self, test_loader, loss_network, style_weight=100_000, feature_weight=1):
        """stransfer/network.py:772-796."""
        losses = []
        for test_batch in test_loader:
            test_batch = _dev(test_batch.squeeze(1)).contiguous()
            with torch.no_grad():
                y = torch.clamp(self(test_batch), min=0, max=255).contiguous()
                loss_network(y, content_image=test_batch)
                s = style_weight * loss_network.get_total_current_style_loss()
                f = feature_weight * loss_network.get_total_current_feature_loss()
            losses.append(float(s + f))
        avg = torch.mean(torch.tensor(losses)) if losses else torch.tensor(float("nan"))
        LOGGER.info("Average test loss: %.8f", float(avg))
        return avg

    def process_image(self, image_path: str, style_name="nsp", out_dir="results/") -> None:
        """stransfer/network.py:798-832."""
        self.load_state_dict(_load_latest_model_weigths(model_name="fast_st",
                                                        style_name=style_name))
        image = img_utils.image_loader(os.path.join(constants.PROJECT_ROOT_PATH, image_path))
        with torch.no_grad():
            out = self(image)
        out_dir = os.path.join(constants.PROJECT_ROOT_PATH, out_dir)
        os.makedirs(out_dir, exist_ok=True)
        img_utils.imshow(out, path=os.path.join(out_dir, f"converted_fast_st_{style_name}.png"))


class VideoTransformNet(ImageTransformNet):
    """stransfer/network.py:835-1158: 6-channel first conv ([frame, previous
    stylised frame]); temporal loss (one fused HIP reduction); video_train on
    train.VideoTrainer; process_video on the graph-captured per-frame engine
    (video.py)."""

    def __init__(self, style_image: torch.Tensor, batch_size=4, fast_transfer_dict=None):
        super().__init__(style_image, batch_size)
        self[0] = Conv2d(6, 32, kernel_size=9, stride=1, padding=4,
                         padding_mode="reflection").to(constants.DEVICE)
        if fast_transfer_dict is not None:
            if isinstance(fast_transfer_dict, str):
                fast_transfer_dict = adaptive_torch_load(fast_transfer_dict)
            fast_transfer_dict = dict(fast_transfer_dict)
            del fast_transfer_dict["0.weight"]
            del fast_transfer_dict["0.bias"]
            sd = self.state_dict().copy()
            sd.update(fast_transfer_dict)
            self.load_state_dict(sd)
            self.has_external_weights = True
        else:
            self.has_external_weights = False

    def process_video(self, video_path: str, style_name="nsp", working_dir="workdir/",
                      out_dir="results/", fps=24.0):
        """stransfer/network.py:1071-1158 on the graph-captured per-frame engine
        (styletransfer_amd/video.py); frames come from imageio when installed, or from
        a directory of frames / a .npy frame array."""
        from . import video
        self.load_state_dict(_load_latest_model_weigths(model_name="video_st",
                                                        style_name=style_name))
        return video.process_video(self, video_path, style_name, working_dir, out_dir, fps)

    def get_temporal_loss(self, old_content, old_stylized, current_content, current_stylized,
                          temporal_weight=1) -> torch.Tensor:
        """||stylized - old_stylized|| / (||content - old_content|| + 1) * w
        (stransfer/network.py:885-903), differentiable in current_stylized."""
        return A.TemporalLossFn.apply(current_stylized, old_stylized, current_content,
                                      old_content, float(temporal_weight))

    def video_train(self, style_name="nsp", epochs=50, temporal_weight=0.8, style_weight=100_000,
                    feature_weight=1, content_weight=1, video_loader=None):
        """stransfer/network.py:905-1069 on train.VideoTrainer.  `video_loader`
        overrides dataset.VideoDataset(batch_size=self.batch_size) (an iterable of
        per-batch frame readers, e.g. VideoDataset(videos=[...]))."""
        from .train import VideoTrainer
        tb_writer = get_tensorboard_writer(f"runs/video-style-transfer_{style_name}")
        video_folder = f"video_samples_{style_name}/"
        shutil.rmtree(video_folder, ignore_errors=True)
        os.makedirs(video_folder, exist_ok=True)
        trainer = VideoTrainer(self, self.style_image, style_weight=style_weight,
                               content_weight=content_weight, temporal_weight=temporal_weight)
        LOGGER.info('Training video network with "%s" optimizer', type(trainer.opt_head))
        iteration = 0
        video_loader = video_loader if video_loader is not None else \
            dataset.VideoDataset(batch_size=self.batch_size)
        for epoch in range(epochs):
            if epoch == 0 and self.has_external_weights:
                LOGGER.info("Freezing weights imported from fast transfer network for the "
                            "first epoch")
                trainer.set_frozen(True)
            if epoch == 1 and self.has_external_weights:
                LOGGER.info("Unfreezing all weights")
                trainer.set_frozen(False)
            ckpt = f"data/models/video_st_{style_name}_epoch{epoch}.pth"
            if os.path.isfile(ckpt):
                self.load_state_dict(adaptive_torch_load(ckpt))
                continue
            LOGGER.info("Starting epoch %d", epoch)
            for video_batch in video_loader:
                trainer.reset_sequence()
                for batch in dataset.iterate_on_video_batches(video_batch):
                    batch = batch.to(trainer.device, torch.float32).contiguous()
                    if iteration % 20 == 0:
                        total = trainer.evaluate(batch)
                        tb_writer.add_scalar("data/fst_train_loss", total, iteration)
                        LOGGER.info("Epoch: %d\tBatch Loss: %.4f", epoch, float(total))
                    if iteration % 50 == 0 and not isinstance(tb_writer, _NullWriter):
                        old = trainer.old[1] if trainer.old is not None else batch
                        with torch.no_grad():
                            img = torch.clamp(self(torch.cat([batch, old], dim=1)), 0, 255)
                        k = min(2, img.shape[0] - 1)  # the reference logs sample 2
                        tb_writer.add_image("data/fst_images",
                                            img_utils.concat_images(img[k], batch[k]), iteration)
                    iteration += 1
                    trainer.step(batch)
            os.makedirs("data/models", exist_ok=True)
            torch.save(self.state_dict(), ckpt)
        return trainer
