"""fast_st training step on libstx, single GPU or data-parallel over RCCL.

One step = the `static_train` closure + `optimizer.step` of the reference
(stransfer/network.py:690-731, :765):

    y = itn(batch); loss_network(y, content_image=batch)
    total = style_weight*sum(style) + content_weight*content + TV(y); total.backward(); adam

Parameters and gradients of the ImageTransformNet live in ONE flat fp32 buffer
each (the nn.Parameters are views), so the data-parallel exchange is a single
RCCL all-reduce of 1,679,235 floats per step and Adam is a single kernel.

Data-parallel scaling trap: style/content are batch MEANS, TV is
a batch SUM.  With the global batch split into W equal shards, the gradient of
the single-device loss equals SUM over ranks of the gradient of
    (style_weight*style_r + content_weight*content_r) / W + TV_r,
which is what each rank back-propagates before the SUM all-reduce.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import ops
from . import autograd as A
from . import constants
from . import vgg as V
from .optim import FlatAdam, bump_versions


def flatten_parameters(module: torch.nn.Module, device):
    """Re-home every parameter (and its .grad) as a view of one flat buffer."""
    params = [p for p in module.parameters()]
    total = sum(p.numel() for p in params)
    flat = torch.empty(total, device=device, dtype=torch.float32)
    grad = torch.zeros(total, device=device, dtype=torch.float32)
    o = 0
    for p in params:
        n = p.numel()
        flat[o:o + n].copy_(p.data.reshape(-1))
        p.data = flat[o:o + n].view_as(p)
        p.grad = grad[o:o + n].view_as(p)
        o += n
    return flat, grad


class FastStTrainer:
    def __init__(self, itn, style_image, style_weight=100_000, content_weight=1, lr=1e-3,
                 world_size=1, process_group=None, vgg_weights=None, tv_factor=1e-6):
        dev = constants.DEVICE if not isinstance(style_image, torch.Tensor) or \
            not style_image.is_cuda else style_image.device
        self.itn = itn
        self.device = torch.device(dev)
        self.feat = V.VGGFeatures(V.load_vgg19_weights(vgg_weights), self.device)
        style = style_image.to(self.device, torch.float32)
        if style.dim() == 3:
            style = style.unsqueeze(0)
        self.style_image = style
        self.targets = self.feat.style_targets(style)
        self.sw, self.cw, self.tv = float(style_weight), float(content_weight), float(tv_factor)
        self.world = int(world_size)
        self.pg = process_group
        self.exchanges = 0  # flat-gradient all-reduces issued
        self.flat, self.flat_grad = flatten_parameters(itn, self.device)
        self.params = list(itn.parameters())
        if self.world > 1:
            # replicas must start identical (e.g. static_train's default torch init is
            # drawn independently per process): rank 0's parameters win
            dist.broadcast(self.flat, src=self._src(), group=self.pg)
            bump_versions(self.params)
        self.opt = FlatAdam(self.flat, self.flat_grad, lr=lr, params=self.params)
        # the backward's seed gradient d total / d total = 1, allocated once (autograd's
        # default seed is a fill launch per step)
        self._one = torch.ones((), device=self.device, dtype=torch.float32)
        self.vgg_weights = vgg_weights
        self._graph = None  # (replay, static batch, static loss) of train_step
        from .layers import Conv2d
        # every conv slab of the ITN re-prepped in two launches per step
        self.slabs = ops.TrainedSlabs(m for m in itn.modules() if isinstance(m, Conv2d))

    def _src(self):
        """Global rank of the group's rank 0."""
        if self.pg is None:
            return 0
        return dist.get_global_rank(self.pg, 0)

    def _param_ptrs(self):
        return tuple(p.data_ptr() for p in self.params) + (self.slabs.generation,)

    def resync_params(self):
        """No-op: load_state_dict copies into the flat views in place."""

    def loss_network(self):
        """A StyleNetwork (reference API) with the same VGG weights and style targets,
        for static_test (stransfer/network.py:661-663)."""
        from .network import StyleNetwork
        return StyleNetwork(self.style_image, torch.rand([1, 3, 256, 256]),
                            vgg_weights=self.vgg_weights)

    def _total(self, batch, y):
        with torch.no_grad():
            c4 = V.content_target(self.feat, batch, amax=ops.ARENA.take_span(5, batch.device))
        w = self.world
        if torch.is_grad_enabled() and y.requires_grad:
            # one fused scalar: folded loss weights, TV value + gradient in one pass
            return A.FastStLossFn.apply(y, c4, self.feat, self.targets, self.sw / w,
                                        self.cw / w, self.tv)
        losses = A.VGGLossFn.apply(y, c4, self.feat, self.targets, False)  # feature loss unused
        tv = A.TVLossFn.apply(y, self.tv)
        return (self.sw / w) * losses[:5].sum() + (self.cw / w) * losses[5] + tv

    def _fwd_bwd(self, batch: torch.Tensor) -> torch.Tensor:
        """Local loss and gradient (into flat_grad) of one batch."""
        self.flat_grad.zero_()
        self.slabs.prep()
        ops.ARENA.begin(self.device)  # InstanceNorm outputs carry their max|.| to the convs
        ops.PGRADS.begin()            # one launch for all InstanceNorm parameter gradients
        ops.SIDE.begin(self.device)   # weight gradients on a side stream
        try:
            y = self.itn(batch)
            total = self._total(batch, y)
            total.backward(self._one)
            ops.PGRADS.flush()
        finally:
            ops.SIDE.end()
            ops.PGRADS.active = False
            ops.ARENA.end()
        return total.detach()

    def _exchange(self):
        # an explicit process group forces the exchange even at world 1 (the RCCL path
        # exercised on one GPU: a 1-rank SUM is the identity)
        if self.world > 1 or self.pg is not None:
            dist.all_reduce(self.flat_grad, op=dist.ReduceOp.SUM, group=self.pg)
            self.exchanges += 1

    def step(self, batch: torch.Tensor) -> torch.Tensor:
        batch = batch.to(self.device, torch.float32).contiguous()
        total = self._fwd_bwd(batch)
        self._exchange()
        self.opt.step()
        return total

    def capture(self, batch: torch.Tensor, warmup: int = 1):
        """Capture the training step into hipGraphs over a static copy of `batch` --
        the fast_st analogue of vgg.GatysEngine's per-iteration graph: the ~240
        launches of a step replay without per-op host work.  Two graphs: (zero grad,
        ITN forward, VGG losses, backward) and the flat Adam update; the RCCL
        all-reduce of the flat gradient (world > 1) runs eagerly between them, so no
        collective is ever captured.  `warmup` eager steps run first (they train like
        any step and size every workspace).  Returns (replay, static_batch,
        static_loss): copy the next batch into static_batch, then call replay()."""
        static = batch.to(self.device, torch.float32).contiguous().clone()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self.warmup_loss = self.step(static)
        torch.cuda.current_stream(self.device).wait_stream(side)
        g_fb, g_up = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        # thread_local: a process-group watchdog thread may query its events meanwhile
        with ops.graph_capture(g_fb, capture_error_mode="thread_local"):
            loss = self._fwd_bwd(static)
        with ops.graph_capture(g_up, pool=g_fb.pool(), capture_error_mode="thread_local"):
            self.opt.step()
        ptrs = self._param_ptrs()
        # every older graph refuses to replay (pointer check below): the slabs of
        # earlier generations are dead
        self.slabs.release_retired()

        def replay():
            if self._param_ptrs() != ptrs:
                # the graphs hold the captured parameter, gradient and slab pointers
                raise RuntimeError("FastStTrainer: parameters were re-homed after capture(); "
                                   "capture again")
            g_fb.replay()
            self._exchange()
            g_up.replay()
            bump_versions(self.params)  # the graph's Adam is invisible to autograd
        return replay, static, loss

    def train_step(self, batch: torch.Tensor, graph: bool = True) -> torch.Tensor:
        """step() for a stream of batches: the first batch of a shape is trained by the
        capture's warm-up step (eager) and the step is captured; every later batch of
        that shape is copied into the static input and replayed.  Other shapes (a
        short last batch) run eagerly.  Returns the local loss (device tensor; a
        view of the graph's static output on replays)."""
        batch = batch.to(self.device, torch.float32).contiguous()
        if not graph:
            return self.step(batch)
        if self._graph is not None and self._graph[3] != self._param_ptrs():
            self._graph = None  # parameters re-homed: the captured pointers are stale
        if self._graph is None:
            self._graph = self.capture(batch, warmup=1) + (self._param_ptrs(),)
            return self.warmup_loss
        replay, static, loss, _ = self._graph
        if static.shape != batch.shape:
            return self.step(batch)
        static.copy_(batch)
        replay()
        return loss

    @torch.no_grad()
    def evaluate(self, batch: torch.Tensor) -> torch.Tensor:
        batch = batch.to(self.device, torch.float32).contiguous()
        return self._total(batch, self.itn(batch))


class VideoTrainer(FastStTrainer):
    """One `video_train` step of VideoTransformNet (stransfer/network.py:905-1069):

        y = net(cat([batch, old_stylised], dim=1))
        total = style_weight*style + content_weight*content + TV(y)
                + ||y - old_stylised|| / (||batch - old_content|| + 1) * temporal_weight
        total.backward(); Adam;  (old_content, old_stylised) <- (batch, y)

    on the same flat-buffer machinery as FastStTrainer (the temporal term is one
    fused HIP reduction, autograd.TemporalLossFn).  A new video batch starts with
    old = (batch, batch) (reset_sequence).  The reference freezes every parameter
    but the first conv's during epoch 0 when it starts from fast_st weights: Adam
    then keeps no state for the frozen tensors, so here the flat buffers are split
    into two Adam instances (the 6-channel head conv, the rest) whose step counters
    advance independently -- the same bias correction as torch's per-parameter
    state."""

    def __init__(self, net, style_image, style_weight=100_000, content_weight=1,
                 temporal_weight=0.8, lr=1e-3, vgg_weights=None, tv_factor=1e-6):
        super().__init__(net, style_image, style_weight=style_weight,
                         content_weight=content_weight, lr=lr, vgg_weights=vgg_weights,
                         tv_factor=tv_factor)
        self.tw = float(temporal_weight)
        head = [net[0].weight, net[0].bias]
        assert all(a is b for a, b in zip(head, self.params[:2])), "first conv must lead"
        n0 = sum(p.numel() for p in head)
        self.opt_head = FlatAdam(self.flat[:n0], self.flat_grad[:n0], lr=lr, params=head)
        self.opt_rest = FlatAdam(self.flat[n0:], self.flat_grad[n0:], lr=lr,
                                 params=self.params[2:])
        self.frozen = False
        self.old = None

    def set_frozen(self, frozen: bool):
        """Freeze (requires_grad=False, no Adam step) every parameter but the head's."""
        self.frozen = bool(frozen)
        for name, p in self.itn.named_parameters():
            if not name.startswith("0."):
                p.requires_grad = not self.frozen

    def reset_sequence(self):
        self.old = None

    def _video_total(self, batch, y, old_c, old_s):
        return self._total(batch, y) + A.TemporalLossFn.apply(y, old_s, batch, old_c, self.tw)

    def _inputs(self, batch):
        batch = batch.to(self.device, torch.float32).contiguous()
        old_c, old_s = self.old if self.old is not None else (batch, batch)
        return batch, old_c, old_s, torch.cat([batch, old_s], dim=1)

    def step(self, batch: torch.Tensor) -> torch.Tensor:
        batch, old_c, old_s, x6 = self._inputs(batch)
        self.flat_grad.zero_()
        self.slabs.prep()
        ops.ARENA.begin(self.device)
        ops.PGRADS.begin()
        ops.SIDE.begin(self.device)
        try:
            y = self.itn(x6)
            total = self._video_total(batch, y, old_c, old_s)
            total.backward(self._one)
            ops.PGRADS.flush()
        finally:
            ops.SIDE.end()
            ops.PGRADS.active = False
            ops.ARENA.end()
        self.old = (batch, y.detach())
        self.opt_head.step()
        if not self.frozen:
            self.opt_rest.step()
        return total.detach()

    @torch.no_grad()
    def evaluate(self, batch: torch.Tensor) -> torch.Tensor:
        """The closure's loss for `batch` without a step (the sequence is unchanged)."""
        batch, old_c, old_s, x6 = self._inputs(batch)
        return self._video_total(batch, self.itn(x6), old_c, old_s)
