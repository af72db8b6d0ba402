"""Adam on the HIP kernel (stx_adam_step), torch.optim.Adam semantics.

Reference: `StyleNetwork.get_content_optimizer` (stransfer/network.py:403-409) and
`ImageTransformNet.get_optimizer` (:643-649) both use `optim.Adam` defaults
(lr 1e-3, betas (0.9, 0.999), eps 1e-8).  The step counter is kept on the
device so the update can live inside a captured hipGraph.
"""
from __future__ import annotations

import torch

from . import ops


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False):
        if weight_decay != 0 or amsgrad:
            raise NotImplementedError("weight_decay / amsgrad (unused by the reference)")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0,
                                      amsgrad=False))

    def _state(self, p):
        st = self.state[p]
        if not st:
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["step_dev"] = torch.zeros(1, dtype=torch.int32, device=p.device)
            st["ws"] = torch.zeros(16, dtype=torch.float32, device=p.device)
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_contiguous() or not p.grad.is_contiguous():
                    raise RuntimeError("stx Adam needs contiguous params/grads")
                st = self._state(p)
                ops.adam_step(p, p.grad, st["exp_avg"], st["exp_avg_sq"], st["step_dev"],
                              st["ws"], group["lr"], b1, b2, group["eps"])
        return loss


class FlatAdam:
    """Adam over one flat parameter buffer (single launch for all tensors)."""

    def __init__(self, flat_param, flat_grad, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.p, self.g = flat_param, flat_grad
        self.m = torch.zeros_like(flat_param)
        self.v = torch.zeros_like(flat_param)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=flat_param.device)
        self.ws = torch.zeros(16, dtype=torch.float32, device=flat_param.device)
        self.lr, self.betas, self.eps = lr, betas, eps

    def step(self):
        ops.adam_step(self.p, self.g, self.m, self.v, self.step_dev, self.ws, self.lr,
                      self.betas[0], self.betas[1], self.eps)
