"""Adam on the HIP kernel (stx_adam_step), torch.optim.Adam semantics.

Reference: `StyleNetwork.get_content_optimizer` (stransfer/network.py:403-409) and
`ImageTransformNet.get_optimizer` (:643-649) both use `optim.Adam` defaults
(lr 1e-3, betas (0.9, 0.999), eps 1e-8).  The step counter is kept on the
device so the update can live inside a captured hipGraph.
"""
from __future__ import annotations

import torch
from torch.autograd.graph import increment_version

from . import ops


def bump_versions(params):
    """In-place updates through the C ABI are invisible to autograd's version counters;
    bump them so caches keyed on `_version` (layers.Conv2d.prepped: the weight slabs)
    see the new values."""
    for p in params:
        increment_version(p)


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
                increment_version(p)
        return loss


class FlatAdam:
    """Adam over one flat parameter buffer (single launch for all tensors)."""

    def __init__(self, flat_param, flat_grad, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 params=()):
        self.p, self.g = flat_param, flat_grad
        self.params = list(params)  # the nn.Parameter views (version bumps)
        self.m = torch.zeros_like(flat_param)
        self.v = torch.zeros_like(flat_param)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=flat_param.device)
        self.ws = torch.zeros(16, dtype=torch.float32, device=flat_param.device)
        self.lr, self.betas, self.eps = lr, betas, eps

    def step(self):
        ops.adam_step(self.p, self.g, self.m, self.v, self.step_dev, self.ws, self.lr,
                      self.betas[0], self.betas[1], self.eps)
        bump_versions(self.params)


class LBFGS(torch.optim.Optimizer):
    """torch.optim.LBFGS (torch 2.10 semantics, no line search) on libstx, for
    StyleNetwork.train_gatys (stransfer/network.py:411-458:
    `optim.LBFGS([input_img.requires_grad_()])` with the defaults lr=1, max_iter=20,
    max_eval=25, tolerance_grad=1e-7, tolerance_change=1e-9, history_size=100).

    The direction is torch's two-loop recursion in its compact form (lbfgs.hip:
    stx_lbfgs_direction): the pair update, the history dots, an fp64 m x m solve, the
    combination d = -H g, g.d and x += t d are a fixed launch sequence whatever the
    history length, with the history ring, R, Y^T Y, H_diag, t and torch's n_iter in
    a device state block.  The host reads back exactly the values torch's control
    flow branches on: after the closure (loss, max|g|) and after the direction (g.d,
    max|t d|) -- two small reads per iteration, as torch's own `.item()`-style tests.
    vgg.GatysLBFGS runs the same control flow (`run`) with the direction, the VGG
    closure and the gradient statistics captured as one hipGraph per iteration (one
    host read per iteration)."""

    NSCAL = 16

    def __init__(self, params, lr=1, max_iter=20, max_eval=None, tolerance_grad=1e-7,
                 tolerance_change=1e-9, history_size=100, line_search_fn=None):
        if line_search_fn is not None:
            raise NotImplementedError("line_search_fn (the reference uses None)")
        if max_eval is None:
            max_eval = max_iter * 5 // 4
        super().__init__(params, dict(lr=lr, max_iter=max_iter, max_eval=max_eval,
                                      tolerance_grad=tolerance_grad,
                                      tolerance_change=tolerance_change,
                                      history_size=history_size, line_search_fn=None))
        if len(self.param_groups) != 1 or len(self.param_groups[0]["params"]) != 1:
            raise ValueError("LBFGS optimises one tensor (the image), as the reference")
        self._p = self.param_groups[0]["params"][0]
        self._hist = int(history_size)
        self._buf = None

    # -- device buffers -------------------------------------------------------------
    def _buffers(self, n, dev):
        if self._buf is None:
            from ._native import lib
            L = lib()
            m = self._hist
            hb, sb, wb = L.stx_lbfgs_hist_bytes(n, m), L.stx_lbfgs_state_bytes(m), \
                L.stx_lbfgs_ws(n, m)
            if not (hb and sb and wb):
                raise ValueError(f"LBFGS: history_size {m} outside 1..256")
            npad = hb // (4 * 2 * (m + 1))
            self._buf = dict(
                n=n, hist=torch.zeros(hb // 4, device=dev, dtype=torch.float32),
                state=torch.zeros(sb, device=dev, dtype=torch.uint8),
                ws=torch.zeros(wb, device=dev, dtype=torch.uint8),
                prev_g=torch.zeros(npad, device=dev, dtype=torch.float32),
                scal=torch.zeros(self.NSCAL, device=dev, dtype=torch.float32),
                loss=torch.zeros(1, device=dev, dtype=torch.float32),
                # pinned mirror of scal: one D2H copy per read, no gather kernel
                host=torch.zeros(self.NSCAL, dtype=torch.float32, pin_memory=True))
        return self._buf

    def grad_stats(self, g, loss=None, clear=None):
        """scal[0..2] = loss, max|g|, sum|g| of a fresh gradient (stx_lbfgs_grad_stats);
        loss: a device scalar (None: scal[0] untouched)."""
        from ._native import check, lib
        b = self._buf
        check(lib().stx_lbfgs_grad_stats(
            g.data_ptr(), g.numel(), None if loss is None else loss.data_ptr(),
            b["scal"].data_ptr(), None if clear is None else clear.data_ptr(),
            0 if clear is None else clear.numel(), b["ws"].data_ptr(), b["ws"].numel(),
            ops._stream()), "stx_lbfgs_grad_stats")

    def direction(self, g):
        """One torch loop iteration up to the next closure (stx_lbfgs_direction)."""
        from ._native import check, lib
        b = self._buf
        grp = self.param_groups[0]
        check(lib().stx_lbfgs_direction(
            self._p.data.view(-1).data_ptr(), g.data_ptr(), b["prev_g"].data_ptr(),
            b["hist"].data_ptr(), b["n"], self._hist, float(grp["lr"]),
            float(grp["tolerance_change"]), b["state"].data_ptr(), b["scal"].data_ptr(),
            b["ws"].data_ptr(), b["ws"].numel(), ops._stream()), "stx_lbfgs_direction")

    def _scal(self, *idx):
        """scal[idx] on the host: one async copy into the pinned mirror + a stream sync."""
        b = self._buf
        b["host"].copy_(b["scal"], non_blocking=True)
        return self._scal_host(*idx)

    def _scal_host(self, *idx):
        """scal[idx] from the pinned mirror once the current stream's work (which ends with
        the mirror copy, e.g. a captured graph's last node) is done."""
        torch.cuda.current_stream().synchronize()
        h = self._buf["host"].tolist()
        return [h[i] for i in idx]

    def _grad(self):
        g = self._p.grad
        if g is None:
            raise RuntimeError("LBFGS: the closure produced no gradient")
        if not g.is_contiguous():
            g = g.contiguous()
        return g.view(-1)

    def _eval(self, closure):
        """closure() -> (returned loss, host loss, max|g|): one host read."""
        with torch.enable_grad():
            ret = closure()
        g = self._grad()
        if torch.is_tensor(ret):
            self._buf["loss"].copy_(ret.detach().reshape(1))
            self.grad_stats(g, self._buf["loss"])
            loss, gmax = self._scal(0, 1)
        else:
            self.grad_stats(g)
            loss, gmax = float(ret), self._scal(1)[0]
        return ret, loss, gmax, g

    @torch.no_grad()
    def step(self, closure):
        if closure is None:
            raise RuntimeError("LBFGS needs a closure")
        p = self._p
        if not p.is_contiguous():
            raise RuntimeError("LBFGS: the parameter must be contiguous")
        self._buffers(p.numel(), p.device)

        def evaluate():
            return self._eval(closure)

        def move(g):
            self.direction(g)
            increment_version(p)
            gtd, t, smax, flag = self._scal(3, 4, 5, 6)
            return gtd, t, smax, bool(flag)
        return self.run(evaluate, move)

    def run(self, evaluate, move, first=None, on_eval=None):
        """torch.optim.LBFGS.step's control flow (no line search).
        evaluate() -> (returned loss, host loss, max|g|, g): a closure evaluation.
        move(g) -> (g.d, t, max|t d|, stopped): the direction and x += t d (not applied
        when stopped, i.e. g.d > -tolerance_change).
        first: an evaluation already made at the current point (GatysLBFGS) or None.
        on_eval(loss): called for every evaluation torch counts (host loss)."""
        grp = self.param_groups[0]
        max_iter, max_eval = grp["max_iter"], grp["max_eval"]
        tol_grad, tol_change = grp["tolerance_grad"], grp["tolerance_change"]
        st = self.state[self._p]
        st.setdefault("func_evals", 0)
        st.setdefault("n_iter", 0)
        orig_loss, loss, gmax, g = first if first is not None else evaluate()
        if on_eval is not None:
            on_eval(loss)
        current_evals = 1
        st["func_evals"] += 1
        if gmax <= tol_grad:
            return orig_loss
        prev_loss = st.get("prev_loss")
        n_iter = 0
        while n_iter < max_iter:
            n_iter += 1
            st["n_iter"] += 1
            prev_loss = loss
            gtd, t, smax, stopped = move(g)
            if stopped:   # gtd > -tolerance_change: torch breaks before moving x
                break
            opt_cond = False
            ls_evals = 0
            if n_iter != max_iter:
                _, loss, gmax, g = evaluate()
                if on_eval is not None:
                    on_eval(loss)
                opt_cond = gmax <= tol_grad
                ls_evals = 1
            current_evals += ls_evals
            st["func_evals"] += ls_evals
            if n_iter == max_iter or current_evals >= max_eval or opt_cond:
                break
            if smax <= tol_change:             # max|d * t|
                break
            if abs(loss - prev_loss) < tol_change:
                break
        st["prev_loss"] = prev_loss
        return orig_loss
