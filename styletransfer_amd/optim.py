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
    """torch.optim.LBFGS (torch 2.10 semantics, no line search) on libstx vector
    kernels, for StyleNetwork.train_gatys (stransfer/network.py:411-458:
    `optim.LBFGS([input_img.requires_grad_()])` with the defaults lr=1, max_iter=20,
    max_eval=25, tolerance_grad=1e-7, tolerance_change=1e-9, history_size=100).

    Every vector operation (dot products, the two-loop recursion, the parameter
    update) is a HIP kernel (stx_vec_reduce / stx_vec_axpby); the 0-d quantities
    torch keeps as device tensors (ys, rho_i, alpha_i, H_diag, the step size t) stay
    in one device scalar array, so the recursion runs without host round trips.
    The host reads back exactly the values torch's control flow branches on
    (ys > 1e-10, g.d, max|g|, max|t d|, the closure's loss)."""

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
        self._hist = history_size
        # scalar array: 0 ys, 1 yy, 2 H_diag, 3 t, 4 gtd, 5 reduction tmp, 6 coef,
        # 7 lr, 8 zero, 9 one; rho_k at 16+k, alpha_k at 16+hist+k (ring slots k)
        self._S = None

    # -- kernels ----------------------------------------------------------------
    def _axpby(self, y, x, a=1.0, a_dev=None, sgn=1.0, b=0.0):
        from ._native import check, lib
        check(lib().stx_vec_axpby(y.data_ptr(), None if x is None else x.data_ptr(), y.numel(),
                                  float(a), a_dev, float(sgn), float(b), ops._stream()),
              "stx_vec_axpby")

    def _red(self, a, b, op, out, mul=None, add=None, sgn=1.0):
        from ._native import check, lib
        L = lib()
        wp, wn = ops.WS.get(L.stx_vec_ws(), a.device)
        check(L.stx_vec_reduce(a.data_ptr(), None if b is None else b.data_ptr(), a.numel(), op,
                               out, mul, add, float(sgn), wp, wn, ops._stream()),
              "stx_vec_reduce")

    def _sc(self, op, i, j, k):
        from ._native import check, lib
        check(lib().stx_scalar_op(self._S.data_ptr(), op, i, j, k, ops._stream()),
              "stx_scalar_op")

    def _sp(self, i):
        """device pointer of scalar slot i"""
        return self._S.data_ptr() + 4 * i

    def _host(self, i):
        return float(self._S[i])

    def _hosts(self, *idx):
        """Several scalar slots in one device->host read."""
        return self._S[list(idx)].tolist()

    def _loss_slot(self, loss, i=10):
        """Park the closure's loss in slot i (device copy, no sync); returns a thunk
        for python-number losses, which have no device value."""
        if torch.is_tensor(loss):
            self._S[i:i + 1].copy_(loss.detach().reshape(1))
            return None
        return float(loss)

    def _grad(self):
        g = self._p.grad
        if g is None:
            raise RuntimeError("LBFGS: the closure produced no gradient")
        if not g.is_contiguous():
            g = g.contiguous()
        return g.view(-1)

    @torch.no_grad()
    def step(self, closure):
        if closure is None:
            raise RuntimeError("LBFGS needs a closure")
        group = self.param_groups[0]
        lr, max_iter, max_eval = group["lr"], group["max_iter"], group["max_eval"]
        tol_grad, tol_change = group["tolerance_grad"], group["tolerance_change"]
        H = self._hist
        p = self._p
        dev = p.device
        if self._S is None:
            self._S = torch.zeros(16 + 2 * H, device=dev, dtype=torch.float32)
            self._S[7] = float(lr)
            self._S[9] = 1.0
        st = self.state[p]
        st.setdefault("func_evals", 0)
        st.setdefault("n_iter", 0)
        with torch.enable_grad():
            orig_loss = closure()
        hl = self._loss_slot(orig_loss)
        current_evals = 1
        st["func_evals"] += 1
        g = self._grad()
        n = g.numel()
        self._red(g, None, 2, self._sp(11))
        loss, gmax = self._hosts(10, 11)                  # one sync: loss, max|g|
        loss = loss if hl is None else hl
        if gmax <= tol_grad:
            return orig_loss
        d = st.get("d")
        prev_g = st.get("prev_flat_grad")
        prev_loss = st.get("prev_loss")
        dirs, stps, slots = st.get("old_dirs"), st.get("old_stps"), st.get("slots")
        t_host = st.get("t_host")
        n_iter = 0
        while n_iter < max_iter:
            n_iter += 1
            st["n_iter"] += 1
            if st["n_iter"] == 1:
                d = torch.empty(n, device=dev, dtype=torch.float32)
                self._axpby(d, g, -1.0)
                dirs, stps, slots = [], [], []
                self._sc(3, 9, 8, 2)  # H_diag = 1
            else:
                y = torch.empty_like(g)
                s = torch.empty_like(g)
                self._axpby(y, g)
                self._axpby(y, prev_g, -1.0, b=1.0)          # y = g - prev_g
                self._axpby(s, d, 1.0, self._sp(3))           # s = d * t
                self._red(y, s, 0, self._sp(0))               # ys
                if self._host(0) > 1e-10:
                    if len(dirs) == H:
                        dirs.pop(0)
                        stps.pop(0)
                        k = slots.pop(0)
                    else:
                        k = len(slots)
                    dirs.append(y)
                    stps.append(s)
                    slots.append(k)
                    self._sc(4, 0, -1, 16 + k)                 # rho_k = 1 / ys
                    self._red(y, y, 0, self._sp(1))           # yy
                    self._sc(0, 0, 1, 2)                       # H_diag = ys / yy
                # two-loop recursion, all scalars on the device
                q = torch.empty_like(g)
                self._axpby(q, g, -1.0)
                for i in range(len(dirs) - 1, -1, -1):
                    k = slots[i]
                    self._red(stps[i], q, 0, self._sp(16 + H + k), mul=self._sp(16 + k))
                    self._axpby(q, dirs[i], 1.0, self._sp(16 + H + k), sgn=-1.0, b=1.0)
                d = torch.empty_like(g)
                self._axpby(d, q, 1.0, self._sp(2))           # d = r = q * H_diag
                for i in range(len(dirs)):
                    k = slots[i]
                    # coef = alpha_i - rho_i * (dirs_i . r)
                    self._red(dirs[i], d, 0, self._sp(6), mul=self._sp(16 + k),
                              add=self._sp(16 + H + k), sgn=-1.0)
                    self._axpby(d, stps[i], 1.0, self._sp(6), b=1.0)
            if prev_g is None:
                prev_g = torch.empty_like(g)
            self._axpby(prev_g, g)
            prev_loss = loss
            if st["n_iter"] == 1:
                self._red(g, None, 1, self._sp(5))             # sum |g|
                self._sc(5, 5, 9, 3)                           # t = min(1, 1/sum|g|)
                self._sc(1, 3, 7, 3)                           # t *= lr
            else:
                self._sc(3, 7, 8, 3)                           # t = lr
            self._red(g, d, 0, self._sp(4))                    # gtd
            t_host, gtd = self._hosts(3, 4)                    # one sync: t, g.d
            if gtd > -tol_change:
                break
            ls_evals = 0
            self._axpby(p.data.view(-1), d, 1.0, self._sp(3), b=1.0)   # x += t d
            increment_version(p)
            opt_cond = False
            self._red(d, None, 2, self._sp(12))                # max|d| (for the last test)
            dmax = None
            if n_iter != max_iter:
                with torch.enable_grad():
                    hl = self._loss_slot(closure())
                g = self._grad()
                self._red(g, None, 2, self._sp(11))
                loss, gmax, dmax = self._hosts(10, 11, 12)     # one sync: loss, max|g|, max|d|
                loss = loss if hl is None else hl
                opt_cond = gmax <= tol_grad
                ls_evals = 1
            current_evals += ls_evals
            st["func_evals"] += ls_evals
            if n_iter == max_iter or current_evals >= max_eval or opt_cond:
                break
            if dmax is None:
                dmax = self._host(12)
            if abs(t_host) * dmax <= tol_change:               # max|d * t|
                break
            if abs(loss - prev_loss) < tol_change:
                break
        st.update(d=d, prev_flat_grad=prev_g, prev_loss=prev_loss, old_dirs=dirs,
                  old_stps=stps, slots=slots, t_host=t_host)
        return orig_loss
