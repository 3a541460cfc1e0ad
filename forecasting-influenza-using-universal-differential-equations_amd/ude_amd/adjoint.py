"""``odeint_adjoint`` with torchdiffeq's signature and semantics (0.2.x ``adjoint.py``).

BASELINE configs[2] ("Dopri5 adaptive stepping + dense output + adjoint backward"); the
reference imports the solver API (lib/VAE.py:5) but never calls the adjoint, so
the specification is torchdiffeq's published algorithm:

* forward: ``odeint(func, y0, t, rtol, atol, method, options)`` without autograd -- for a UDE
  module on a HIP device the fused gfx950 dopri5 solve (csrc/ude_dopri5.h);
* backward: for i = T-1 .. 1, solve the augmented system
  ``[vjp_t, y, a_y, a_theta]`` from t[i] back to t[i-1] with the adjoint method (default: the
  forward method) and tolerances (default: the forward ones), the augmented dynamics
  ``(vjp_t, f(t, y), -a_y^T df/dy, -a_y^T df/dtheta)`` run backwards in time (torchdiffeq
  negates t and the function, ``_ReverseFunc``), with the error norm
  ``max(|vjp_t|, rms(y), rms(a_y), max_p rms(a_theta_p))`` (``default_adjoint_norm``; the
  'seminorm' option drops the parameter term); after each segment y is reset to the forward
  solution at t[i-1] and a_y receives the output cotangent there.
* the forward solve runs under no_grad, so quantities the RHS records on the side (params /
  tracker, hence posterior() / the Fa norm) carry no gradient, as in torchdiffeq.

The augmented state lives in one flat tensor (torchdiffeq's ``_TupleFunc`` flattening) stepped by
ude_amd.adaptive.eager_dopri5 or the fixed grids.  For a deterministic UDE module on a HIP device
(the adjoint parameters its own, in C-ABI order; t without gradient) the backward is fused
(``_FusedAug``): the weights are packed once, every reversed augmented evaluation
``(-vjp_t, -f, a^T df/dy, a^T df/dtheta)`` is ONE gfx950 launch (ude_rhs_eval_vjp: evaluation and
VJP, written straight into the flat derivative), and the Dormand-Prince stage / error / dense-output
combinations are single passes (ude_lincomb_hc, ude_scaled_sumsq) and the controller's scalars live on
the host (``adaptive.host_scalar_dopri5``: one read of the device error ratio / next step size per
attempt, ude_dopri_ratio).  Otherwise every augmented
evaluation calls the RHS module and ``torch.autograd.grad`` through it (for the UDE modules on a
HIP device one evaluation kernel + one VJP kernel, ude_amd/eval_rhs.py).
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from . import adaptive as _adaptive


def _rms(x: torch.Tensor) -> torch.Tensor:
    return x.abs().pow(2).mean().sqrt()


def _mixed_norm(tensors: Sequence[torch.Tensor]):
    if len(tensors) == 0:
        return 0.0
    return max([_rms(x) for x in tensors])


class _Flat:
    """Shapes of a tuple state and the flatten / split maps (torchdiffeq ``_TupleFunc``)."""

    def __init__(self, shapes: Sequence[torch.Size]):
        self.shapes = list(shapes)
        self.sizes = [int(torch.Size(s).numel()) for s in self.shapes]

    def flat(self, tensors: Sequence[torch.Tensor]) -> torch.Tensor:
        return torch.cat([x.reshape(-1) for x in tensors])

    def split(self, flat: torch.Tensor) -> List[torch.Tensor]:
        out, off = [], 0
        for s, n in zip(self.shapes, self.sizes):
            out.append(flat[off:off + n].view(s))
            off += n
        return out


def find_parameters(module) -> List[torch.Tensor]:
    return [p for p in module.parameters() if p.requires_grad]


SUMSQ_WS = 1025          # doubles per ude_scaled_sumsq output (UDE_SUMSQ_WS)


class _FusedAug:
    """The reversed augmented dynamics of a deterministic UDE module on a HIP device, fused.

    Flat state [vjp_t | y (N, R, L) | a_y (N, R, L) | a_theta (params, C-ABI order)]; its derivative
    in s = -t is [-vjp_t', -f(y), a_y^T df/dy, a_y^T df/dtheta] = ude_rhs_eval_vjp with cot = a_y and
    f scaled by -1, written into the output vector's slices by one call (the evaluation + VJP kernel and
    one tail launch).  ``comb_hc`` / ``ratio_dt`` serve adaptive.host_scalar_dopri5 (coefficients by
    value, ude_lincomb_hc; the error ratio and next step size from ude_dopri_ratio over the y / a_y pieces'
    ude_scaled_sumsq sums, the parameter pieces' RMS in PyTorch for the mixed norm); ``comb`` / ``ratio``
    are the same passes behind eager_dopri5's ``vec`` interface."""

    def __init__(self, func, y: torch.Tensor, adjoint_params, seminorm: bool):
        from . import eval_rhs
        from . import fused as _fused
        self.plan = eval_rhs._plan(eval_rhs.deterministic_config(func), y.shape[0], func.fa_weight(), y.device)
        self.lib = self.plan.lib
        self.stream = _fused._stream(y.device)
        lins = func.ude_linears()
        ws_ = [l.weight.detach().contiguous() for l in lins]
        bs_ = [l.bias.detach().contiguous() for l in lins]
        self.pack = torch.empty(self.plan.sizes.pack_bytes // 4, dtype=torch.float32, device=y.device)
        self.lib.pack(self.plan.desc, [w.data_ptr() for w in ws_], [b.data_ptr() for b in bs_], self.pack.data_ptr(),
                      self.stream)
        self.ws = torch.empty(max(self.plan.ws_bytes // 4, 1), dtype=torch.float32, device=y.device)
        self.nrl = int(y.numel())
        self.psizes = [int(p.numel()) for p in adjoint_params]
        self.seminorm = seminorm
        self.ssq = torch.empty(2 * SUMSQ_WS, dtype=torch.float64, device=y.device)
        self.status = torch.zeros(3, dtype=torch.float64, device=y.device)
        self.evals = 0

    @staticmethod
    def eligible(func, y: torch.Tensor, adjoint_params, t_requires_grad: bool) -> bool:
        from . import eval_rhs
        from .rhs import _UDEModule
        if t_requires_grad or not isinstance(func, _UDEModule) or func.uncertainty != "none":
            return False
        if not (y.is_cuda and y.dtype == torch.float32 and y.dim() == 3 and eval_rhs.eligible(func, y)):
            return False
        abi = []
        for lin in func.ude_linears():
            abi += [lin.weight, lin.bias]
        return [id(p) for p in adjoint_params] == [id(p) for p in abi]

    def __call__(self, s, yf: torch.Tensor) -> torch.Tensor:
        self.evals += 1
        out = torch.empty_like(yf)
        out[:1].zero_()
        b, ob, n = yf.data_ptr(), out.data_ptr(), self.nrl
        self.lib.rhs_eval_vjp(self.plan.desc, self.plan.prob, self.pack.data_ptr(), b + 4, b + 4 * (1 + n), ob + 4,
                              -1.0, ob + 4 * (1 + n), self.ws.data_ptr(), ob + 4 * (1 + 2 * n), self.stream)
        return out

    # comb / ratio: eager_dopri5's ``vec`` interface (device-scalar coefficients, PyTorch ratio) -- the
    # operator chain host_scalar_dopri5 is checked against bit for bit (tests/test_adjoint.py)
    def comb(self, base, ks, c) -> torch.Tensor:
        out = torch.empty_like(ks[0])
        c = c.to(torch.float32).contiguous()
        self.lib.lincomb(out.numel(), None if base is None else base.data_ptr(), [k.data_ptr() for k in ks],
                         c.data_ptr(), out.data_ptr(), self.stream)
        self._keep = c                                    # alive until the stream has read it
        return out

    def comb_hc(self, base, ks, coef) -> torch.Tensor:
        """base + sum_j coef[j] ks[j] with host (fp32) coefficients: ude_lincomb_hc."""
        out = torch.empty_like(ks[0])
        self.lib.lincomb_hc(out.numel(), None if base is None else base.data_ptr(), [k.data_ptr() for k in ks],
                            [float(c) for c in coef], out.data_ptr(), self.stream)
        return out

    def ratio_dt(self, err, y, y1, dt: float, nonfinite: torch.Tensor):
        """(error ratio, next step size, non-finite flag) of one attempt in one host read: the y / a_y
        pieces' sums of squares (ude_scaled_sumsq), the parameter pieces' RMS as ratio() forms them
        (mixed norm only), then ude_dopri_ratio."""
        n = self.nrl
        for i, off in enumerate((1, 1 + n)):
            self.lib.scaled_sumsq(n, err.data_ptr() + 4 * off, y.data_ptr() + 4 * off, y1.data_ptr() + 4 * off,
                                  self.atol, self.rtol, self.ssq.data_ptr() + 8 * i * SUMSQ_WS, self.stream)
        extra, n_extra = None, 0
        if not self.seminorm and self.psizes:
            off = 1 + 2 * n
            r = err[off:] / (self.atol + self.rtol * torch.max(y[off:].abs(), y1[off:].abs()))
            extra = torch.stack([_rms(x).double() for x in torch.split(r, self.psizes)])
            n_extra = extra.numel()
        self.lib.dopri_ratio(err.data_ptr(), y.data_ptr(), y1.data_ptr(), self.atol, self.rtol, self.ssq.data_ptr(),
                             [n, n], None if extra is None else extra.data_ptr(), n_extra, dt, nonfinite.data_ptr(),
                             self.status.data_ptr(), self.stream)
        rf, dt_next, bad = self.status.tolist()
        return rf, dt_next, bad != 0.0

    def ratio(self, err, y, y1, atol: float, rtol: float) -> torch.Tensor:
        n = self.nrl
        for i, off in enumerate((1, 1 + n)):
            self.lib.scaled_sumsq(n, err.data_ptr() + 4 * off, y.data_ptr() + 4 * off, y1.data_ptr() + 4 * off,
                                  atol, rtol, self.ssq.data_ptr() + 8 * i * SUMSQ_WS, self.stream)
        tol0 = atol + rtol * torch.max(y[:1].abs(), y1[:1].abs())
        parts = [(err[:1] / tol0).abs().reshape(()).double(),
                 (self.ssq[0] / n).sqrt(), (self.ssq[SUMSQ_WS] / n).sqrt()]
        if not self.seminorm and self.psizes:
            off = 1 + 2 * n
            r = err[off:] / (atol + rtol * torch.max(y[off:].abs(), y1[off:].abs()))
            parts += [_rms(x).double() for x in torch.split(r, self.psizes)]
        return torch.max(torch.stack(parts))


def _solve_segment(aug_func, flat: _Flat, state: List[torch.Tensor], t_from, t_to, rtol, atol, method, options,
                   norm_of_tuple, fused: "_FusedAug" = None):
    """odeint(augmented_dynamics, state, [t_from, t_to]) with t_to < t_from, returning the state
    at t_to: solved forwards in s = -t on the negated function (torchdiffeq _ReverseFunc)."""
    y0 = flat.flat(state)
    s_pair = torch.stack([-t_from, -t_to])

    def f_rev(s, yf):
        # the negated pieces written straight into one flat vector (no cat + negate pass)
        out = torch.empty_like(yf)
        for piece, view in zip(aug_func(-s, flat.split(yf)), flat.split(out)):
            torch.neg(piece.reshape(view.shape), out=view)
        return out

    opts = dict(options or {})
    if method == "dopri5" and fused is not None:
        # the fused backward: host-mirrored controller scalars, one host read per attempt
        fused.atol, fused.rtol = float(atol), float(rtol)
        sol = _adaptive.host_scalar_dopri5(fused, y0, s_pair, rtol, atol, opts.pop("first_step", None),
                                           opts.pop("max_num_steps", _adaptive.MAX_NUM_STEPS),
                                           lambda v: norm_of_tuple(flat.split(v)), fused)
    elif method == "dopri5":
        sol = _adaptive.eager_dopri5(f_rev, y0, s_pair, rtol, atol, opts.pop("first_step", None),
                                     opts.pop("max_num_steps", _adaptive.MAX_NUM_STEPS),
                                     norm=lambda v: norm_of_tuple(flat.split(v)))
    elif method in ("rk4", "euler", "midpoint"):
        from .solvers import eager_fixed_grid
        sol = eager_fixed_grid(f_rev if fused is None else fused, y0, s_pair, method, opts.pop("step_size", None))
    else:
        raise NotImplementedError(f"adjoint_method '{method}' is not implemented (dopri5 / rk4 / euler / midpoint are)")
    return flat.split(sol[1])


class _OdeintAdjoint(torch.autograd.Function):
    @staticmethod
    def forward(ctx, func, y0, t, rtol, atol, method, options, adjoint_rtol, adjoint_atol, adjoint_method,
                adjoint_options, t_requires_grad, *adjoint_params):
        from .solvers import odeint
        with torch.no_grad():
            ans = odeint(func, y0, t, rtol=rtol, atol=atol, method=method, options=options)
        ctx.func = func
        ctx.cfg = (adjoint_rtol, adjoint_atol, adjoint_method, adjoint_options, t_requires_grad)
        ctx.save_for_backward(t, ans, *adjoint_params)
        return ans

    @staticmethod
    def backward(ctx, grad_y):
        func = ctx.func
        adjoint_rtol, adjoint_atol, adjoint_method, adjoint_options, t_requires_grad = ctx.cfg
        t, y, *adjoint_params = ctx.saved_tensors
        adjoint_params = tuple(adjoint_params)
        options = dict(adjoint_options or {})
        seminorm = options.pop("norm", None) == "seminorm"

        def adjoint_norm(parts):
            vt, yy, ay, *ap = parts
            n = torch.max(torch.stack([vt.abs().reshape(()), _rms(yy), _rms(ay)]))
            if not seminorm and ap:
                n = torch.max(n, _mixed_norm(ap))
            return n

        # the RHS appends to its tracking lists on every call (lib/models.py:137, :252); the
        # augmented evaluations of the backward are not part of any loss, so their entries are
        # dropped again (thousands of (N, R, 5) tensors per backward otherwise)
        lists = [getattr(func, n) for n in ("params", "tracker") if isinstance(getattr(func, n, None), list)]
        lens = [len(x) for x in lists]

        counts = {"evals": 0}
        fused = _FusedAug(func, y[-1], adjoint_params, seminorm) \
            if _FusedAug.eligible(func, y[-1], adjoint_params, t_requires_grad) else None

        def augmented_dynamics(tt, y_aug):
            counts["evals"] += 1
            yy, adj_y = y_aug[1], y_aug[2]
            with torch.enable_grad():
                t_ = tt.detach().requires_grad_(True)
                yv = yy.detach().requires_grad_(True)
                # no gradient wrt time unless t requires it (torchdiffeq: func(t if t_requires_grad else t_, y))
                func_eval = func(t_ if t_requires_grad else tt.detach(), yv)
                grads = torch.autograd.grad(func_eval, (t_, yv) + adjoint_params, -adj_y, allow_unused=True)
            for lst, n in zip(lists, lens):
                del lst[n:]
            vjp_t, vjp_y, *vjp_params = grads
            vjp_t = torch.zeros_like(tt) if vjp_t is None else vjp_t
            vjp_y = torch.zeros_like(yy) if vjp_y is None else vjp_y
            vjp_params = [torch.zeros_like(p) if g is None else g for p, g in zip(adjoint_params, vjp_params)]
            return [vjp_t.reshape(()).to(yy.dtype), func_eval.detach(), vjp_y.detach()] + \
                [g.detach() for g in vjp_params]

        with torch.no_grad():
            zero = torch.zeros((), dtype=y.dtype, device=y.device)
            aug_state = [zero, y[-1], grad_y[-1]] + [torch.zeros_like(p) for p in adjoint_params]
            flat = _Flat([a.shape for a in aug_state])
            time_vjps = torch.empty(len(t), dtype=t.dtype, device=t.device) if t_requires_grad else None
            for i in range(len(t) - 1, 0, -1):
                if t_requires_grad:
                    fe = func(t[i], y[i])
                    dLd_cur_t = fe.reshape(-1).dot(grad_y[i].reshape(-1))
                    aug_state[0] = aug_state[0] - dLd_cur_t
                    time_vjps[i] = dLd_cur_t
                aug_state = list(_solve_segment(augmented_dynamics, flat, aug_state, t[i], t[i - 1], adjoint_rtol,
                                                adjoint_atol, adjoint_method, options, adjoint_norm, fused))
                aug_state[1] = y[i - 1]
                aug_state[2] = aug_state[2] + grad_y[i - 1]
            if t_requires_grad:
                # aug_state[0] already is dL/dt0: -sum_i g_i . f(t_i, y_i) carried back through the
                # vjp_t dynamics (torchdiffeq: time_vjps[0] = aug_state[0], no negation)
                time_vjps[0] = aug_state[0]
        try:
            func.last_adjoint_info = {"augmented_evals": counts["evals"] + (fused.evals if fused else 0),
                                      "seminorm": seminorm, "fused": fused is not None}
        except AttributeError:
            pass
        adj_y = aug_state[2]
        adj_params = aug_state[3:]
        return (None, adj_y, time_vjps, None, None, None, None, None, None, None, None, None, *adj_params)


def odeint_adjoint(func, y0, t, *, rtol=1e-7, atol=1e-9, method=None, options=None, event_fn=None,
                   adjoint_rtol=None, adjoint_atol=None, adjoint_method=None, adjoint_options=None,
                   adjoint_params=None):
    """torchdiffeq.odeint_adjoint (tensor y0; no events)."""
    if event_fn is not None:
        raise NotImplementedError("event handling is not supported")
    if not isinstance(func, torch.nn.Module) and adjoint_params is None:
        raise ValueError("func must be an instance of nn.Module to specify the adjoint parameters; "
                         "alternatively they can be specified explicitly via the `adjoint_params` argument.")
    method = "dopri5" if method is None else method
    adjoint_params = tuple(find_parameters(func)) if adjoint_params is None else tuple(adjoint_params)
    adjoint_params = tuple(p for p in adjoint_params if p.requires_grad)
    adjoint_rtol = rtol if adjoint_rtol is None else adjoint_rtol
    adjoint_atol = atol if adjoint_atol is None else adjoint_atol
    if adjoint_method is None:
        adjoint_method = method
    if adjoint_options is None:
        adjoint_options = {k: v for k, v in (options or {}).items() if k != "norm"} \
            if adjoint_method == method else {}
    return _OdeintAdjoint.apply(func, y0, t, rtol, atol, method, options, adjoint_rtol, adjoint_atol,
                                adjoint_method, adjoint_options, bool(t.requires_grad), *adjoint_params)
