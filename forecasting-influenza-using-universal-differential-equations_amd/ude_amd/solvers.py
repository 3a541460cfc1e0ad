"""``odeint`` with torchdiffeq's signature (the reference's solver API).

``odeint(func, y0, t, *, rtol=1e-7, atol=1e-9, method=None, options=None,
event_fn=None)`` as imported by lib/VAE.py:5 and run_ode.py:24 and called as
``odeint(ode, z, t, method='rk4', options=dict(step_size=h))``
(lib/VAE.py:137, tuning/tune_encoders.py:221, tuning/tune_node.py:204).

Dispatch:
* ``method='rk4'`` + an RHS of this package (Fp / Fa / FaFp, and the
  Bayes_* classes of lib/in_development/models_bayes.py at the sizes the
  kernels hold) + fp32 state on a HIP device  ->  the fused gfx950 kernel
  (forward + VJP), no fallback: a missing or unloadable library raises;
* anything else (other callables, CPU tensors, fixed-grid 'euler' /
  'midpoint' / 'rk4', Bayesian models too large for the whole-solve kernel)  ->  the
  generic step-by-step solver below, which calls ``func`` once per stage exactly as
  torchdiffeq does; a UDE module on a HIP device then evaluates on the gfx950
  evaluation + VJP kernels (ude_amd/eval_rhs.py).  ``UDE_STRICT=1`` makes a UDE module
  whose evaluations would run as PyTorch operators raise instead.
``method='dopri5'`` (torchdiffeq's default): the fused gfx950 adaptive solve for
a UDE module without autograd (ude_amd/adaptive.py, csrc/ude_dopri5.h), else the
differentiable step-by-step restatement (its evaluations on the gfx950 evaluation
kernels for a UDE module on a HIP device).  ``odeint_adjoint``: ude_amd/adjoint.py.
Other adaptive methods raise NotImplementedError.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Optional

import torch

from .rhs import _UDEModule
from .schedule import build_schedule, fixed_grid
from . import fused as _fused
from . import _native
from . import adaptive as _adaptive

FIXED_METHODS = ("rk4", "euler", "midpoint")
ADAPTIVE_METHODS = ("dopri8", "dopri5", "bosh3", "fehlberg2", "adaptive_heun", "explicit_adams",
                    "implicit_adams", "fixed_adams", "scipy_solver")
ONE_THIRD = 1.0 / 3.0
TWO_THIRDS = 2.0 / 3.0


def _check_t(t: torch.Tensor) -> None:
    if not torch.is_tensor(t):
        raise TypeError("t must be a torch.Tensor")
    if t.dim() != 1:
        raise AssertionError("t must be one dimensional")
    if not torch.is_floating_point(t):
        raise TypeError("t must be a floating point Tensor")
    if len(t) > 1 and not bool((t[1:] > t[:-1]).all()):
        raise AssertionError("t must be strictly increasing")


def _needs_grad(func, y0: torch.Tensor) -> bool:
    return torch.is_grad_enabled() and (y0.requires_grad or any(p.requires_grad for p in func.parameters()))


def _strict() -> bool:
    return os.environ.get("UDE_STRICT", "0") == "1"


def _eval_fused(func, y0: torch.Tensor) -> bool:
    """Whether each evaluation of a step-by-step solve runs on the gfx950 evaluation kernels
    (ude_amd/eval_rhs.py) -- the module's forward on a HIP device."""
    from . import eval_rhs
    return bool(getattr(func, "fused_eval", False)) and eval_rhs.eligible(func, y0)


def fusable(func, y0: torch.Tensor) -> bool:
    if not (isinstance(func, _UDEModule) and y0.is_cuda
            and y0.dtype == torch.float32 and y0.dim() == 3
            and y0.shape[1] == func.n_regions and y0.shape[2] == func.latent_dim
            and all(p.is_cuda and p.dtype == torch.float32 for p in func.parameters())):
        return False
    if func.uncertainty == "bayes":
        # the Bayesian kernels hold two dW accumulator sets in registers: the models
        # that fit are compiled (R = 1 at the reference's sizes; see Model::FITS)
        return _native.config_supported(func.ude_config())
    return func.uncertainty == "none"


# Host-side caches so that a training loop calling odeint with the same time grid
# does not round-trip t through the host (and re-upload the schedule) every call.
# t is keyed by identity + in-place version (a strong reference is kept, so the id
# cannot be reused while cached); plans by the grid's values.
_T_CACHE: "OrderedDict" = OrderedDict()
_PLAN_CACHE: "OrderedDict" = OrderedDict()
_CACHE_MAX = 16


def _lru_put(cache, key, value):
    cache[key] = value
    cache.move_to_end(key)
    while len(cache) > _CACHE_MAX:
        cache.popitem(last=False)


def _host_t(t: torch.Tensor) -> torch.Tensor:
    """Validated host copy of t (torchdiffeq's checks), cached per tensor version."""
    key = (id(t), t._version)
    hit = _T_CACHE.get(key)
    if hit is not None and hit[0] is t:
        return hit[1]
    host = t.detach().cpu()
    _check_t(host)
    _lru_put(_T_CACHE, key, (t, host))
    return host


def plan_for(func: _UDEModule, y0: torch.Tensor, t: torch.Tensor, step_size=None) -> "_fused.Plan":
    """The cached launch plan (schedule on the device, buffer sizes) of a fused solve."""
    th = _host_t(t)
    if isinstance(step_size, torch.Tensor):
        step_size = step_size.detach().cpu()
    step_key = None if step_size is None else (
        step_size.to(th.dtype).numpy().tobytes() if isinstance(step_size, torch.Tensor) else float(step_size))
    bayes = func.uncertainty == "bayes"
    if bayes:
        mus, _ = func.ude_mean_std()
        shapes = [p.shape for p in mus]
    else:
        shapes = func.ude_weight_shapes()
    cfg = func.ude_config()
    fa_w = func.fa_weight()
    key = (cfg, str(th.dtype), th.numpy().tobytes(), step_key, int(y0.shape[0]), float(fa_w), str(y0.device),
           tuple(tuple(s) for s in shapes))
    plan = _PLAN_CACHE.get(key)
    if plan is None:
        sched = build_schedule(th, step_size)
        plan = _fused.make_plan(cfg, sched, y0.shape[0], fa_w, y0.device, list(shapes))
        _lru_put(_PLAN_CACHE, key, plan)
    else:
        _PLAN_CACHE.move_to_end(key)
    return plan


def fused_odeint(func: _UDEModule, y0: torch.Tensor, t: torch.Tensor, step_size=None) -> torch.Tensor:
    plan = plan_for(func, y0, t, step_size)
    if func.uncertainty == "bayes":
        mus, sds = func.ude_mean_std()
        n_par = sum(int(p.numel()) for p in mus)
        eps = func.take_eps(4 * plan.prob.n_steps, n_par, y0.device)
        keep = bool(func.materialize_tracking)
        latent, mean, std, fa_norm, ckpt, sums = _fused.FusedBayesRK4.apply(plan, y0.contiguous(), eps, keep,
                                                                            *(mus + sds))
        stats = (mean, std, fa_norm)
        evals = func._evals_from_checkpoint(ckpt, y0, plan.prob.n_steps, eps) if keep else None
        func._record_fused(stats, plan.n_eval, evals, sums=sums)
    else:
        params = []
        for lin in func.ude_linears():
            params += [lin.weight, lin.bias]
        keep = bool(func.materialize_tracking)
        latent, mean, std, fa_norm, ckpt, sir_token, sums = _fused.FusedRK4.apply(plan, y0.contiguous(), keep,
                                                                                  *params)
        stats = (mean, std, fa_norm)
        latent._ude_sir_token = sir_token
        evals = func._evals_from_checkpoint(ckpt, y0, plan.prob.n_steps) if keep else None
        func._record_fused(stats, plan.n_eval, evals, sums=sums)
    return latent


def _step_rk4(func, t0, dt, t1, y):
    k1 = func(t0, y)
    k2 = func(t0 + dt * ONE_THIRD, y + dt * k1 * ONE_THIRD)
    k3 = func(t0 + dt * TWO_THIRDS, y + dt * (k2 - k1 * ONE_THIRD))
    k4 = func(t1, y + dt * (k1 - k2 + k3))
    return (k1 + 3 * (k2 + k3) + k4) * dt * 0.125


def _step_euler(func, t0, dt, t1, y):
    return dt * func(t0, y)


def _step_midpoint(func, t0, dt, t1, y):
    half = 0.5 * dt
    return dt * func(t0 + half, y + func(t0, y) * half)


_STEPS = {"rk4": _step_rk4, "euler": _step_euler, "midpoint": _step_midpoint}
_STAGES = {"rk4": 4, "euler": 1, "midpoint": 2}


def eager_fixed_grid(func, y0, t, method="rk4", step_size=None):
    step = _STEPS[method]
    grid = fixed_grid(t, step_size).to(y0.device)
    tt = t.to(y0.device)
    out = [y0]
    j = 1
    y = y0
    for n in range(len(grid) - 1):
        t0, t1 = grid[n], grid[n + 1]
        dt = t1 - t0
        y1 = y + step(func, t0, dt, t1, y)
        while j < len(tt) and t1 >= tt[j]:
            if tt[j] == t0:
                out.append(y)
            elif tt[j] == t1:
                out.append(y1)
            else:
                out.append(y + (tt[j] - t0) / (t1 - t0) * (y1 - y))
            j += 1
        y = y1
    return torch.stack(out, 0)


def odeint(func, y0, t, *, rtol=1e-7, atol=1e-9, method=None, options=None, event_fn=None):
    if event_fn is not None:
        raise NotImplementedError("event handling is not supported")
    method = "dopri5" if method is None else method
    if method not in FIXED_METHODS + ADAPTIVE_METHODS:
        raise ValueError('Invalid method "{}". Must be one of {}'.format(
            method, '{"' + '", "'.join(FIXED_METHODS + ADAPTIVE_METHODS) + '"}.'))
    if torch.is_tensor(t) and t.is_cuda and method == "rk4":
        _host_t(t)           # validated once per tensor version, no device sync when cached
    else:
        _check_t(t)
    options = dict(options or {})
    step_size = options.pop("step_size", None)
    if method == "dopri5":
        first_step = options.pop("first_step", None)
        max_num_steps = options.pop("max_num_steps", _adaptive.MAX_NUM_STEPS)
        if fusable(func, y0) and func.uncertainty == "none" and not _needs_grad(func, y0):
            return _adaptive.fused_dopri5(func, y0, t, rtol, atol, first_step, max_num_steps)
        if isinstance(func, _UDEModule) and _strict() and not _eval_fused(func, y0):
            raise RuntimeError("UDE_STRICT=1: this dopri5 solve would not run on the fused gfx950 kernels "
                               f"(grad={_needs_grad(func, y0)}, device={y0.device}, dtype={y0.dtype})")
        return _adaptive.eager_dopri5(func, y0, t, rtol, atol, first_step, max_num_steps)
    if method in ADAPTIVE_METHODS:
        raise NotImplementedError(f"method '{method}' is not implemented (rk4 / euler / midpoint / dopri5 are)")
    if method == "rk4" and fusable(func, y0):
        return fused_odeint(func, y0, t, step_size)
    if isinstance(func, _UDEModule) and _strict() and not _eval_fused(func, y0):
        raise RuntimeError("UDE_STRICT=1: this solve would not run on the fused gfx950 kernels "
                           f"(method={method}, device={y0.device}, dtype={y0.dtype})")
    if getattr(func, "uncertainty", None) == "bayes" and _eval_fused(func, y0):
        # Bayesian RHS evaluated one kernel per evaluation: the whole solve's weight samples
        # are formed up front (the whole-solve kernel's eps stream, ude_amd/bayes.py)
        n_eval = (len(fixed_grid(t, step_size)) - 1) * _STAGES[method]
        with func.presampled(n_eval, y0.device):
            return eager_fixed_grid(func, y0, t, method, step_size)
    return eager_fixed_grid(func, y0, t, method, step_size)
