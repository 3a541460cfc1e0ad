"""Decoder epilogue of the training solve and the nll over its output.

The reference's training step reads the latent of ``odeint`` only through

* ``y_pred = self.dec(self.latent[..., :3])`` (lib/VAE.py:138; Decoder = Flatten + Linear(3R -> R),
  lib/models.py:27-51) reshaped ``(T, S, B, R)`` and permuted ``(B, S, T, R)``, and
* ``reg_loss = 0.1 * latent_init_loss(self.latent[..., :3])`` (lib/VAE.py:186,
  lib/train_functions.py:116-126).

``solve_decode`` runs the training solve with both computed in the forward kernel's output
path (``FusedRK4Dec``, ude_rk4_forward_dec): ``y_hat (T, N, R)`` and the reg sum, and no
``(T, N, R, L)`` latent is written; the latent is rebuilt from the training store only if
something reads it (``LazyLatent``).  ``nll_head`` is ``nll_loss(y_pred, y)``
(lib/train_functions.py:81-90) over ``y_hat`` on the gfx950 nll kernels (per (t, b, r)
sample mean / unbiased std, -log N(y), masked y == -1, mean), forward and backward one pass each.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native
from . import fused as _fused


MAX_TIMES = 2048          # output times the decoder backward's grid-point table holds (DecBwdDims::MAX_T)


def decoder_linear(dec) -> Optional[torch.nn.Linear]:
    """The Linear(3R -> R) of a reference Decoder (lib/models.py:37-40), else None."""
    seq = getattr(dec, "decoder", None)
    if not isinstance(seq, torch.nn.Sequential) or len(seq) != 2:
        return None
    if not isinstance(seq[0], torch.nn.Flatten) or not isinstance(seq[1], torch.nn.Linear):
        return None
    if getattr(dec, "latent_dim", None) != 3:
        return None
    return seq[1]


def eligible(ode, y0: torch.Tensor, linear: Optional[torch.nn.Linear]) -> bool:
    from .solvers import fusable
    R = getattr(ode, "n_regions", None)
    return (linear is not None and fusable(ode, y0) and ode.uncertainty in ("none", "bayes")
            and not ode.materialize_tracking and tuple(linear.weight.shape) == (R, 3 * R)
            and linear.bias is not None and linear.weight.dtype == torch.float32
            and linear.weight.device == y0.device)


class LazyLatent:
    """``VAE.latent`` of a decoder-epilogue solve: materialised (differentiably) on first read."""

    def __init__(self, token, ckpt, y0, plan):
        self._args = (token, ckpt, y0, plan)
        self._value = None

    def get(self) -> torch.Tensor:
        if self._value is None:
            self._value = _fused.materialize_latent(*self._args)
            self._args = None
        return self._value

    @property
    def materialized(self) -> bool:
        return self._value is not None


def solve_decode(ode, y0: torch.Tensor, t: torch.Tensor, step_size, linear: torch.nn.Linear):
    """(y_hat (T, N, R), reg (scalar), LazyLatent, plan) -- or None when the schedule has an output
    time that is not a grid point (the epilogue needs exact hits: torchdiffeq mode y(t1))."""
    from . import solvers
    plan = solvers.plan_for(ode, y0, t, step_size)
    if plan.out_k is None or plan.n_times > MAX_TIMES:
        return None
    if ode.uncertainty == "bayes":
        # every evaluation's weight sample (models_bayes.py:43-48) from the solve's eps stream
        mus, sds = ode.ude_mean_std()
        eps = ode.take_eps(4 * plan.prob.n_steps, sum(int(p.numel()) for p in mus), y0.device)
        yhat, reg, mean, std, fa_norm, token, ckpt, sums = _fused.FusedBayesRK4Dec.apply(
            plan, y0.contiguous(), eps, linear.weight, linear.bias, *(mus + sds))
    else:
        params = []
        for lin in ode.ude_linears():
            params += [lin.weight, lin.bias]
        yhat, reg, mean, std, fa_norm, token, ckpt, sums = _fused.FusedRK4Dec.apply(
            plan, y0.contiguous(), linear.weight, linear.bias, *params)
    ode._record_fused((mean, std, fa_norm), plan.n_eval, sums=sums)
    return yhat, reg, LazyLatent(token, ckpt, y0, plan), plan


class _NllHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lib, desc, T, S, B, yhat, y):
        dev = yhat.device
        stream = _fused._stream(dev)
        ws = torch.empty(max(lib.nll_workspace(desc, T, S, B) // 4, 1), dtype=torch.float32, device=dev)
        out = torch.empty(1, dtype=torch.float32, device=dev)
        yhat, y = yhat.contiguous(), y.contiguous()
        if _fused.EVENTS is not None:
            e0 = _fused._ev(dev); e0.record()
        lib.nll_forward(desc, T, S, B, yhat.data_ptr(), y.data_ptr(), ws.data_ptr(), out.data_ptr(), stream)
        if _fused.EVENTS is not None:
            e1 = _fused._ev(dev); e1.record(); _fused.EVENTS.append(("nll_fwd", e0, e1))
        ctx.meta = (lib, desc, T, S, B)
        ctx.save_for_backward(yhat, y, ws)
        ctx.mark_non_differentiable(ws)
        return out[0], ws

    @staticmethod
    def backward(ctx, g, _gws=None):
        lib, desc, T, S, B = ctx.meta
        yhat, y, ws = ctx.saved_tensors
        dev = yhat.device
        grad = torch.zeros(1, dtype=torch.float32, device=dev) if g is None else g.reshape(1).float()
        dyhat = torch.empty_like(yhat)
        if _fused.EVENTS is not None:
            e0 = _fused._ev(dev); e0.record()
        lib.nll_backward(desc, T, S, B, yhat.data_ptr(), y.data_ptr(), grad.data_ptr(), ws.data_ptr(),
                         dyhat.data_ptr(), _fused._stream(dev))
        if _fused.EVENTS is not None:
            e1 = _fused._ev(dev); e1.record(); _fused.EVENTS.append(("nll_bwd", e0, e1))
        return None, None, None, None, None, dyhat, None


def nll_head(ode, yhat: torch.Tensor, y: torch.Tensor, n_samples: int, batch: int):
    """(nll, group_stats (T, B, R, 2) = per-group sample mean / std) of y_pred = y_hat as lib/VAE.py
    :138 reshapes it, against targets y (B, T, R)."""
    cfg = ode.ude_config()
    lib = _native.library_for(cfg)
    desc = _native.make_desc(cfg)
    T, N, R = yhat.shape
    if N != n_samples * batch or tuple(y.shape) != (batch, T, R) or n_samples < 2:
        raise ValueError(f"nll_head: y_hat {tuple(yhat.shape)} / targets {tuple(y.shape)} do not match "
                         f"S={n_samples}, B={batch}")
    with torch.cuda.device(yhat.device):
        nll, ws = _NllHead.apply(lib, desc, T, int(n_samples), int(batch), yhat, y.to(torch.float32))
    return nll, ws[: T * batch * R * 2].view(T, batch, R, 2)
