"""CPU oracle for ``odeint_adjoint`` -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the checker.

torchdiffeq's ``odeint_adjoint`` (0.2.x ``adjoint.py``, ``OdeintAdjointMethod``) restated:
BASELINE configs[2]'s "adjoint backward".  torchdiffeq is a third-party dependency that is
neither vendored in the reference nor installed here (version unpinned), and the reference
never calls the adjoint, so this restatement is "parity unpinned" w.r.t.
torchdiffeq itself; it is checked by known-answer tests (tests/test_adjoint.py: the adjoint
gradient of a linear ODE against the analytic one, and against autograd through the forward
solve as the tolerances shrink).

Restated: forward ``odeint`` without autograd; backward per output interval, last first:
augmented state ``(vjp_t, y, adj_y, *adj_params)`` integrated from t[i] to t[i-1] by dopri5
(oracle/ude_oracle_dopri5.py) on ``-aug(-s, .)`` (decreasing t is solved as increasing -t,
``_ReverseFunc``), augmented dynamics ``(vjp_t, f, vjp_y, *vjp_params) = (d f . -adj_y)``
through autograd, error norm ``max(|t|, rms(y), rms(adj_y), max_p rms(adj_p))``
(``default_adjoint_norm``), then ``y <- y(t[i-1])`` of the forward solve and
``adj_y += grad_y[i-1]``.
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import torch

from oracle.ude_oracle_dopri5 import odeint_dopri5, rms_norm


def _pieces(flat: torch.Tensor, shapes) -> List[torch.Tensor]:
    out, off = [], 0
    for s in shapes:
        n = int(torch.Size(s).numel())
        out.append(flat[off:off + n].reshape(s))
        off += n
    return out


def adjoint_backward(func: Callable, params: Sequence[torch.Tensor], t: torch.Tensor, ys: torch.Tensor,
                     grad_y: torch.Tensor, rtol: float, atol: float):
    """(d y0, [d p]) of sum(grad_y * odeint(func, y0, t)) by torchdiffeq's adjoint; ys = the
    forward solution at t."""
    params = list(params)
    shapes = [torch.Size([]), ys.shape[1:], ys.shape[1:]] + [p.shape for p in params]

    def aug(tt, state):
        y, a = state[1], state[2]
        with torch.enable_grad():
            yv = y.detach().requires_grad_(True)
            fe = func(tt, yv)
            g = torch.autograd.grad(fe, [yv] + params, -a, allow_unused=True)
        gy = torch.zeros_like(y) if g[0] is None else g[0]
        gp = [torch.zeros_like(p) if x is None else x for p, x in zip(params, g[1:])]
        return [torch.zeros((), dtype=y.dtype), fe.detach(), gy] + gp

    def norm(flat):
        parts = _pieces(flat, shapes)
        n = max(parts[0].abs(), rms_norm(parts[1]), rms_norm(parts[2]))
        if len(parts) > 3:
            n = max(n, max(rms_norm(p) for p in parts[3:]))
        return n

    state = [torch.zeros((), dtype=ys.dtype), ys[-1], grad_y[-1]] + [torch.zeros_like(p) for p in params]
    for i in range(len(t) - 1, 0, -1):
        flat0 = torch.cat([x.reshape(-1) for x in state])

        def f_rev(s, flat):
            return -torch.cat([x.reshape(-1) for x in aug(-s, _pieces(flat, shapes))])

        sol = odeint_dopri5(f_rev, flat0, torch.stack([-t[i], -t[i - 1]]).to(torch.float64), rtol=rtol, atol=atol,
                            norm=norm)
        state = _pieces(sol[1], shapes)
        state[1] = ys[i - 1]
        state[2] = state[2] + grad_y[i - 1]
    return state[2], state[3:]
