"""CPU oracle for adaptive Dormand-Prince (dopri5) solves -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.

``torchdiffeq.odeint(func, y0, t, rtol=1e-7, atol=1e-9, method='dopri5')`` -- the
default method of the solver API the reference imports (lib/VAE.py:5,
run_ode.py:24) and BASELINE configs[2] -- restated from torchdiffeq's published
0.2.x algorithm.  torchdiffeq is a third-party dependency that is NOT vendored
in the reference and NOT installed here (version unpinned by the reference; no
reference test or fixture pins it), so this restatement is pinned by analytic
known-answer tests only (tests/test_dopri5.py): "parity unpinned" w.r.t.
torchdiffeq itself.

What is restated (torchdiffeq names):

* ``_select_initial_step`` (Hairer's heuristic with ``order - 1 = 4``):
  ``scale = atol + |y0| rtol``, ``d0 = rms(y0/scale)``, ``d1 = rms(f0/scale)``,
  ``h0 = 1e-6`` if either < 1e-5 else ``0.01 d0/d1``, one trial evaluation at
  ``y0 + h0 f0``, ``d2 = rms((f1-f0)/scale)/h0``, ``h1 = (0.01/max(d1,d2))^(1/5)``
  (or ``max(1e-6, 1e-3 h0)`` if both tiny), first step ``min(100 h0, h1)``;
* ``RKAdaptiveStepsizeODESolver`` with the Dormand-Prince-Shampine tableau:
  FSAL stages, ``y1`` = the 5th-order solution, error ``dt * sum_j c_err_j k_j``,
  ``error_ratio = rms(err / (atol + rtol max(|y0|,|y1|)))`` over the WHOLE
  state tensor (one step size for the batch), accept iff ``error_ratio <= 1``;
* ``_optimal_step_size`` (safety 0.9, ifactor 10, dfactor 0.2, order 5; no
  shrink limit when accepted);
* dense output: ``_interp_fit`` (4th-order Hermite-like fit through y0, y1,
  ``y_mid = y0 + dt sum_j mid_j k_j`` with the DPS ``C_MID`` weights, f0, f1)
  and ``_interp_evaluate`` at every requested time, using the last accepted
  step whose end reaches it (``_advance``);
* mixed precision: state arithmetic in y's dtype, time-like quantities in
  float64 (the solver's ``dtype``).

Every evaluation of ``func`` is a call the RHS tracks (``params`` / ``tracker``
of lib/models.py), rejected steps and the two start-up evaluations included.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch

# Dormand-Prince-Shampine tableau (torchdiffeq dopri5.py)
ALPHA = [1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0, 1.0]
BETA = [
    [1 / 5],
    [3 / 40, 9 / 40],
    [44 / 45, -56 / 15, 32 / 9],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
    [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84],
]
C_SOL = [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84, 0.0]
C_ERROR = [
    35 / 384 - 1951 / 21600,
    0.0,
    500 / 1113 - 22642 / 50085,
    125 / 192 - 451 / 720,
    -2187 / 6784 - -12231 / 42400,
    11 / 84 - 649 / 6300,
    -1.0 / 60.0,
]
C_MID = [
    6025192743 / 30085553152 / 2, 0.0, 51252292925 / 65400821598 / 2, -2691868925 / 45128329728 / 2,
    187940372067 / 1594534317056 / 2, -1776094331 / 19743644256 / 2, 11237099 / 235043384 / 2,
]
ORDER = 5
SAFETY, IFACTOR, DFACTOR = 0.9, 10.0, 0.2


def rms_norm(x: torch.Tensor) -> torch.Tensor:
    """torchdiffeq ``_rms_norm``: sqrt(mean(|x|^2)) over every element."""
    return x.abs().pow(2).mean().sqrt()


def _lincomb(ks: List[torch.Tensor], coefs: torch.Tensor) -> torch.Tensor:
    """sum_j ks[j] * coefs[j] (the ``k.matmul(c)`` of torchdiffeq)."""
    out = ks[0] * coefs[0]
    for j in range(1, len(ks)):
        out = out + ks[j] * coefs[j]
    return out


def select_initial_step(func, t0, y0, f0, rtol, atol, norm=rms_norm):
    """``_select_initial_step(func, t0, y0, order=4, rtol, atol, norm, f0)``."""
    dt = y0.dtype
    scale = atol + torch.abs(y0) * rtol
    d0 = norm(y0 / scale).abs()
    d1 = norm(f0 / scale).abs()
    if d0 < 1e-5 or d1 < 1e-5:
        h0 = torch.tensor(1e-6, dtype=dt)
    else:
        h0 = 0.01 * d0 / d1
    h0 = h0.abs()
    y1 = y0 + h0 * f0
    f1 = func(t0 + h0, y1)
    d2 = torch.abs(norm((f1 - f0) / scale) / h0)
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = torch.max(torch.tensor(1e-6, dtype=dt), h0 * 1e-3)
    else:
        h1 = (0.01 / torch.max(d1, d2)) ** (1.0 / float(4 + 1))
    h1 = h1.abs()
    return torch.min(100 * h0, h1).to(torch.float64)


def optimal_step_size(last_step: torch.Tensor, error_ratio: torch.Tensor) -> torch.Tensor:
    """``_optimal_step_size`` (float64 time arithmetic)."""
    if error_ratio == 0:
        return last_step * IFACTOR
    dfactor = 1.0 if error_ratio < 1 else DFACTOR
    er = error_ratio.to(torch.float64)
    factor = min(IFACTOR, max(SAFETY / float(er ** (1.0 / ORDER)), dfactor))
    return last_step * factor


def interp_fit(y0, y1, y_mid, f0, f1, dt):
    """``_interp_fit``: coefficients [e, d, c, b, a] of the dense-output polynomial."""
    a = 2 * dt * (f1 - f0) - 8 * (y1 + y0) + 16 * y_mid
    b = dt * (5 * f0 - 3 * f1) + 18 * y0 + 14 * y1 - 32 * y_mid
    c = dt * (f1 - 4 * f0) - 11 * y0 - 5 * y1 + 16 * y_mid
    d = dt * f0
    e = y0
    return [e, d, c, b, a]


def interp_evaluate(coef, t0, t1, t):
    """``_interp_evaluate``: polynomial at x = (t - t0)/(t1 - t0) (x in float64 -> y dtype)."""
    x = ((t - t0) / (t1 - t0)).to(coef[0].dtype)
    total = coef[0] + x * coef[1]
    xp = x
    for c in coef[2:]:
        xp = xp * x
        total = total + xp * c
    return total


class Dopri5Stats:
    def __init__(self):
        self.n_steps = 0
        self.n_accepted = 0
        self.n_evals = 0
        self.steps: List[tuple] = []     # (t0, dt, error_ratio, accepted)


def odeint_dopri5(func: Callable, y0: torch.Tensor, t: torch.Tensor, rtol=1e-7, atol=1e-9,
                  first_step=None, max_num_steps: int = 2 ** 31 - 1, stats: Optional[Dopri5Stats] = None,
                  norm: Callable = rms_norm):
    """``odeint(func, y0, t, rtol, atol, method='dopri5')`` (no events, no step_t / jump_t);
    ``norm`` = the solver's error norm (``options['norm']``, default ``_rms_norm``)."""
    st = stats if stats is not None else Dopri5Stats()
    sd = y0.dtype
    tt = t.to(torch.float64)

    def f(tv, y):
        st.n_evals += 1
        return func(tv, y)

    beta = [torch.tensor(b, dtype=sd) for b in BETA]
    c_err = torch.tensor(C_ERROR, dtype=sd)
    c_mid = torch.tensor(C_MID, dtype=sd)
    rtol_t = torch.tensor(rtol, dtype=torch.float64)
    atol_t = torch.tensor(atol, dtype=torch.float64)

    sol = [y0]
    t0 = tt[0]
    f0 = f(t0.to(sd), y0)
    if first_step is None:
        dt = select_initial_step(f, t0.to(sd), y0, f0, rtol_t.to(sd) if sd == torch.float64 else rtol_t,
                                 atol_t.to(sd) if sd == torch.float64 else atol_t, norm)
    else:
        dt = torch.tensor(first_step, dtype=torch.float64)
    y = y0
    t1 = t0                         # end of the last accepted step (rk_state.t1)
    coef = [y0] * 5
    last_t0 = t0
    for i in range(1, len(tt)):
        next_t = tt[i]
        while next_t > t1:
            assert st.n_steps < max_num_steps, "max_num_steps exceeded"
            assert t1 + dt > t1, f"underflow in dt {float(dt)}"
            assert bool(torch.isfinite(y).all()), "non-finite values in state `y`"
            ts = t1
            te = ts + dt
            dts = dt.to(sd)
            ks = [f0]
            yi = None
            for s in range(6):
                yi = y + _lincomb(ks, beta[s] * dts)
                ks.append(f(te.to(sd) if ALPHA[s] == 1.0 else (ts + ALPHA[s] * dt).to(sd), yi))
            y1 = yi                                            # c_sol == beta[5], c_sol[-1] == 0
            f1 = ks[-1]
            err = _lincomb(ks, dts * c_err)
            error_tol = atol_t + rtol_t * torch.max(y.abs(), y1.abs())
            error_ratio = norm(err / error_tol).abs()
            accept = bool(error_ratio <= 1)
            st.n_steps += 1
            st.steps.append((float(ts), float(dt), float(error_ratio), accept))
            if accept:
                y_mid = y + _lincomb(ks, dts * c_mid)
                coef = interp_fit(y, y1, y_mid, f0, f1, dts)
                last_t0 = ts
                t1 = te
                y, f0 = y1, f1
                st.n_accepted += 1
            dt = optimal_step_size(dt, error_ratio)
        sol.append(interp_evaluate(coef, last_t0, t1, next_t))
    return torch.stack(sol, 0)
