"""Adaptive Dormand-Prince solves (``odeint(..., method='dopri5')``, torchdiffeq's default).

Two executions of the same torchdiffeq 0.2.x algorithm (``RKAdaptiveStepsizeODESolver``
with the Dormand-Prince-Shampine tableau, ``_select_initial_step``,
``_optimal_step_size``, dense output by ``_interp_fit`` / ``_interp_evaluate``; one
step size for the whole batch from the RMS error norm over every state element):

* ``fused_dopri5``: the UDE right-hand sides on a HIP device without autograd
  (validation / forecasting, ``VAE.__call__(training=False)``, lib/VAE.py:127):
  the gfx950 kernels of csrc/ude_dopri5.h through ``ude_dopri5_forward``.  The
  side statistics (``posterior()``, ``tracker``) cover every evaluation, rejected
  steps and the two start-up evaluations included, as the reference's lists do.
* ``eager_dopri5``: any callable, any device, differentiable (autograd through
  every stage and through the step-size controller, as torchdiffeq's odeint).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from . import _native
from . import fused as _fused

_BETA = [
    [1 / 5],
    [3 / 40, 9 / 40],
    [44 / 45, -56 / 15, 32 / 9],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
    [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84],
]
_ALPHA = [1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0, 1.0]
_C_ERROR = [35 / 384 - 1951 / 21600, 0.0, 500 / 1113 - 22642 / 50085, 125 / 192 - 451 / 720,
            -2187 / 6784 - -12231 / 42400, 11 / 84 - 649 / 6300, -1.0 / 60.0]
_C_MID = [6025192743 / 30085553152 / 2, 0.0, 51252292925 / 65400821598 / 2, -2691868925 / 45128329728 / 2,
          187940372067 / 1594534317056 / 2, -1776094331 / 19743644256 / 2, 11237099 / 235043384 / 2]
MAX_NUM_STEPS = 2 ** 31 - 1



# ---------------------------------------------------------------------------
# fused (HIP) forward
# ---------------------------------------------------------------------------
def fused_dopri5(func, y0: torch.Tensor, t: torch.Tensor, rtol=1e-7, atol=1e-9, first_step=None,
                 max_num_steps: int = MAX_NUM_STEPS) -> torch.Tensor:
    cfg = func.ude_config()
    lib = _native.library_for(cfg)
    desc = _native.make_desc(cfg)
    dev = y0.device
    prob = _native.UdeProblem()
    prob.n_traj = int(y0.shape[0])
    prob.n_steps = 0
    prob.n_out = int(len(t)) - 1
    prob.fa_w = float(func.fa_weight())
    dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
    sizes = lib.query(desc, prob, dev_index)
    stream = _fused._stream(dev)
    ws_bytes = lib.dopri5_workspace(desc, prob, dev_index)
    pack = torch.empty(sizes.pack_bytes // 4, dtype=torch.float32, device=dev)
    lins = func.ude_linears()
    ws_t = [l.weight.detach().contiguous() for l in lins]
    bs_t = [l.bias.detach().contiguous() for l in lins]
    lib.pack(desc, [w.data_ptr() for w in ws_t], [b.data_ptr() for b in bs_t], pack.data_ptr(), stream)
    t64 = t.detach().to(device=dev, dtype=torch.float64).contiguous()
    y = y0.detach().contiguous()
    latent = torch.empty((len(t),) + tuple(y.shape), dtype=torch.float32, device=dev)
    ws = torch.empty(max(ws_bytes // 8, 1), dtype=torch.float64, device=dev)
    stats = torch.zeros(5, dtype=torch.float32, device=dev)
    fs = 0.0 if first_step is None else float(first_step)
    info = lib.dopri5_forward(desc, prob, pack.data_ptr(), t64.data_ptr(), float(rtol), float(atol), fs,
                              min(int(max_num_steps), MAX_NUM_STEPS), y.data_ptr(), latent.data_ptr(),
                              ws.data_ptr(), stats.data_ptr(), stream)
    func._record_fused(stats, info.n_evals * prob.n_traj * func.n_regions)
    func.last_solve_info = {"method": "dopri5", "n_steps": info.n_steps, "n_accepted": info.n_accepted,
                            "n_evals": info.n_evals}
    return latent


# ---------------------------------------------------------------------------
# eager (any callable, differentiable)
# ---------------------------------------------------------------------------
def _rms_default(x: torch.Tensor) -> torch.Tensor:
    return x.abs().pow(2).mean().sqrt()


def _dot(ks: List[torch.Tensor], c: torch.Tensor) -> torch.Tensor:
    """sum_i c[i] * ks[i] (torchdiffeq: ``stack(k, -1).matmul(c)``) as a chain of multiply-adds:
    the (n, k) x (k,) matmul is a transposed GEMV that rocBLAS runs with one workgroup per
    output element -- 11 ms for a 10^6-element augmented adjoint state, vs ~20 us here."""
    acc = ks[0] * c[0]
    for i in range(1, len(ks)):
        acc = torch.addcmul(acc, ks[i], c[i])
    return acc


def _initial_dt(func, y0, f0, t0, first_step, rt, at, _rms):
    """torchdiffeq's ``_select_initial_step`` (fp64 device scalar), or the given first step."""
    ydt, dev = y0.dtype, y0.device
    if first_step is not None:
        return torch.as_tensor(first_step, dtype=torch.float64, device=dev)
    scale = at + torch.abs(y0) * rt
    d0 = _rms(y0 / scale).abs()
    d1 = _rms(f0 / scale).abs()
    h0 = torch.tensor(1e-6, dtype=ydt, device=dev) if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    h0 = h0.abs()
    f1 = func(t0.to(ydt) + h0, y0 + h0 * f0)
    d2 = torch.abs(_rms((f1 - f0) / scale) / h0)
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = torch.max(torch.tensor(1e-6, dtype=ydt, device=dev), h0 * 1e-3)
    else:
        h1 = (0.01 / torch.max(d1, d2)) ** (1.0 / 5.0)
    return torch.min(100 * h0, h1.abs()).to(torch.float64)


def host_scalar_dopri5(func, y0: torch.Tensor, t: torch.Tensor, rtol, atol, first_step, max_num_steps: int, norm,
                       hv) -> torch.Tensor:
    """``eager_dopri5(..., vec=...)`` for an autonomous fused right-hand side (odeint_adjoint's fused
    backward), with the controller's scalars on the host: the step size, step ends and stage
    coefficients are mirrored exactly in Python (fp64 sums, fp32 coefficient products as PyTorch forms
    them), the stage / error combinations take their coefficients by value (``hv.comb_hc``: ude_lincomb_hc)
    and the error ratio and next step size come from one device kernel (``hv.ratio_dt``: ude_dopri_ratio)
    read with the state's finiteness flag in ONE host transfer per attempt.  The same decisions and the
    same arithmetic as the operator chain (tests/test_adjoint.py), without its ~60 scalar kernels per
    attempt.  ``func(None, y)``: the evaluation time is not passed (the fused RHS ignores it)."""
    import numpy as np
    f32 = np.float32
    ydt, dev = y0.dtype, y0.device
    tt = t.to(device=dev, dtype=torch.float64)
    tt_h = tt.tolist()
    rt = torch.as_tensor(rtol, dtype=torch.float64, device=dev)
    at = torch.as_tensor(atol, dtype=torch.float64, device=dev)
    beta32 = [[f32(b) for b in row] for row in _BETA]
    cerr32 = [f32(c) for c in _C_ERROR]
    cmid32 = [f32(c) for c in _C_MID]
    f0 = func(tt[0].to(ydt), y0)
    dt_h = float(_initial_dt(func, y0, f0, tt[0], first_step, rt, at, norm))
    out = [y0]
    y, fy = y0, f0
    t_end_h = seg_t0_h = tt_h[0]
    last = None
    n_steps = 0
    nonfin = torch.logical_not(torch.isfinite(y).all())
    for i in range(1, len(tt_h)):
        while tt_h[i] > t_end_h:
            if n_steps >= max_num_steps:
                raise AssertionError("max_num_steps exceeded")
            te_h = t_end_h + dt_h
            if not te_h > t_end_h:
                raise AssertionError(f"underflow in dt {dt_h}")
            dts = f32(dt_h)
            ks = [fy]
            yi = y
            for s in range(6):
                yi = hv.comb_hc(y, ks, [b * dts for b in beta32[s]])
                ks.append(func(None, yi))
            y1, f1 = yi, ks[-1]
            err = hv.comb_hc(None, ks, [c * dts for c in cerr32])
            rf, dt_next, bad = hv.ratio_dt(err, y, y1, dt_h, nonfin)
            if bad:
                raise AssertionError("non-finite values in state `y`")
            n_steps += 1
            if rf <= 1:
                last = (y, fy, y1, f1, ks, dts)
                seg_t0_h, t_end_h = t_end_h, te_h
                y, fy = y1, f1
                nonfin = torch.logical_not(torch.isfinite(y).all())
            dt_h = dt_next
        yl, fyl, y1l, f1l, ksl, dts_l = last
        # torchdiffeq's dense output with eager_dopri5's operations (0-dim fp32 device scalars)
        dtl = torch.tensor(float(dts_l), dtype=ydt, device=dev)
        y_mid = hv.comb_hc(yl, ksl, [c * dts_l for c in cmid32])
        a = 2 * dtl * (f1l - fyl) - 8 * (y1l + yl) + 16 * y_mid
        b = dtl * (5 * fyl - 3 * f1l) + 18 * yl + 14 * y1l - 32 * y_mid
        c = dtl * (f1l - 4 * fyl) - 11 * yl - 5 * y1l + 16 * y_mid
        coef = [yl, dtl * fyl, c, b, a]
        x = torch.tensor(float(f32((tt_h[i] - seg_t0_h) / (t_end_h - seg_t0_h))), dtype=ydt, device=dev)
        total = coef[0] + x * coef[1]
        xp = x
        for cc in coef[2:]:
            xp = xp * x
            total = total + xp * cc
        out.append(total)
    return torch.stack(out, 0)


def eager_dopri5(func, y0: torch.Tensor, t: torch.Tensor, rtol=1e-7, atol=1e-9, first_step=None,
                 max_num_steps: int = MAX_NUM_STEPS, norm=None, vec=None) -> torch.Tensor:
    """``norm``: torchdiffeq's error norm (default the RMS over every element, ``_rms_norm``);
    odeint_adjoint passes its mixed norm over the augmented state's pieces.  ``vec`` (optional):
    ``vec.comb(base, ks, c)`` = base + sum_j c[j] ks[j] and ``vec.ratio(err, y, y1)`` = the error
    ratio, each one pass over the state (odeint_adjoint's fused path: ude_lincomb /
    ude_scaled_sumsq) instead of a chain of PyTorch operators.  The dense-output coefficients are
    formed only for the step an output time falls in (same arithmetic, not per accepted step)."""
    _rms = _rms_default if norm is None else norm
    comb = (lambda base, ks, c: (_dot(ks, c) if base is None else base + _dot(ks, c))) if vec is None else vec.comb
    ydt = y0.dtype
    dev = y0.device
    tt = t.to(device=dev, dtype=torch.float64)
    rt = torch.as_tensor(rtol, dtype=torch.float64, device=dev)
    at = torch.as_tensor(atol, dtype=torch.float64, device=dev)
    beta = [torch.tensor(b, dtype=ydt, device=dev) for b in _BETA]
    c_err = torch.tensor(_C_ERROR, dtype=ydt, device=dev)
    c_mid = torch.tensor(_C_MID, dtype=ydt, device=dev)

    t0 = tt[0]
    f0 = func(t0.to(ydt), y0)
    dt = _initial_dt(func, y0, f0, t0, first_step, rt, at, _rms)

    out = [y0]
    y, fy = y0, f0
    t_end = t0
    seg_t0 = t0
    last = None        # the last accepted step: (y, f(y), y1, f(y1), ks, dt)
    n_steps = 0
    # one host read per attempt: the error ratio, the step's end time and the underflow / finiteness
    # checks of its start travel together (the checks are raised in the same order, before the
    # attempt is used); t_end_h mirrors the device t_end exactly (fp64 both)
    tt_h = tt.tolist()
    t_end_h = tt_h[0]
    for i in range(1, len(tt)):
        next_t = tt[i]
        while tt_h[i] > t_end_h:
            if n_steps >= max_num_steps:
                raise AssertionError("max_num_steps exceeded")
            ts, te = t_end, t_end + dt
            flags = torch.stack([torch.logical_not(te > ts), torch.logical_not(torch.isfinite(y).all())])
            dts = dt.to(ydt)
            ks = [fy]
            yi = y
            for s in range(6):
                yi = comb(y, ks, beta[s] * dts)
                ti = te if _ALPHA[s] == 1.0 else ts + _ALPHA[s] * dt
                ks.append(func(ti.to(ydt), yi))
            y1, f1 = yi, ks[-1]
            err = comb(None, ks, dts * c_err)
            if vec is None:
                ratio = _rms(err / (at + rt * torch.max(y.abs(), y1.abs()))).abs()
            else:
                ratio = vec.ratio(err, y, y1)
            n_steps += 1
            rf, te_h, underflow, nonfinite = torch.cat([ratio.detach().double().reshape(1), te.detach().reshape(1),
                                                         flags.double()]).tolist()
            if underflow:
                raise AssertionError(f"underflow in dt {float(dt)}")
            if nonfinite:
                raise AssertionError("non-finite values in state `y`")
            if rf <= 1:
                last = (y, fy, y1, f1, ks, dts)
                seg_t0, t_end, t_end_h = ts, te, te_h
                y, fy = y1, f1
            if rf == 0:
                dt = dt * 10.0
            else:
                dfac = 1.0 if rf < 1 else 0.2
                fac = torch.clamp(0.9 / ratio.to(torch.float64) ** 0.2, min=dfac, max=10.0)
                dt = dt * fac
        yl, fyl, y1l, f1l, ksl, dtl = last
        y_mid = comb(yl, ksl, dtl * c_mid)
        a = 2 * dtl * (f1l - fyl) - 8 * (y1l + yl) + 16 * y_mid
        b = dtl * (5 * fyl - 3 * f1l) + 18 * yl + 14 * y1l - 32 * y_mid
        c = dtl * (f1l - 4 * fyl) - 11 * yl - 5 * y1l + 16 * y_mid
        coef = [yl, dtl * fyl, c, b, a]
        x = ((next_t - seg_t0) / (t_end - seg_t0)).to(ydt)
        total = coef[0] + x * coef[1]
        xp = x
        for cc in coef[2:]:
            xp = xp * x
            total = total + xp * cc
        out.append(total)
    return torch.stack(out, 0)
