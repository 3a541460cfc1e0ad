"""Fused training loss head over the solve's latent (csrc/ude_loss.h).

``fused_loss_head(ode, latent, decoder_linear, y, n_samples, batch)`` returns
``(nll, reg)`` with

* ``nll = nll_loss(y_pred, y)`` (lib/train_functions.py:81-90) for
  ``y_pred = Decoder(latent[..., :3])`` reshaped / permuted as lib/VAE.py:138 does,
* ``reg = latent_init_loss(latent[..., :3])`` (lib/train_functions.py:116-126),

forward and backward each one gfx950 kernel pass over the latent (no slice copies,
no permuted reductions) instead of ~20 PyTorch kernels.  Used by the drop-in
``VAE.calc_loss`` when the prediction it is handed is the model's own decoder output.
"""
from __future__ import annotations

import torch

from . import _native
from . import fused as _fused


class _LossHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lib, desc, T, S, B, latent, sir_token, W, b, y):
        dev = latent.device
        stream = _fused._stream(dev)
        dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
        nbytes = lib.loss_workspace(desc, T, S, B, dev_index)
        ws = torch.empty(max(nbytes // 8, 1), dtype=torch.float64, device=dev)
        out = torch.empty(2, dtype=torch.float32, device=dev)
        latent, W, b, y = latent.contiguous(), W.contiguous(), b.contiguous(), y.contiguous()
        if _fused.EVENTS is not None:
            e0 = _fused._ev(dev); e0.record()
        lib.loss_forward(desc, T, S, B, latent.data_ptr(), W.data_ptr(), b.data_ptr(), y.data_ptr(), ws.data_ptr(),
                         out.data_ptr(), stream)
        if _fused.EVENTS is not None:
            e1 = _fused._ev(dev); e1.record(); _fused.EVENTS.append(("loss_fwd", e0, e1))
        ctx.meta = (lib, desc, T, S, B)
        # a latent straight from the fused solve takes its (S, I, R-only) cotangent compactly,
        # as the gradient of the solve's sir_token output (fused.sir_token_like)
        ctx.compact = sir_token is not None
        ctx.save_for_backward(latent, W, b, y, ws)
        ctx.mark_non_differentiable(ws)
        # ws starts with the per-(t, b, r) sample mean / std of the predictions ((T, B, R, 2))
        return out[0], out[1], ws

    @staticmethod
    def backward(ctx, g_nll, g_reg, _g_ws=None):
        lib, desc, T, S, B = ctx.meta
        latent, W, b, y, ws = ctx.saved_tensors
        with torch.cuda.device(latent.device):
            return _LossHead._backward(lib, desc, T, S, B, latent, W, b, y, ws, g_nll, g_reg, ctx.compact)

    @staticmethod
    def _backward(lib, desc, T, S, B, latent, W, b, y, ws, g_nll, g_reg, compact):
        dev = latent.device
        zero = torch.zeros((), dtype=torch.float32, device=dev)
        grad = torch.stack([zero if g_nll is None else g_nll.float().reshape(()),
                            zero if g_reg is None else g_reg.float().reshape(())])
        dW = torch.empty_like(W)
        db = torch.empty_like(b)
        if _fused.EVENTS is not None:
            e0 = _fused._ev(dev); e0.record()
        dl3 = dlat = None
        if compact:
            N, R = latent.shape[1], latent.shape[2]
            dl3 = torch.empty((T, N, R, 3), dtype=torch.float32, device=dev)
            lib.loss_backward_sir(desc, T, S, B, latent.data_ptr(), W.data_ptr(), b.data_ptr(), y.data_ptr(),
                                  grad.data_ptr(), ws.data_ptr(), dl3.data_ptr(), dW.data_ptr(), db.data_ptr(),
                                  _fused._stream(dev))
        else:
            dlat = torch.empty_like(latent)
            lib.loss_backward(desc, T, S, B, latent.data_ptr(), W.data_ptr(), b.data_ptr(), y.data_ptr(),
                              grad.data_ptr(), ws.data_ptr(), dlat.data_ptr(), dW.data_ptr(), db.data_ptr(),
                              _fused._stream(dev))
        if _fused.EVENTS is not None:
            e1 = _fused._ev(dev); e1.record(); _fused.EVENTS.append(("loss_bwd", e0, e1))
        return None, None, None, None, None, dlat, dl3, dW, db, None


_FITS = {}
# hand the S, I, R cotangent to the fused solve's backward compactly (fused.sir_token_like) when the
# latent comes straight from it; False: always write the full (T, N, R, L) d latent
COMPACT = True


def _fits(cfg, T: int, S: int, B: int, device: torch.device) -> bool:
    """Whether the kernel takes (T, S, B): the sample count bounds its per-group register /
    LDS tiles (pad16(S) <= 128, LDS <= 160 KiB), which ude_loss_head_workspace checks."""
    key = (cfg, T, S, B, str(device))
    hit = _FITS.get(key)
    if hit is None:
        try:
            lib = _native.library_for(cfg)
            dev_index = device.index if device.index is not None else torch.cuda.current_device()
            lib.loss_workspace(_native.make_desc(cfg), T, S, B, dev_index)
            hit = True
        except _native.UdeError:
            hit = False
        _FITS[key] = hit
    return hit


def eligible(ode, latent: torch.Tensor, linear, n_samples: int, batch: int) -> bool:
    R = ode.n_regions
    if not (latent.is_cuda and latent.dtype == torch.float32 and latent.dim() == 4 and n_samples >= 2
            and latent.shape[1] == n_samples * batch and latent.shape[2] == R
            and latent.shape[3] == ode.latent_dim and latent.is_contiguous() and latent.data_ptr() % 16 == 0
            and isinstance(linear, torch.nn.Linear) and tuple(linear.weight.shape) == (R, 3 * R)
            and linear.bias is not None and linear.weight.dtype == torch.float32
            and linear.weight.device == latent.device
            and _native.config_supported(ode.ude_config())):
        return False
    return _fits(ode.ude_config(), int(latent.shape[0]), int(n_samples), int(batch), latent.device)


def fused_loss_head(ode, latent: torch.Tensor, linear: torch.nn.Linear, y: torch.Tensor, n_samples: int,
                    batch: int, group_stats: bool = False):
    """(nll, reg); with group_stats=True also the (T, B, R, 2) per-group prediction mean / std
    (the Normal parameters nll_loss builds, for the caller's argument validation)."""
    cfg = ode.ude_config()
    lib = _native.library_for(cfg)
    desc = _native.make_desc(cfg)
    T = int(latent.shape[0])
    if tuple(y.shape) != (batch, T, ode.n_regions):
        raise ValueError(f"targets {tuple(y.shape)} do not match (B, T, R) = {(batch, T, ode.n_regions)}")
    with torch.cuda.device(latent.device):
        token = getattr(latent, "_ude_sir_token", None) if COMPACT else None
        nll, reg, ws = _LossHead.apply(lib, desc, T, int(n_samples), int(batch), latent, token, linear.weight,
                                       linear.bias, y.to(torch.float32))
    if group_stats:
        R = ode.n_regions
        return nll, reg, ws.view(torch.float32)[: T * batch * R * 2].view(T, batch, R, 2)
    return nll, reg
