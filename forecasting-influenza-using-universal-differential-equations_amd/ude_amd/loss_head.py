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
    def forward(ctx, lib, desc, T, S, B, latent, W, b, y):
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
        ctx.save_for_backward(latent, W, b, y, ws)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_nll, g_reg):
        lib, desc, T, S, B = ctx.meta
        latent, W, b, y, ws = ctx.saved_tensors
        dev = latent.device
        zero = torch.zeros((), dtype=torch.float32, device=dev)
        grad = torch.stack([zero if g_nll is None else g_nll.float().reshape(()),
                            zero if g_reg is None else g_reg.float().reshape(())])
        dlat = torch.empty_like(latent)
        dW = torch.empty_like(W)
        db = torch.empty_like(b)
        if _fused.EVENTS is not None:
            e0 = _fused._ev(dev); e0.record()
        lib.loss_backward(desc, T, S, B, latent.data_ptr(), W.data_ptr(), b.data_ptr(), y.data_ptr(),
                          grad.data_ptr(), ws.data_ptr(), dlat.data_ptr(), dW.data_ptr(), db.data_ptr(),
                          _fused._stream(dev))
        if _fused.EVENTS is not None:
            e1 = _fused._ev(dev); e1.record(); _fused.EVENTS.append(("loss_bwd", e0, e1))
        return None, None, None, None, None, dlat, dW, db, None


def eligible(ode, latent: torch.Tensor, linear, n_samples: int, batch: int) -> bool:
    R = ode.n_regions
    return (latent.is_cuda and latent.dtype == torch.float32 and latent.dim() == 4 and n_samples >= 2
            and latent.shape[1] == n_samples * batch and latent.shape[2] == R and latent.shape[3] >= 3
            and isinstance(linear, torch.nn.Linear) and tuple(linear.weight.shape) == (R, 3 * R)
            and linear.bias is not None and linear.weight.dtype == torch.float32 and linear.weight.is_cuda
            and _native.config_supported(ode.ude_config()))


def fused_loss_head(ode, latent: torch.Tensor, linear: torch.nn.Linear, y: torch.Tensor, n_samples: int,
                    batch: int):
    cfg = ode.ude_config()
    lib = _native.library_for(cfg)
    desc = _native.make_desc(cfg)
    T = int(latent.shape[0])
    if tuple(y.shape) != (batch, T, ode.n_regions):
        raise ValueError(f"targets {tuple(y.shape)} do not match (B, T, R) = {(batch, T, ode.n_regions)}")
    return _LossHead.apply(lib, desc, T, int(n_samples), int(batch), latent, linear.weight, linear.bias,
                           y.to(torch.float32))
