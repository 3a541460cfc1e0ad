"""One evaluation of a UDE right-hand side on the gfx950 kernels (csrc/ude_eval.h).

``Fp / Fa / FaFp.forward(t, x)`` (lib/models.py:129-146, :177-188, :230-254) and the Bayesian
``forward`` (lib/in_development/models_bayes.py:69-265) on a HIP device call ``rhs_eval``:
one kernel computes the returned derivative and the tensors the reference appends to
``params`` (rates) and ``tracker`` (Fa); autograd's backward through the call is one VJP
kernel (plus the deterministic gradient reductions).  So every solve that evaluates the
module step by step -- adaptive dopri5 with autograd, ``odeint_adjoint``'s augmented
dynamics, euler / midpoint, the Bayesian RHS at sizes the fused whole-solve kernel does not
hold -- runs one kernel per evaluation instead of ~40 PyTorch operators, with the reference's
exact tracking-list semantics.

Bayesian layers: each evaluation's sample ``w = mu + eps * |std|`` is drawn and formed by the
layers themselves (the reference's RNG order and fp32 op order, autograd into mu and std), and
the kernel evaluates the RHS with that sample as a deterministic weight set.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _native
from . import fused as _fused


class _Plan:
    def __init__(self, cfg, n: int, fa_w: float, device: torch.device):
        self.lib = _native.library_for(cfg)
        self.desc = _native.make_desc(cfg)
        self.prob = _native.UdeProblem()
        self.prob.n_traj = int(n)
        self.prob.n_steps = 1
        self.prob.n_out = 0
        self.prob.fa_w = float(fa_w)
        dev_index = device.index if device.index is not None else torch.cuda.current_device()
        self.sizes = self.lib.query(self.desc, self.prob, dev_index)
        self.ws_bytes = self.lib.rhs_workspace(self.desc, self.prob, dev_index)
        kind = cfg[0]
        self.has_p = kind in ("Fp", "FaFp")
        self.has_a = kind in ("Fa", "FaFp")


_PLANS: Dict[tuple, _Plan] = {}


def _plan(cfg, n: int, fa_w: float, device: torch.device) -> _Plan:
    key = (cfg, int(n), float(fa_w), str(device))
    p = _PLANS.get(key)
    if p is None:
        if len(_PLANS) > 64:
            _PLANS.clear()
        p = _PLANS[key] = _Plan(cfg, n, fa_w, device)
    return p


class _FusedEval(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan: _Plan, shapes, x: torch.Tensor, *wb: torch.Tensor):
        """``shapes`` None: wb = (W, b) per Linear; else wb = (one flat weight vector,) holding
        the tensors of ``shapes`` back to back (C-ABI order), whose gradient comes back flat."""
        dev = x.device
        stream = _fused._stream(dev)
        N, R, L = x.shape
        if shapes is None:
            ws_ = [w.contiguous() for w in wb[0::2]]
            bs_ = [b.contiguous() for b in wb[1::2]]
            ptrs = [t.data_ptr() for t in ws_], [t.data_ptr() for t in bs_]
        else:
            flat = wb[0].contiguous()
            offs, off = [], 0
            for shp in shapes:
                offs.append(flat.data_ptr() + 4 * off)
                off += int(torch.Size(shp).numel())
            if off != flat.numel() or flat.dtype != torch.float32:
                raise ValueError(f"flat weights: {flat.numel()} {flat.dtype} elements, the model has {off} fp32")
            ptrs = offs[0::2], offs[1::2]
        pack = torch.empty(plan.sizes.pack_bytes // 4, dtype=torch.float32, device=dev)
        plan.lib.pack(plan.desc, ptrs[0], ptrs[1], pack.data_ptr(), stream)
        x = x.contiguous()
        f = torch.empty_like(x)
        rates = torch.empty((N, R, 2), dtype=torch.float32, device=dev) if plan.has_p else x.new_empty(0)
        fa = torch.empty((N, R, 3), dtype=torch.float32, device=dev) if plan.has_a else x.new_empty(0)
        plan.lib.rhs_forward(plan.desc, plan.prob, pack.data_ptr(), x.data_ptr(), f.data_ptr(),
                             rates.data_ptr() if plan.has_p else None, fa.data_ptr() if plan.has_a else None, stream)
        ctx.plan = plan
        ctx.flat = shapes is not None
        ctx.shapes = [t.shape for t in wb]
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, pack)
        return f, rates, fa

    @staticmethod
    def backward(ctx, gf, grates, gfa):
        plan: _Plan = ctx.plan
        x, pack = ctx.saved_tensors
        dev = x.device
        n_wb = len(ctx.shapes)
        if gf is None and grates is None and gfa is None:
            return (None, None, None) + (None,) * n_wb
        gf = torch.zeros_like(x) if gf is None else gf.contiguous().float()
        grates = None if (grates is None or not plan.has_p) else grates.contiguous().float()
        gfa = None if (gfa is None or not plan.has_a) else gfa.contiguous().float()
        dx = torch.empty_like(x)
        ws = torch.empty(max(plan.ws_bytes // 4, 1), dtype=torch.float32, device=dev)
        dparams = torch.empty(plan.sizes.n_params, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            plan.lib.rhs_vjp(plan.desc, plan.prob, pack.data_ptr(), x.data_ptr(), gf.data_ptr(),
                             None if grates is None else grates.data_ptr(), None if gfa is None else gfa.data_ptr(),
                             dx.data_ptr(), ws.data_ptr(), dparams.data_ptr(), _fused._stream(dev))
        if ctx.flat:
            return None, None, dx, dparams
        return (None, None, dx) + tuple(_fused._split(dparams, ctx.shapes))


def eligible(module, x: torch.Tensor) -> bool:
    if not (getattr(module, "fused_eval", True) and x.is_cuda and x.dtype == torch.float32 and x.dim() == 3
            and x.shape[1] == module.n_regions and x.shape[2] == module.latent_dim and x.shape[0] > 0
            and all(w.is_cuda and w.dtype == torch.float32 and w.device == x.device for w in module.parameters())):
        return False
    return _native.config_supported(deterministic_config(module))


def deterministic_config(module):
    kind, R, L, net, aug = module.ude_config()
    return (kind[1:] if kind.startswith("B") else kind, R, L, net, aug)


def rhs_eval(module, x: torch.Tensor, weights
             ) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
    """(f, rates, Fa) of one evaluation; weights = (W, b) per Linear in C-ABI order (rate net
    first), or those tensors back to back in one 1-D tensor (a pre-drawn Bayesian sample row).
    rates / Fa are None for the net the module does not have."""
    plan = _plan(deterministic_config(module), x.shape[0], module.fa_weight(), x.device)
    with torch.cuda.device(x.device):
        if isinstance(weights, torch.Tensor):
            f, rates, fa = _FusedEval.apply(plan, module.ude_weight_shapes(), x, weights)
        else:
            f, rates, fa = _FusedEval.apply(plan, None, x, *weights)
    return f, (rates if plan.has_p else None), (fa if plan.has_a else None)
