"""UDE right-hand sides with the reference's module interface.

Same class names, constructor signatures, attributes and ``state_dict`` keys as
``lib/models.py``: ``Fp`` (:109-156, keys ``Fp_net.{1,3,..}``), ``Fa``
(:158-197, ``aug_net.{0,2,..}``), ``FaFp`` (:199-265, ``net.*`` /
``aug_net.*``), so reference checkpoints load unchanged and, under the same
torch seed, the default initialisation draws the same weights.

``forward(t, x)`` is one eager evaluation with the reference semantics (used
when the module is called directly or by a non-fused solver).  Inside
``odeint(..., method='rk4')`` on a HIP device the whole solve runs in the
fused gfx950 kernel instead; the kernel then returns the side statistics the
loss reads (rate mean / std for ``posterior()``, the Fa norm for ``tracker``)
rather than per-eval tensors, see ``_record_fused``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
from torch import nn
from torch.distributions import Normal


def _linear_stack(n_in: int, sizes: Sequence[int], n_out: int, lead_flatten: bool) -> nn.ModuleList:
    """[Flatten?] Lin(n_in->s0) (ELU Lin(s_{i-1}->s_i))* Lin(s_last->n_out).

    Module indices (and so state_dict keys) follow lib/models.py:118-124: the
    ELU sits between consecutive hidden Linears only, so the last hidden Linear
    feeds the output Linear without an activation.
    """
    mods: List[nn.Module] = [nn.Flatten()] if lead_flatten else []
    widths = [n_in] + list(sizes)
    mods.append(nn.Linear(widths[0], widths[1]))
    for a, b in zip(widths[1:-1], widths[2:]):
        mods.extend([nn.ELU(inplace=True), nn.Linear(a, b)])
    mods.append(nn.Linear(widths[-1], n_out))
    return nn.ModuleList(mods)


def _run_stack(stack, h: torch.Tensor) -> torch.Tensor:
    for m in stack:
        h = m(h)
    return h


def _sir_flux(rates: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """[-b S I, b S I - g I, g I] with rates (N,R,2) = [b, g] (lib/models.py:139-142)."""
    infect = rates[..., 0] * x[..., 0] * x[..., 1]
    recover = rates[..., 1] * x[..., 1]
    return torch.stack([-infect, infect - recover, recover], dim=-1)


def _finish(flux3: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Append zero derivatives for dims >= 3 and zero entries outside [-1, 2]."""
    res = torch.cat([flux3, torch.zeros_like(x[..., 3:])], -1)
    res[(x > 2) | (x < -1)] = 0.0
    return res


class _FusedList(list):
    """Per-evaluation entries materialised from a fused solve (``materialize_tracking``): the
    reference's list contents for readers.  ``posterior()`` takes those evaluations from the
    solve's exact sufficient statistics instead, so they are not counted twice; entries appended
    by eager evaluations (evaluation kernel, autograd dopri5, euler ...) are not in ``fused_ids``
    and are pooled as usual."""

    def __init__(self, *args):
        super().__init__(*args)
        self.fused_ids = set()


def eager_params(params) -> list:
    """The entries of a ``params`` list that no fused solve's statistics already cover."""
    if isinstance(params, _FusedList):
        return [p for p in params if id(p) not in params.fused_ids]
    return list(params)


class _TrackerView(torch.autograd.Function):
    """Materialised A-net outputs of every evaluation (E, N, R, 3) whose gradient is handed to
    the solve as d |Fa| (the kernel back-propagates d|Fa|/dFa = Fa / |Fa| through every
    evaluation).  Exact for functions of the norm, torch.norm(torch.stack(tracker)) being the
    reference's only use (lib/VAE.py:180); other functions of the entries get that projection."""

    @staticmethod
    def forward(ctx, fa_norm, fa_all):
        ctx.save_for_backward(fa_norm, fa_all)
        return fa_all.clone()

    @staticmethod
    def backward(ctx, g):
        fa_norm, fa_all = ctx.saved_tensors
        nrm = fa_norm.reshape(())
        d = torch.where(nrm > 0, (g.double() * fa_all.double()).sum() / nrm.double(),
                        torch.zeros((), dtype=torch.float64, device=g.device)).to(fa_norm.dtype)
        return d.reshape(fa_norm.shape), None


class _NormOfOne(torch.autograd.Function):
    """torch.norm of one non-negative value (the solve's |Fa|): the value itself, as a view.  Its
    cotangent goes back unchanged -- d|x|/dx = 1 for x > 0; at |Fa| = 0 the kernel ignores d|Fa|, as
    torch's norm backward gives 0 there."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return x.view(())

    @staticmethod
    def backward(ctx, g):
        return g.view(ctx.shape)


class FaNormEntry(torch.Tensor):
    """``tracker`` entry of a fused solve: its |Fa| (one value, the norm of every A-net output of the
    solve).  The reference reads the tracker as ``torch.norm(torch.stack(ode.tracker))`` (lib/VAE.py:180)
    -- the norm of all entries together.  For a tracker of ONE such entry that expression is the entry
    itself: stack is served as a view and the norm by ``_NormOfOne`` (no device operators, the
    cotangent handed straight to the solve's d|Fa|).  Everything else -- several entries, other norms,
    any other operator -- runs the stock operators on plain tensors."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is torch.stack and len(args) >= 1 and isinstance(args[0], (list, tuple)) and len(args[0]) == 1 \
                and isinstance(args[0][0], FaNormEntry) and args[0][0].numel() == 1 and "out" not in kwargs:
            dim = kwargs.get("dim", args[1] if len(args) > 1 else 0)
            with torch._C.DisableTorchFunctionSubclass():
                v = args[0][0].unsqueeze(dim)
            return v.as_subclass(FaNormEntry)
        if func in (torch.norm, torch.Tensor.norm, torch.linalg.vector_norm) and len(args) >= 1 \
                and isinstance(args[0], FaNormEntry) and args[0].numel() == 1 and len(args) == 1 \
                and all(kwargs.get(k) in (None, "fro", 2, 2.0) for k in ("p", "ord")) \
                and all(kwargs.get(k) is None for k in ("dim", "dtype", "out")) and not kwargs.get("keepdim"):
            with torch._C.DisableTorchFunctionSubclass():
                return _NormOfOne.apply(args[0])
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **kwargs)


class _UDEModule(nn.Module):
    """Shared tracking / posterior logic of the three RHS classes."""

    ode_type = "FaFp"
    uncertainty = "none"
    # forward(t, x) on a HIP device: one gfx950 kernel per evaluation (ude_amd/eval_rhs.py)
    fused_eval = True
    # opt-in: after a fused solve, fill ``params`` / ``tracker`` with one (N, R, 2) rate tensor /
    # one (N, R, 3) A-net tensor per RHS evaluation, as the reference's forward appends them
    # (lib/models.py:137, :187, :238, :252); recomputed from the solve's stage checkpoints
    materialize_tracking = False

    def _init_tracking(self):
        self.params = []
        self.tracker = []
        self._fused_rates: List[Tuple[float, torch.Tensor, torch.Tensor]] = []
        # (n_eval, stats, fp64 sums) of every fused solve that reported its sums (``_record_fused``)
        self._fused_sums: List[Tuple[float, torch.Tensor, torch.Tensor]] = []

    # ``params`` is the list of recorded rates (lib/models.py:137).  A fused solve records its rates
    # as sufficient statistics (``_fused_rates``) next to that list, so assigning a new list -- the
    # reference's reset idiom ``ode.params = []`` (tuning/tune_Fp.py:88), which drops every rate the
    # module has recorded -- drops those statistics too; ``posterior()`` then pools only the solves
    # that ran after the assignment, as the reference's list does.
    @property
    def params(self):
        return self._params

    @params.setter
    def params(self, value):
        self._params = value
        self._fused_rates = []
        self._fused_sums = []

    def clear_tracking(self):
        """Resets the trackers (lib/models.py:148-150)."""
        self.params = []              # also drops the fused solves' rate statistics
        self.tracker = []

    # -- fused-solver side statistics ------------------------------------------
    def _record_fused(self, stats, n_eval: int, evals=None, sums=None) -> None:
        """stats = (mean (2), std (2), |Fa| (1)) of one fused solve -- its three outputs (or a legacy
        [mean_b, mean_g, std_b, std_g, |Fa|] vector); evals = the materialised (rates (E, N, R, 2),
        Fa (E, N, R, 3)) of its evaluations, or None; sums = the solve's fp64 totals (sum b, sum g,
        sum b^2, sum g^2, sum Fa^2), read by the data-parallel statistics exchange
        (distributed.sync_side_stats).  The solve's outputs are used as they are: posterior() and the
        tracker norm add no device operator between the solve and the loss."""
        from .fused import split_stats
        s_mean, s_std, s_fa = split_stats(stats)
        if sums is not None and evals is None:
            self._fused_sums.append((float(n_eval), (s_mean, s_std, s_fa), sums))
        if self.ode_type in ("Fp", "FaFp"):
            self._fused_rates.append((float(n_eval), s_mean, s_std))
            if evals is not None:
                if not isinstance(self.params, _FusedList):
                    self._params = _FusedList(self.params)     # the same rates: no reset
                entries = evals[0].unbind(0)
                self.params.extend(entries)
                self.params.fused_ids.update(id(e) for e in entries)
        if self.ode_type in ("Fa", "FaFp"):
            if evals is not None:
                self.tracker.extend(_TrackerView.apply(s_fa, evals[1]).unbind(0))
            else:
                # torch.norm(torch.stack(tracker)) over this entry == |Fa| of the solve,
                # and over several entries == the norm of all of them together.
                self.tracker.append(s_fa.as_subclass(FaNormEntry))

    @torch.no_grad()
    def _evals_from_checkpoint(self, ckpt: torch.Tensor, y0: torch.Tensor, n_steps: int, chunk: int = 64):
        """Every evaluation's rates / A-net output, recomputed from the stage inputs the
        training forward checkpoints ([tile][step][stage][3R][16], include/ude_rk4.h) and the
        static latent dims of y0."""
        N, R, L = y0.shape
        tiles = (N + 15) // 16
        E = 4 * n_steps
        dyn = ckpt[: tiles * n_steps * 4 * 3 * R * 16].view(tiles, E, 3 * R, 16)
        static = y0.detach()[..., 3:]
        rates = torch.empty((E, N, R, 2), dtype=y0.dtype, device=y0.device) if self.ode_type != "Fa" else None
        fas = torch.empty((E, N, R, 3), dtype=y0.dtype, device=y0.device) if self.ode_type != "Fp" else None
        for e0 in range(0, E, chunk):
            e1 = min(E, e0 + chunk)
            d = dyn[:, e0:e1].permute(1, 0, 3, 2).reshape(e1 - e0, tiles * 16, R, 3)[:, :N]
            x = torch.cat([d, static.unsqueeze(0).expand(e1 - e0, N, R, L - 3)], -1).reshape(-1, R, L)
            if rates is not None:
                rates[e0:e1] = torch.abs(_run_stack(self._p_stack(), x)).reshape(e1 - e0, N, R, 2)
            if fas is not None:
                h = x if self.ode_type == "FaFp" else self.flatten(x)
                fas[e0:e1] = _run_stack(self._a_stack(), h).reshape(e1 - e0, N, R, 3)
        return rates, fas

    def posterior(self) -> Normal:
        """Normal(mean, unbiased std) of every recorded rate; clears them (:152-156)."""
        groups = []
        eager = eager_params(self.params)
        if eager:
            p = torch.stack(eager).reshape(-1, 2)
            groups.append((float(p.shape[0]), p.mean(0), p.std(0)))
        groups.extend(self._fused_rates)
        self.params = []              # clears the fused solves' statistics with the list
        if not groups:
            torch.stack([])  # same error as the reference on an empty tracker
        if len(groups) == 1:
            _, m, s = groups[0]
        else:
            n_tot = sum(g[0] for g in groups)
            m = sum(g[0] * g[1] for g in groups) / n_tot
            ss = sum((g[0] - 1.0) * g[2] ** 2 + g[0] * (g[1] - m) ** 2 for g in groups)
            s = torch.sqrt(ss / (n_tot - 1.0))
        # Normal's argument validation reads the device values back (two host syncs
        # per training step on a HIP device); it stays on for host tensors
        return Normal(m, s, validate_args=False if m.is_cuda else None)

    # -- description consumed by the fused solver -----------------------------
    def ude_config(self):
        net = tuple(self._p_sizes) if self.ode_type in ("Fp", "FaFp") else None
        aug = tuple(self._a_sizes) if self.ode_type in ("Fa", "FaFp") else None
        return (self.ode_type, self.n_regions, self.latent_dim, net, aug)

    def ude_linears(self) -> List[nn.Linear]:
        """Linears in C-ABI order: rate net layers, then augmentation net layers."""
        out: List[nn.Linear] = []
        if self.ode_type in ("Fp", "FaFp"):
            out += [m for m in self._p_stack() if isinstance(m, nn.Linear)]
        if self.ode_type in ("Fa", "FaFp"):
            out += [m for m in self._a_stack() if isinstance(m, nn.Linear)]
        return out

    def fa_weight(self) -> float:
        return float(getattr(self, "Fa_w", 1.0))

    def ude_weight_shapes(self) -> List[torch.Size]:
        """Shapes of (W, b) per Linear in C-ABI order."""
        out: List[torch.Size] = []
        for lin in self.ude_linears():
            out += [lin.weight.shape, lin.bias.shape]
        return out

    def _eval_weights(self) -> List[torch.Tensor]:
        out: List[torch.Tensor] = []
        for lin in self.ude_linears():
            out += [lin.weight, lin.bias]
        return out

    def _fused_forward(self, x: torch.Tensor):
        """forward() on the gfx950 evaluation kernel when x lives on a HIP device (else None):
        the same return value and the same params / tracker entries as the eager code."""
        if not (x.is_cuda and self.fused_eval):
            return None
        from . import eval_rhs
        if not eval_rhs.eligible(self, x):
            return None
        f, rates, fa = eval_rhs.rhs_eval(self, x, self._eval_weights())
        if rates is not None:
            self.params.append(rates)
        if fa is not None:
            self.tracker.append(fa)
        return f


class Fp(_UDEModule):
    """Physics RHS with MLP-learned SIR rates ("CONN"), lib/models.py:109-156."""

    def __init__(self, n_regions=1, latent_dim=8, net_sizes=[20, 20], **kwargs):
        super().__init__()
        self.n_regions = n_regions
        self.latent_dim = latent_dim
        self.ode_type = "Fp"
        self.uncertainty = "none"
        self._p_sizes = list(net_sizes)
        self.Fp_net = _linear_stack(n_regions * latent_dim, net_sizes, 2 * n_regions, lead_flatten=True)
        self._init_tracking()

    def _p_stack(self):
        return self.Fp_net

    def forward(self, t, x):
        f = self._fused_forward(x)
        if f is not None:
            return f
        rates = torch.abs(_run_stack(self.Fp_net, x)).reshape(-1, self.n_regions, 2)
        self.params.append(rates)
        return _finish(_sir_flux(rates, x), x)


class Fa(_UDEModule):
    """Pure MLP RHS ("SONN"), lib/models.py:158-197."""

    def __init__(self, n_regions=1, latent_dim=8, net_sizes=[32, 32], aug_net_sizes=[32, 32], nhidden_fa=32,
                 **kwargs):
        super().__init__()
        self.ode_type = "Fa"
        self.uncertainty = "none"
        self.n_regions = n_regions
        self.latent_dim = latent_dim
        self.flatten = nn.Flatten()
        self._a_sizes = list(aug_net_sizes)
        self.aug_net = _linear_stack(n_regions * latent_dim, aug_net_sizes, 3 * n_regions, lead_flatten=False)
        self._init_tracking()

    def _a_stack(self):
        return self.aug_net

    def forward(self, t, x):
        f = self._fused_forward(x)
        if f is not None:
            return f
        fa = _run_stack(self.aug_net, self.flatten(x)).reshape(-1, self.n_regions, 3)
        res = _finish(fa, x)
        self.tracker.append(fa)
        return res


class FaFp(_UDEModule):
    """Physics + MLP augmentation RHS ("UONN"), lib/models.py:199-265."""

    def __init__(self, n_regions=1, latent_dim=8, net_sizes=[20, 20], aug_net_sizes=[32, 32], **kwargs):
        super().__init__()
        self.n_regions = n_regions
        self.latent_dim = latent_dim
        self.ode_type = "FaFp"
        self.uncertainty = "none"
        self._p_sizes = list(net_sizes)
        self._a_sizes = list(aug_net_sizes)
        self.net = _linear_stack(n_regions * latent_dim, net_sizes, 2 * n_regions, lead_flatten=True)
        self.aug_net = _linear_stack(n_regions * latent_dim, aug_net_sizes, 3 * n_regions, lead_flatten=True)
        self.Fa_w = 1.0
        self._init_tracking()

    def _p_stack(self):
        return self.net

    def _a_stack(self):
        return self.aug_net

    def forward(self, t, x):
        f = self._fused_forward(x)
        if f is not None:
            return f
        rates = torch.abs(_run_stack(self.net, x)).reshape(-1, self.n_regions, 2)
        self.params.append(rates)
        fa = _run_stack(self.aug_net, x).reshape(-1, self.n_regions, 3)
        res = _finish(_sir_flux(rates, x) + self.Fa_w * fa, x)
        self.tracker.append(fa)
        return res


UDE_CLASSES = (Fp, Fa, FaFp)
