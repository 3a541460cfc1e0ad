"""Bayesian UDE right-hand sides (lib/in_development/models_bayes.py:12-265).

Every Linear is a ``Dense_Variational``: on EACH call a fresh weight sample
``w = mu + eps * |sigma|`` (:43-48), so every RHS evaluation inside a solve
sees new weights.  Same names, constructor signatures, ``state_dict`` keys
(``w_mean``, ``w_std``, ``b_mean``, ``b_std``) and ``get_kl`` as the reference.

Called directly (or by a non-fused solver) a module draws its noise with
``torch.randn_like`` per layer per call, as the reference.  Inside
``odeint(..., method='rk4')`` on a HIP device the whole solve runs in the fused
gfx950 kernel instead (``fused.FusedBayesRK4``): the solve's draws are one
``(4 * n_steps, n_params)`` standard-normal stream -- row e for RHS evaluation e,
each row in the order the reference's layers call ``make_z`` within one
evaluation (torch parameter order) -- from torch's generator on the device, or
the stream set with ``set_eps_stream`` (used by the parity tests to inject the
reference's draws).
"""
from __future__ import annotations

import contextlib

import math
from typing import List, Optional, Tuple

import torch
from torch import nn
import torch.distributions as dist

from .rhs import _UDEModule, _finish, _run_stack, _sir_flux


class Dense_Variational(nn.Module):
    def __init__(self, in_features, out_features, bias=True, prior_std=1.0):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.prior_std = prior_std
        self.w_mean = nn.Parameter(torch.empty(out_features, in_features))
        self.w_std = nn.Parameter(torch.empty(out_features, in_features))
        if bias:
            self.bias = True
            self.b_mean = nn.Parameter(torch.empty(out_features))
            self.b_std = nn.Parameter(torch.empty(out_features))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.kaiming_uniform_(self.w_mean, a=math.sqrt(5))
        nn.init.constant_(self.w_std, 0.1)
        if self.bias is not None:
            bound = 1.0 / math.sqrt(self.in_features)
            nn.init.uniform_(self.b_mean, -bound, bound)
            nn.init.constant_(self.b_std, 0.1)

    def make_z(self):
        with torch.no_grad():
            self.z = [torch.randn_like(self.w_mean), torch.randn_like(self.b_mean)]

    def forward(self, x):
        self.make_z()
        w = self.w_mean + self.z[0] * torch.abs(self.w_std)
        b = self.b_mean + self.z[1] * torch.abs(self.b_std)
        return nn.functional.linear(x, w, b)

    def make_prior(self):
        s = self.prior_std
        self.prior = [dist.Normal(torch.zeros_like(self.w_mean), s * torch.ones_like(self.w_mean)),
                      dist.Normal(torch.zeros_like(self.b_mean), s * torch.ones_like(self.b_mean))]
        return self.prior

    def make_posterior(self):
        self.posterior = [dist.Normal(self.w_mean, torch.abs(self.w_std)),
                          dist.Normal(self.b_mean, torch.abs(self.b_std))]
        return self.posterior

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"


def _variational_stack(n_in, sizes, n_out, prior_std, lead_flatten=True):
    mods = [nn.Flatten()] if lead_flatten else []
    widths = [n_in] + list(sizes)
    mods.append(Dense_Variational(widths[0], widths[1], prior_std=prior_std))
    for a, b in zip(widths[1:-1], widths[2:]):
        mods.extend([nn.ELU(inplace=True), Dense_Variational(a, b, prior_std=prior_std)])
    mods.append(Dense_Variational(widths[-1], n_out, prior_std=prior_std))
    return nn.ModuleList(mods)


def _kl_of(stacks):
    total, count = 0, 0
    for stack in stacks:
        for layer in stack:
            if isinstance(layer, Dense_Variational):
                kls = [dist.kl_divergence(q, p).mean() for q, p in zip(layer.make_posterior(), layer.make_prior())]
                total = total + sum(kls) / 2
                count += 1
    return total / count


class _BayesBase(_UDEModule):
    uncertainty = "bayes"

    # -- description consumed by the fused solver ---------------------------------
    def ude_config(self):
        kind, R, L, net, aug = super().ude_config()
        return ("B" + kind, R, L, net, aug)

    def _variational(self) -> List[Dense_Variational]:
        out: List[Dense_Variational] = []
        if self.ode_type in ("Fp", "FaFp"):
            out += [m for m in self.Fp_net if isinstance(m, Dense_Variational)]
        if self.ode_type in ("Fa", "FaFp"):
            out += [m for m in self.aug_net if isinstance(m, Dense_Variational)]
        return out

    def ude_mean_std(self) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
        """(means, stds) in C-ABI / torch order: per layer weight then bias, rate net first."""
        mus, sds = [], []
        for lay in self._variational():
            mus += [lay.w_mean, lay.b_mean]
            sds += [lay.w_std, lay.b_std]
        return mus, sds

    def ude_weight_shapes(self) -> List[torch.Size]:
        return [p.shape for p in self.ude_mean_std()[0]]

    def _eval_weights(self):
        """This evaluation's weight sample, drawn and formed by the layers exactly as their
        forward does (make_z per layer in call order; w = mean + z * |std|, :43-48) -- or, with
        a stream set by ``set_eps_stream``, its next row (torch parameter order per layer) --
        or, inside a fixed-grid solve (``presampled``), the next pre-formed sample row."""
        pre = getattr(self, "_presampled", None)
        if pre is not None:
            k = self._pre_row
            if k >= len(pre):
                raise RuntimeError(f"presampled weights: evaluation {k + 1} of a solve drawn for {len(pre)}")
            self._pre_row = k + 1
            return pre[k]
        eps = getattr(self, "_eps_next", None)
        row = None
        if eps is not None:
            k = getattr(self, "_eps_row", 0)
            row = eps[k]
            self._eps_row = k + 1
            if self._eps_row >= eps.shape[0]:
                self._eps_next, self._eps_row = None, 0
        out: List[torch.Tensor] = []
        off = 0
        for lay in self._variational():
            if row is None:
                lay.make_z()
            else:
                nw, nb = lay.w_mean.numel(), lay.b_mean.numel()
                lay.z = [row[off:off + nw].view_as(lay.w_mean), row[off + nw:off + nw + nb].view_as(lay.b_mean)]
                off += nw + nb
            out += [lay.w_mean + lay.z[0] * torch.abs(lay.w_std), lay.b_mean + lay.z[1] * torch.abs(lay.b_std)]
        return out

    def _nets(self, x):
        """Eager evaluation of the nets: (rates (N, R, 2) or None, Fa (N, R, 3) or None).  The layers
        draw their own z (make_z, models_bayes.py:30-32, :43-48); with an eps stream set
        (``set_eps_stream``) the evaluation takes its next row instead, in the layers' call order."""
        R = self.n_regions
        wb = self._eval_weights() if getattr(self, "_eps_next", None) is not None else None

        def run(stack, h, k):
            for m in stack:
                if wb is not None and isinstance(m, Dense_Variational):
                    h = nn.functional.linear(h, wb[k], wb[k + 1])
                    k += 2
                else:
                    h = m(h)
            return h, k

        rates = fa = None
        k = 0
        if self.ode_type in ("Fp", "FaFp"):
            h, k = run(self.Fp_net, x, k)
            rates = torch.abs(h).reshape(-1, R, 2)
        if self.ode_type in ("Fa", "FaFp"):
            h, k = run(self.aug_net, x, k)
            fa = h.reshape(-1, R, 3)
        return rates, fa

    @torch.no_grad()
    def _evals_from_checkpoint(self, ckpt: torch.Tensor, y0: torch.Tensor, n_steps: int, eps: torch.Tensor = None):
        """``materialize_tracking`` for the Bayesian RHS: every evaluation's rates / A-net output,
        recomputed from the stage inputs the training forward checkpoints and evaluation e's own
        weight sample w_e = mean + eps[e] |std| (the row the whole-solve kernel used)."""
        N, R, L = y0.shape
        tiles = (N + 15) // 16
        E = 4 * n_steps
        dyn = ckpt[: tiles * n_steps * 4 * 3 * R * 16].view(tiles, E, 3 * R, 16)
        static = y0.detach()[..., 3:]
        mus, sds = self.ude_mean_std()
        mu = torch.cat([p.detach().reshape(-1) for p in mus])
        sd = torch.cat([p.detach().reshape(-1).abs() for p in sds])
        shapes = [p.shape for p in mus]
        rates = torch.empty((E, N, R, 2), dtype=y0.dtype, device=y0.device) if self.ode_type != "Fa" else None
        fas = torch.empty((E, N, R, 3), dtype=y0.dtype, device=y0.device) if self.ode_type != "Fp" else None

        def run(stack, h, wb, k):
            for m in stack:
                if isinstance(m, Dense_Variational):
                    h = nn.functional.linear(h, wb[k], wb[k + 1])
                    k += 2
                else:
                    h = m(h)
            return h, k

        for e in range(E):
            flat = mu + eps[e].to(mu) * sd
            wb, off = [], 0
            for shp in shapes:
                n = 1
                for v in shp:
                    n *= v
                wb.append(flat[off:off + n].view(shp))
                off += n
            d = dyn[:, e].permute(0, 2, 1).reshape(tiles * 16, R, 3)[:N]
            x = torch.cat([d, static], -1)
            k = 0
            if rates is not None:
                h, k = run(self.Fp_net, x, wb, k)
                rates[e] = torch.abs(h).reshape(N, R, 2)
            if fas is not None:
                h, k = run(self.aug_net, x, wb, k)
                fas[e] = h.reshape(N, R, 3)
        return rates, fas

    def set_eps_stream(self, eps: Optional[torch.Tensor]) -> None:
        """Use ``eps`` ((4 * n_steps, n_params)) as the draws of the next solve: the fused
        whole-solve kernel takes all of it, evaluations one at a time take a row each."""
        self._eps_next = eps
        self._eps_row = 0

    @contextlib.contextmanager
    def presampled(self, n_eval: int, device):
        """Draw the weight samples of a whole solve's ``n_eval`` evaluations at once --
        ``w = mean + eps * |std|`` on the (n_eval, n_params) stream ``take_eps`` hands the
        fused whole-solve kernel (same rows, same fp32 ops as one evaluation at a time) -- and
        serve evaluation e row e.  Three device operators per solve instead of four per layer
        per evaluation, and one gradient reduction over the rows instead of an accumulation
        per evaluation (autograd: mean and std receive the row gradients through the stack)."""
        mus, sds = self.ude_mean_std()
        n_par = sum(int(p.numel()) for p in mus)
        eps = self.take_eps(n_eval, n_par, device)
        mu = torch.cat([p.reshape(-1) for p in mus])
        sd = torch.cat([p.reshape(-1) for p in sds])
        self._presampled, self._pre_row = (mu + eps * torch.abs(sd)).unbind(0), 0
        try:
            yield
        finally:
            self._presampled = None

    def take_eps(self, n_eval: int, n_params: int, device) -> torch.Tensor:
        eps = getattr(self, "_eps_next", None)
        self._eps_next = None
        if eps is None:
            return torch.randn((n_eval, n_params), device=device)
        if tuple(eps.shape) != (n_eval, n_params):
            raise ValueError(f"eps stream has shape {tuple(eps.shape)}, the solve needs {(n_eval, n_params)}")
        return eps.to(device=device, dtype=torch.float32)


class Bayes_Fp(_BayesBase):
    def __init__(self, n_regions=1, latent_dim=8, net_sizes=[20, 20], prior_std=0.1, **kwargs):
        super().__init__()
        self.n_regions, self.latent_dim = n_regions, latent_dim
        self.ode_type, self.uncertainty = "Fp", "bayes"
        self._p_sizes = list(net_sizes)
        self.Fp_net = _variational_stack(n_regions * latent_dim, net_sizes, 2 * n_regions, prior_std)
        self._init_tracking()

    def forward(self, t, x):
        f = self._fused_forward(x)
        if f is not None:
            return f
        rates, _ = self._nets(x)
        self.params.append(rates)
        return _finish(_sir_flux(rates, x), x)

    def get_kl(self):
        return _kl_of([self.Fp_net])


class Bayes_Fa(_BayesBase):
    def __init__(self, n_regions=1, latent_dim=8, aug_net_sizes=[32, 32], nhidden_fa=32, prior_std=0.1, **kwargs):
        super().__init__()
        self.n_regions, self.latent_dim = n_regions, latent_dim
        self.ode_type, self.uncertainty = "Fa", "bayes"
        self._a_sizes = list(aug_net_sizes)
        self.aug_net = _variational_stack(n_regions * latent_dim, aug_net_sizes, 3 * n_regions, prior_std)
        self._init_tracking()

    def forward(self, t, x):
        f = self._fused_forward(x)
        if f is not None:
            return f
        _, fa = self._nets(x)
        res = _finish(fa, x)
        self.tracker.append(fa)
        return res

    def get_kl(self):
        return _kl_of([self.aug_net])


class Bayes_FaFp(_BayesBase):
    def __init__(self, n_regions=1, latent_dim=8, net_sizes=[20, 20], aug_net_sizes=[32, 32], prior_std=0.1,
                 **kwargs):
        super().__init__()
        self.n_regions, self.latent_dim = n_regions, latent_dim
        self.ode_type, self.uncertainty = "FaFp", "bayes"
        self._p_sizes, self._a_sizes = list(net_sizes), list(aug_net_sizes)
        self.Fp_net = _variational_stack(n_regions * latent_dim, net_sizes, 2 * n_regions, prior_std)
        self.aug_net = _variational_stack(n_regions * latent_dim, aug_net_sizes, 3 * n_regions, prior_std)
        self.Fa_w = 1.0
        self._init_tracking()

    def forward(self, t, x):
        f = self._fused_forward(x)
        if f is not None:
            return f
        rates, fa = self._nets(x)
        self.params.append(rates)
        res = _finish(_sir_flux(rates, x) + self.Fa_w * fa, x)
        self.tracker.append(fa)
        return res

    def get_kl(self):
        return _kl_of([self.Fp_net, self.aug_net])
