"""CPU oracle for the Bayesian UDE right-hand sides -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.

Restates ``lib/in_development/models_bayes.py``:

* ``Dense_Variational.forward`` (:43-48): a fresh weight sample
  ``w = w_mean + z_w * |w_std|``, ``b = b_mean + z_b * |b_std|`` on EVERY call
  (``make_z`` :30-32 draws ``z`` with ``randn_like``), then ``linear``;
* ``Bayes_Fp.forward`` (:88-105), ``Bayes_Fa.forward`` (:151-162),
  ``Bayes_FaFp.forward`` (:216-240): the same RHS algebra as the deterministic
  classes (``|.|`` rates -> SIR flux, ``Fp + Fa_w * Fa``, zero derivative for
  latent dims >= 3, zero outside ``[-1, 2]``), with the layer rule of
  :78-84 (ELU between consecutive hidden layers only).

The random draws are INJECTED: ``eps`` is a ``(E, n_params)`` tensor in torch
parameter order (per layer: ``w`` then ``b``; rate net first, then the
augmentation net), row ``e`` feeding the ``e``-th RHS evaluation of the solve
-- the order in which the reference's layers call ``make_z`` within one
evaluation.  The fused kernel takes the same stream, so both sides see the
same weight samples (torch's RNG stream itself is not reproduced).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import torch

from .ude_oracle import odeint_rk4


@dataclass
class OracleBayesRHS:
    """Variational weights of one Bayes_* RHS in nn.Linear layout (out, in)."""
    kind: str                       # 'Fp' | 'Fa' | 'FaFp'
    n_regions: int
    latent_dim: int
    p_mu: List[torch.Tensor] = field(default_factory=list)     # [w0, b0, w1, b1, ...]
    p_sd: List[torch.Tensor] = field(default_factory=list)
    a_mu: List[torch.Tensor] = field(default_factory=list)
    a_sd: List[torch.Tensor] = field(default_factory=list)
    fa_w: float = 1.0
    eps: Optional[torch.Tensor] = None
    n_calls: int = 0
    params: List[torch.Tensor] = field(default_factory=list)
    tracker: List[torch.Tensor] = field(default_factory=list)

    def mu_sd(self):
        """(means, stds) in torch parameter order (rate net first)."""
        return list(self.p_mu) + list(self.a_mu), list(self.p_sd) + list(self.a_sd)

    def n_params(self) -> int:
        return sum(int(t.numel()) for t in self.mu_sd()[0])

    @classmethod
    def from_module(cls, mod, dtype=None) -> "OracleBayesRHS":
        """Read w_mean / w_std / b_mean / b_std out of a Bayes_* module."""
        def grab(seq):
            mu, sd = [], []
            for m in seq:
                if hasattr(m, "w_mean"):
                    for a, b in ((m.w_mean, m.w_std), (m.b_mean, m.b_std)):
                        a, b = a.detach().clone(), b.detach().clone()
                        if dtype is not None:
                            a, b = a.to(dtype), b.to(dtype)
                        mu.append(a)
                        sd.append(b)
            return mu, sd
        kind = mod.ode_type
        o = cls(kind=kind, n_regions=mod.n_regions, latent_dim=mod.latent_dim)
        if kind in ("Fp", "FaFp"):
            o.p_mu, o.p_sd = grab(mod.Fp_net)
        if kind in ("Fa", "FaFp"):
            o.a_mu, o.a_sd = grab(mod.aug_net)
        o.fa_w = float(getattr(mod, "Fa_w", 1.0))
        return o

    def _sample(self, mu, sd, row, off):
        """Dense_Variational.forward's weight sample (models_bayes.py:45-46)."""
        out = []
        for m, s in zip(mu, sd):
            n = m.numel()
            z = row[off:off + n].reshape(m.shape).to(m.dtype)
            out.append(m + z * torch.abs(s))
            off += n
        return out, off

    @staticmethod
    def _mlp(h, wb):
        k = len(wb) // 2
        for i in range(k):
            h = torch.nn.functional.linear(h, wb[2 * i], wb[2 * i + 1])
            if i < k - 2:
                h = torch.nn.functional.elu(h)
        return h

    def __call__(self, t, x):
        assert self.eps is not None, "inject eps before solving"
        row = self.eps[self.n_calls]
        self.n_calls += 1
        R = self.n_regions
        mask = (x > 2) | (x < -1)
        if getattr(self, "record_masks", False):      # test instrumentation (S, I, R decisions)
            self.masks.append(mask[..., :3].detach().clone())
        flat = x.reshape(x.shape[0], -1)
        off = 0
        if self.kind in ("Fp", "FaFp"):
            wb, off = self._sample(self.p_mu, self.p_sd, row, off)
            p = torch.abs(self._mlp(flat, wb)).reshape(-1, R, 2)
            self.params.append(p)
            plus_i = p[..., 0] * x[..., 0] * x[..., 1]
            minus_i = p[..., 1] * x[..., 1]
            flux = torch.stack([-plus_i, plus_i - minus_i, minus_i], dim=-1)
        if self.kind in ("Fa", "FaFp"):
            wb, off = self._sample(self.a_mu, self.a_sd, row, off)
            fa = self._mlp(flat, wb).reshape(-1, R, 3)
            self.tracker.append(fa)
            flux = fa if self.kind == "Fa" else flux + self.fa_w * fa
        res = torch.cat([flux, torch.zeros_like(x[..., 3:])], -1)
        return torch.where(mask, torch.zeros_like(res), res)

    def clear_tracking(self):
        self.params = []
        self.tracker = []
        self.masks = []
        self.n_calls = 0

    def posterior(self):
        params = torch.stack(self.params).reshape(-1, 2)
        self.params = []
        return torch.distributions.Normal(params.mean(0), params.std(0))


def solve_and_grad_bayes(rhs: OracleBayesRHS, eps: torch.Tensor, y0: torch.Tensor, t: torch.Tensor, step_size,
                         dlatent: Optional[torch.Tensor] = None, dmean=None, dstd=None, dnorm=None):
    """Forward solve with injected eps; with cotangents, the VJP w.r.t. y0, every
    mean and every (raw) std.  Returns dict(latent, mean, std, fa_norm, grads)."""
    want = dlatent is not None
    y0 = y0.detach().clone().requires_grad_(want)
    mu, sd = rhs.mu_sd()
    for p in mu + sd:
        p.requires_grad_(want)
    rhs.clear_tracking()
    rhs.eps = eps
    out = {}
    with torch.set_grad_enabled(want):
        latent = odeint_rk4(rhs, y0, t, step_size)
        assert rhs.n_calls == eps.shape[0], (rhs.n_calls, tuple(eps.shape))
        loss = (latent * dlatent).sum() if want else None
        out["latent"] = latent.detach()
        if rhs.kind in ("Fa", "FaFp"):
            norm = torch.norm(torch.stack(rhs.tracker))
            out["fa_norm"] = norm.detach().reshape(1)
            if want and dnorm is not None:
                loss = loss + dnorm * norm
        if rhs.kind in ("Fp", "FaFp"):
            post = rhs.posterior()
            out["mean"], out["std"] = post.loc.detach(), post.scale.detach()
            if want and dmean is not None:
                loss = loss + (post.loc * dmean).sum() + (post.scale * dstd).sum()
        if want:
            g = torch.autograd.grad(loss, [y0] + mu + sd, allow_unused=True)
            fill = [torch.zeros_like(v) if gi is None else gi.detach() for gi, v in zip(g, [y0] + mu + sd)]
            out["grads"] = {"y0": fill[0], "mu": fill[1:1 + len(mu)], "sd": fill[1 + len(mu):]}
    rhs.clear_tracking()
    return out
