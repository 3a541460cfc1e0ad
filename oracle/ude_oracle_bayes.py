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
    # test instrumentation: "rev4" / "fwd4" sum every Linear's K products in blocks of 4, last / first
    # block first (more samples of fp32 rounding, as OracleRHS.k_order)
    k_order: str = "torch"

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

    def _linear(self, h, w, b):
        if self.k_order[:3] not in ("rev", "fwd"):
            return torch.nn.functional.linear(h, w, b)
        K, kb = h.shape[-1], int(self.k_order[3:])
        acc = b.expand(h.shape[:-1] + (w.shape[0],))
        blocks = range(0, K, kb)
        for k0 in (reversed(blocks) if self.k_order.startswith("rev") else blocks):
            acc = acc + h[..., k0:k0 + kb] @ w[:, k0:k0 + kb].T
        return acc

    def _mlp(self, h, wb):
        k = len(wb) // 2
        for i in range(k):
            h = self._linear(h, wb[2 * i], wb[2 * i + 1])
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


def _bayes_chunk_stats(args):
    """Pass 1 of ``solve_and_grad_bayes_chunked`` for one chunk: latent and fp64 side-statistic sums."""
    rhs, eps, y0c, t, step_size, threads = args
    if threads:
        torch.set_num_threads(threads)
    with torch.no_grad():
        rhs.clear_tracking()
        rhs.eps = eps
        lat = odeint_rk4(rhs, y0c, t, step_size)
        out = {"latent": lat}
        if rhs.params:
            p = torch.stack(rhs.params).reshape(-1, 2).double()
            out["n"], out["s1"], out["s2"] = p.shape[0], p.sum(0), p.pow(2).sum(0)
        if rhs.tracker:
            out["sf"] = float(torch.stack(rhs.tracker).double().pow(2).sum())
    rhs.clear_tracking()
    return out


def _bayes_chunk_grad(args):
    """Pass 2: the chunk's share of the loss gradient (the side statistics held at their global
    values, as oracle/ude_oracle.py _chunk_grad): d y0 of the chunk, d mean / d raw std of every layer."""
    rhs, eps, y0c, t, step_size, dlc, dmean, dstd, dnorm, mean, std, norm, n, threads = args
    if threads:
        torch.set_num_threads(threads)
    dt = y0c.dtype
    mu, sd = rhs.mu_sd()
    for w in mu + sd:
        w.requires_grad_(True)
    yc = y0c.detach().clone().requires_grad_(True)
    rhs.clear_tracking()
    rhs.eps = eps
    lat = odeint_rk4(rhs, yc, t, step_size)
    loss = (lat * dlc.to(dt)).sum()
    if mean is not None and dmean is not None:
        p = torch.stack(rhs.params).reshape(-1, 2)
        m, s = mean.to(dt), std.to(dt)
        loss = loss + (p.sum(0) * dmean.to(dt) / n).sum() \
            + ((p - m).pow(2).sum(0) * dstd.to(dt) / (2.0 * (n - 1) * s)).sum()
    if norm is not None and dnorm is not None and float(norm) > 0:
        loss = loss + dnorm * torch.stack(rhs.tracker).pow(2).sum() / (2.0 * norm.to(dt))
    g = torch.autograd.grad(loss, [yc] + mu + sd, allow_unused=True)
    rhs.clear_tracking()
    for w in mu + sd:
        w.requires_grad_(False)
    return [torch.zeros_like(v) if gi is None else gi.detach() for gi, v in zip(g, [yc] + mu + sd)]


def solve_and_grad_bayes_chunked(rhs: OracleBayesRHS, eps: torch.Tensor, y0: torch.Tensor, t: torch.Tensor,
                                 step_size, dlatent: Optional[torch.Tensor], dmean=None, dstd=None, dnorm=None,
                                 chunk: int = 256, workers: int = 1):
    """``solve_and_grad_bayes`` over trajectory chunks on ``workers`` spawned CPU processes (full-size
    batches; every chunk draws the same eps rows -- a weight sample is shared by the whole batch within
    one evaluation, models_bayes.py:43-48).  Exact: the side statistics couple the trajectories only
    through their global values (pass 1), their gradient is linear in per-trajectory terms once those
    are known (pass 2; oracle/ude_oracle.py solve_and_grad_chunked).  Returns dict(latent, mean, std,
    fa_norm, grads = {y0, mu, sd})."""
    import math
    N = y0.shape[0]
    dt = y0.dtype
    starts = list(range(0, N, chunk))
    threads = max(1, torch.get_num_threads() // workers) if workers > 1 else 0

    def run(fn, jobs):
        if workers <= 1:
            return [fn(j) for j in jobs]
        import multiprocessing as mp
        from concurrent.futures import ProcessPoolExecutor
        with ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
            return list(ex.map(fn, jobs))

    rhs.clear_tracking()
    st = run(_bayes_chunk_stats, [(rhs, eps, y0[c0:c0 + chunk], t, step_size, threads) for c0 in starts])
    out = {"latent": torch.cat([s["latent"] for s in st], 1)}
    mean = std = norm = None
    n = 0
    if "s1" in st[0]:
        n = sum(s["n"] for s in st)
        s1 = sum(s["s1"] for s in st)
        s2 = sum(s["s2"] for s in st)
        mean = s1 / n
        std = torch.sqrt(torch.clamp(s2 - n * mean * mean, min=0.0) / (n - 1))
        out["mean"], out["std"] = mean.to(dt), std.to(dt)
    if "sf" in st[0]:
        norm = torch.tensor(math.sqrt(sum(s["sf"] for s in st)), dtype=torch.float64)
        out["fa_norm"] = norm.to(dt).reshape(1)
    if dlatent is None:
        return out
    gl = run(_bayes_chunk_grad, [(rhs, eps, y0[c0:c0 + chunk], t, step_size, dlatent[:, c0:c0 + chunk], dmean, dstd,
                                  dnorm, mean, std, norm, n, threads) for c0 in starts])
    n_mu = len(rhs.mu_sd()[0])
    acc = [sum(g[1 + i] for g in gl[1:]) + gl[0][1 + i] if len(gl) > 1 else gl[0][1 + i] for i in range(2 * n_mu)]
    out["grads"] = {"y0": torch.cat([g[0] for g in gl], 0), "mu": acc[:n_mu], "sd": acc[n_mu:]}
    return out
