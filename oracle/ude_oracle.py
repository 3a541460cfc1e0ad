"""CPU oracle for the UDE RK4 hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (the package's ``odeint`` on a HIP device) never calls it.

What it restates (pure PyTorch, any dtype, autograd for the VJP):

* the RHS semantics of ``lib/models.py`` -- ``Fp.forward`` (:129-146),
  ``Fa.forward`` (:177-188), ``FaFp.forward`` (:230-254): flattened joint MLP(s),
  ``|.|`` rates -> SIR flux ``[-b S I, b S I - g I, g I]``, ``Fp + Fa_w * Fa``,
  zero derivative for latent dims >= 3, zero where the state is outside
  ``[-1, 2]`` (strict comparisons, :130), and the per-eval tracking of rates
  (``params``, :137/:238) and ``Fa`` (``tracker``, :187/:252);
* ``posterior()`` (:152-156): ``Normal(mean, unbiased std)`` over every
  recorded rate;
* the torchdiffeq fixed-grid RK4 integrator called at ``lib/VAE.py:137`` and
  ``tuning/tune_encoders.py:221``.  torchdiffeq is a third-party dependency
  that is NOT vendored in the reference and NOT installed here (version
  unpinned by the reference).  Its published algorithm is restated from the
  0.2.x sources: ``FixedGridODESolver._grid_constructor_from_step_size``
  (grid = arange(ceil((t1-t0)/h + 1)) * h + t0 with the last point clamped to
  t[-1], all in t's dtype), ``FixedGridODESolver.integrate`` (exact-hit /
  linear interpolation output rule) and ``rk4_alt_step_func`` (Kutta's 3/8
  rule).  Integrator parity is therefore pinned by analytic known-answer
  tests (tests/test_oracle.py), not by torchdiffeq itself.

The oracle is pinned against golden vectors generated in the build container
by running the reference's own RHS classes (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch

ONE_THIRD = 1.0 / 3.0
TWO_THIRDS = 2.0 / 3.0


# ---------------------------------------------------------------------------
# RHS restatement (lib/models.py)
# ---------------------------------------------------------------------------

def mlp_layers(in_dim: int, sizes: Sequence[int], out_dim: int) -> List[Tuple[int, int, bool]]:
    """(in, out, elu_after) per Linear, following lib/models.py:118-124.

    For ``sizes=[h1..hk]``: Lin(in->h1), then ELU+Lin(h_{i-1}->h_i) for i>=2,
    then Lin(hk->out).  So an ELU follows Lin_i only for i < k-1 (0-based):
    the last hidden Linear and the output Linear have no activation.
    """
    dims = [in_dim] + list(sizes) + [out_dim]
    k = len(sizes)
    return [(dims[i], dims[i + 1], i < k - 1) for i in range(k + 1)]


@dataclass
class OracleRHS:
    """Weights of one UDE right-hand side in nn.Linear layout (out, in)."""
    kind: str                      # 'Fp' | 'Fa' | 'FaFp'
    n_regions: int
    latent_dim: int
    p_w: List[torch.Tensor] = field(default_factory=list)
    p_b: List[torch.Tensor] = field(default_factory=list)
    p_act: List[bool] = field(default_factory=list)
    a_w: List[torch.Tensor] = field(default_factory=list)
    a_b: List[torch.Tensor] = field(default_factory=list)
    a_act: List[bool] = field(default_factory=list)
    fa_w: float = 1.0
    params: List[torch.Tensor] = field(default_factory=list)
    tracker: List[torch.Tensor] = field(default_factory=list)
    # test instrumentation: record every evaluation's mask decisions on the S, I, R dims
    # ((x > 2) | (x < -1), lib/models.py:130) -- the RHS is discontinuous there
    record_masks: bool = False
    masks: List[torch.Tensor] = field(default_factory=list)
    margins: List[torch.Tensor] = field(default_factory=list)     # per evaluation: (N,) distance to the boundary
    # test instrumentation: "rev<k>" (k = 2, 4, 8, 16 ...) sums every Linear's K products in blocks of k,
    # last block first, "fwd<k>" first block first (fwd4: the order of an MFMA K chain) -- the same fp32
    # arithmetic with other summation orders (more samples of fp32 rounding)
    k_order: str = "torch"

    def _linear(self, h, w, b):
        if self.k_order[:3] not in ("rev", "fwd"):
            return torch.nn.functional.linear(h, w, b)
        K, kb = h.shape[-1], int(self.k_order[3:])
        acc = b.expand(h.shape[:-1] + (w.shape[0],))
        blocks = range(0, K, kb)
        for k0 in (reversed(blocks) if self.k_order.startswith("rev") else blocks):
            acc = acc + h[..., k0:k0 + kb] @ w[:, k0:k0 + kb].T
        return acc

    def _mlp(self, h, ws, bs, acts):
        for w, b, act in zip(ws, bs, acts):
            h = self._linear(h, w, b)
            if act:
                h = torch.nn.functional.elu(h)
        return h

    def __call__(self, t, x):
        # x: (N, R, L).  Mirrors lib/models.py:230-254 (FaFp) and siblings.
        R = self.n_regions
        mask = (x > 2) | (x < -1)
        if self.record_masks:
            self.masks.append(mask[..., :3].detach().clone())
            xs = x[..., :3].detach()
            self.margins.append(torch.minimum((xs - 2).abs(), (xs + 1).abs()).reshape(x.shape[0], -1).amin(1))
        flat = x.reshape(x.shape[0], -1)
        parts = []
        if self.kind in ("Fp", "FaFp"):
            p = torch.abs(self._mlp(flat, self.p_w, self.p_b, self.p_act)).reshape(-1, R, 2)
            self.params.append(p)
            plus_i = p[..., 0] * x[..., 0] * x[..., 1]
            minus_i = p[..., 1] * x[..., 1]
            flux = torch.stack([-plus_i, plus_i - minus_i, minus_i], dim=-1)
        if self.kind in ("Fa", "FaFp"):
            fa = self._mlp(flat, self.a_w, self.a_b, self.a_act).reshape(-1, R, 3)
            self.tracker.append(fa)
            flux = fa if self.kind == "Fa" else flux + self.fa_w * fa
        res = torch.cat([flux, torch.zeros_like(x[..., 3:])], -1)
        return torch.where(mask, torch.zeros_like(res), res)

    def clear_tracking(self):
        self.params = []
        self.tracker = []
        self.masks = []
        self.margins = []

    def posterior(self):
        params = torch.stack(self.params).reshape(-1, 2)
        self.params = []
        return torch.distributions.Normal(params.mean(0), params.std(0))

    @classmethod
    def from_module(cls, mod, dtype=None) -> "OracleRHS":
        """Read weights out of a reference-layout module (Fp/Fa/FaFp)."""
        def grab(seq):
            lins = [m for m in seq if isinstance(m, torch.nn.Linear)]
            ws = [l.weight.detach().clone() for l in lins]
            bs = [l.bias.detach().clone() for l in lins]
            if dtype is not None:
                ws = [w.to(dtype) for w in ws]
                bs = [b.to(dtype) for b in bs]
            k = len(lins) - 1
            acts = [i < k - 1 for i in range(len(lins))]
            return ws, bs, acts
        kind = mod.ode_type
        o = cls(kind=kind, n_regions=mod.n_regions, latent_dim=mod.latent_dim)
        if kind in ("Fp", "FaFp"):
            seq = mod.net if hasattr(mod, "net") else mod.Fp_net
            o.p_w, o.p_b, o.p_act = grab(seq)
        if kind in ("Fa", "FaFp"):
            o.a_w, o.a_b, o.a_act = grab(mod.aug_net)
        o.fa_w = float(getattr(mod, "Fa_w", 1.0))
        return o

    def requires_grad_(self):
        for w in self.p_w + self.p_b + self.a_w + self.a_b:
            w.requires_grad_(True)
        return self

    def weights(self) -> List[torch.Tensor]:
        out = []
        for w, b in zip(self.p_w, self.p_b):
            out += [w, b]
        for w, b in zip(self.a_w, self.a_b):
            out += [w, b]
        return out


# ---------------------------------------------------------------------------
# torchdiffeq fixed-grid RK4 restatement
# ---------------------------------------------------------------------------

def make_grid(t: torch.Tensor, step_size) -> torch.Tensor:
    """_grid_constructor_from_step_size: arithmetic in t's dtype."""
    start, end = t[0], t[-1]
    niters = torch.ceil((end - start) / step_size + 1).item()
    grid = torch.arange(0, niters, dtype=t.dtype) * step_size + start
    grid[-1] = t[-1]
    return grid


def output_schedule(t: torch.Tensor, grid: torch.Tensor):
    """Which output index is written after which grid step, and how.

    Returns a list of (j, step, mode, slope) with mode 0: y0 (t==t0),
    1: y1 (t==t1), 2: linear interpolation with ``slope`` (FixedGridODESolver
    .integrate / _linear_interp).  Output 0 is always y0 itself.
    """
    sched = []
    j = 1
    for n in range(len(grid) - 1):
        t0, t1 = grid[n], grid[n + 1]
        while j < len(t) and t1 >= t[j]:
            if t[j] == t0:
                sched.append((j, n, 0, 0.0))
            elif t[j] == t1:
                sched.append((j, n, 1, 1.0))
            else:
                slope = (t[j] - t0) / (t1 - t0)
                sched.append((j, n, 2, float(slope)))
            j += 1
    return sched


def rk4_alt_step(func, t0, dt, t1, y0):
    """rk4_alt_step_func (3/8 rule) with f0 evaluated first (RK4._step_func)."""
    k1 = func(t0, y0)
    k2 = func(t0 + dt * ONE_THIRD, y0 + dt * k1 * ONE_THIRD)
    k3 = func(t0 + dt * TWO_THIRDS, y0 + dt * (k2 - k1 * ONE_THIRD))
    k4 = func(t1, y0 + dt * (k1 - k2 + k3))
    return (k1 + 3 * (k2 + k3) + k4) * dt * 0.125


def odeint_rk4(func, y0: torch.Tensor, t: torch.Tensor, step_size=None) -> torch.Tensor:
    """odeint(func, y0, t, method='rk4', options=dict(step_size=h)).

    The time grid, dt and interpolation slopes are computed in t's dtype
    exactly as torchdiffeq does; they are then cast to y0's dtype.  With an
    fp32 t and an fp64 y0 this gives the fp32 reference's schedule evaluated
    in fp64 state arithmetic (the precision-lifted oracle).
    """
    grid = t if step_size is None else make_grid(t, step_size)
    assert grid[0] == t[0] and grid[-1] == t[-1]
    sdt = y0.dtype
    sol = [None] * len(t)
    sol[0] = y0
    j = 1
    y = y0
    for n in range(len(grid) - 1):
        t0, t1 = grid[n], grid[n + 1]
        dt = (t1 - t0).to(sdt)
        y1 = y + rk4_alt_step(func, t0.to(sdt), dt, t1.to(sdt), y)
        while j < len(t) and t1 >= t[j]:
            if t[j] == t0:
                sol[j] = y
            elif t[j] == t1:
                sol[j] = y1
            else:
                slope = ((t[j] - t0) / (t1 - t0)).to(sdt)
                sol[j] = y + slope * (y1 - y)
            j += 1
        y = y1
    return torch.stack(sol, 0)


# ---------------------------------------------------------------------------
# One "training step" of the hot path: forward + VJP with side statistics
# ---------------------------------------------------------------------------

@dataclass
class SolveResult:
    latent: torch.Tensor
    mean: Optional[torch.Tensor]
    std: Optional[torch.Tensor]
    fa_norm: Optional[torch.Tensor]
    grads: Optional[dict] = None
    masks: Optional[torch.Tensor] = None
    margin: Optional[torch.Tensor] = None      # (N,) min distance of S, I, R to the mask boundary


def solve_and_grad(rhs: OracleRHS, y0: torch.Tensor, t: torch.Tensor, step_size,
                   dlatent: Optional[torch.Tensor] = None,
                   dmean: Optional[torch.Tensor] = None,
                   dstd: Optional[torch.Tensor] = None,
                   dnorm: Optional[float] = None) -> SolveResult:
    """Forward solve; if cotangents are given, VJP w.r.t. y0 and all weights.

    Scalar loss = <latent, dlatent> + <mean, dmean> + <std, dstd> + dnorm*|Fa|.
    """
    want_grad = dlatent is not None
    y0 = y0.detach().clone().requires_grad_(want_grad)
    ws = rhs.weights()
    for w in ws:
        w.requires_grad_(want_grad)
    rhs.clear_tracking()
    with torch.set_grad_enabled(want_grad):
        latent = odeint_rk4(rhs, y0, t, step_size)
        mean = std = norm = None
        if rhs.kind in ("Fa", "FaFp"):
            norm = torch.norm(torch.stack(rhs.tracker))
        if rhs.kind in ("Fp", "FaFp"):
            post = rhs.posterior()
            mean, std = post.loc, post.scale
        res = SolveResult(latent.detach(), None if mean is None else mean.detach(),
                          None if std is None else std.detach(),
                          None if norm is None else norm.detach())
        if want_grad:
            loss = (latent * dlatent).sum()
            if mean is not None and dmean is not None:
                loss = loss + (mean * dmean).sum() + (std * dstd).sum()
            if norm is not None and dnorm is not None:
                loss = loss + dnorm * norm
            gr = torch.autograd.grad(loss, [y0] + ws, allow_unused=True)
            names = ["y0"]
            for i in range(len(rhs.p_w)):
                names += [f"p_w{i}", f"p_b{i}"]
            for i in range(len(rhs.a_w)):
                names += [f"a_w{i}", f"a_b{i}"]
            res.grads = {n: (torch.zeros_like(v) if g is None else g.detach())
                         for n, g, v in zip(names, gr, [y0] + ws)}
    rhs.clear_tracking()
    return res


def _chunk_stats(args):
    """Pass 1 of ``solve_and_grad_chunked`` for one chunk: latent and fp64 side-statistic sums."""
    rhs, y0c, t, step_size, threads = args
    if threads:
        torch.set_num_threads(threads)
    with torch.no_grad():
        rhs.clear_tracking()
        lat = odeint_rk4(rhs, y0c, t, step_size)
        out = {"latent": lat}
        if rhs.params:
            p = torch.stack(rhs.params).reshape(-1, 2).double()
            out["n"], out["s1"], out["s2"] = p.shape[0], p.sum(0), p.pow(2).sum(0)
        if rhs.tracker:
            out["sf"] = float(torch.stack(rhs.tracker).double().pow(2).sum())
        if rhs.record_masks:
            out["masks"] = torch.stack(rhs.masks)
            out["margin"] = torch.stack(rhs.margins).amin(0)
    rhs.clear_tracking()
    return out


def _chunk_grad(args):
    """Pass 2 of ``solve_and_grad_chunked`` for one chunk: gradient of its surrogate loss."""
    rhs, y0c, t, step_size, dlc, dmean, dstd, dnorm, mean, std, norm, n, threads = args
    if threads:
        torch.set_num_threads(threads)
    dt = y0c.dtype
    ws = rhs.weights()
    for w in ws:
        w.requires_grad_(True)
    yc = y0c.detach().clone().requires_grad_(True)
    rhs.clear_tracking()
    lat = odeint_rk4(rhs, yc, t, step_size)
    loss = (lat * dlc.to(dt)).sum()
    if mean is not None and dmean is not None:
        p = torch.stack(rhs.params).reshape(-1, 2)
        m, s = mean.to(dt), std.to(dt)
        loss = loss + (p.sum(0) * dmean.to(dt) / n).sum() \
            + ((p - m).pow(2).sum(0) * dstd.to(dt) / (2.0 * (n - 1) * s)).sum()
    if norm is not None and dnorm is not None and float(norm) > 0:
        loss = loss + dnorm * torch.stack(rhs.tracker).pow(2).sum() / (2.0 * norm.to(dt))
    gr = torch.autograd.grad(loss, [yc] + ws, allow_unused=True)
    rhs.clear_tracking()
    for w in ws:
        w.requires_grad_(False)
    return [torch.zeros_like(v) if g is None else g.detach() for g, v in zip(gr, [yc] + ws)]


def solve_and_grad_chunked(rhs: OracleRHS, y0: torch.Tensor, t: torch.Tensor, step_size,
                           dlatent: Optional[torch.Tensor], dmean: Optional[torch.Tensor] = None,
                           dstd: Optional[torch.Tensor] = None, dnorm: Optional[float] = None,
                           chunk: int = 256, workers: int = 1, masks: bool = False) -> SolveResult:
    """``solve_and_grad`` over trajectory chunks (bounded autograd memory for full-size batches),
    optionally spread over ``workers`` spawned CPU processes (small-GEMM autograd does not use
    many intra-op threads well).

    Trajectories are independent; only the side statistics couple them, and their gradients are
    linear in per-trajectory terms once the global values are known:
      d mean / d p_i = 1/n,  d std / d p_i = (p_i - mean) / ((n-1) std),  d|Fa| / d Fa_i = Fa_i / |Fa|.
    Pass 1 (no autograd) gives the global statistics (fp64 sums); pass 2 back-propagates each
    chunk's surrogate  <lat_c, dl_c> + sum_i [dmean p_i / n + dstd (p_i - mean)^2 / (2 (n-1) std)]
    + dnorm sum_i Fa_i^2 / (2 |Fa|)  (mean, std, |Fa| held constant), whose gradient equals the
    chunk's share of the full loss gradient.  Weight gradients are summed over chunks in order.
    masks=True also returns every evaluation's mask decisions on S, I, R: ``res.masks``
    (E, N, R, 3) bool, evaluation order k1..k4 per step.
    """
    N = y0.shape[0]
    dt = y0.dtype
    rhs.clear_tracking()
    starts = list(range(0, N, chunk))
    threads = max(1, torch.get_num_threads() // workers) if workers > 1 else 0

    def run(fn, jobs):
        if workers <= 1:
            return [fn(j) for j in jobs]
        import multiprocessing as mp
        from concurrent.futures import ProcessPoolExecutor
        with ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
            return list(ex.map(fn, jobs))

    rhs.record_masks = masks
    st = run(_chunk_stats, [(rhs, y0[c0:c0 + chunk], t, step_size, threads) for c0 in starts])
    rhs.record_masks = False
    latent = torch.cat([s["latent"] for s in st], 1)
    mean = std = norm = None
    n = 0
    if "s1" in st[0]:
        n = sum(s["n"] for s in st)
        s1 = sum(s["s1"] for s in st)
        s2 = sum(s["s2"] for s in st)
        mean = s1 / n
        std = torch.sqrt(torch.clamp(s2 - n * mean * mean, min=0.0) / (n - 1))
    if "sf" in st[0]:
        norm = torch.tensor(math.sqrt(sum(s["sf"] for s in st)), dtype=torch.float64)
    res = SolveResult(latent, None if mean is None else mean.to(dt), None if std is None else std.to(dt),
                      None if norm is None else norm.to(dt))
    if masks:
        res.masks = torch.cat([s["masks"] for s in st], 1)
        res.margin = torch.cat([s["margin"] for s in st], 0)
    if dlatent is None:
        return res
    gl = run(_chunk_grad, [(rhs, y0[c0:c0 + chunk], t, step_size, dlatent[:, c0:c0 + chunk], dmean, dstd, dnorm,
                            mean, std, norm, n, threads) for c0 in starts])
    names = ["y0"]
    for i in range(len(rhs.p_w)):
        names += [f"p_w{i}", f"p_b{i}"]
    for i in range(len(rhs.a_w)):
        names += [f"a_w{i}", f"a_b{i}"]
    res.grads = {"y0": torch.cat([g[0] for g in gl], 0)}
    for i, nm in enumerate(names[1:]):
        acc = gl[0][1 + i]
        for g in gl[1:]:
            acc = acc + g[1 + i]
        res.grads[nm] = acc
    return res


def normwise_rel(a: torch.Tensor, b: torch.Tensor) -> float:
    """||a - b|| / max(||b||, tiny), in fp64."""
    a = a.double()
    b = b.double()
    den = max(float(torch.linalg.vector_norm(b)), 1e-30)
    return float(torch.linalg.vector_norm(a - b)) / den
