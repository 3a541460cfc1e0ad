"""Memory fallback for stored activations (SURVEY 5 long-horizon row).

The training forward stores every stage's activation rows for the backward (UdeSizes.act_bytes:
7.7 GB for the 4096 x 365-step north-star solve; M3's 1,024,000 trajectories over a daily year
would need ~1.9 TB).  Above a budget (default: half of the free HBM; ude_amd.fused.ACT_BUDGET /
UDE_ACT_BUDGET_BYTES) the plan sets UdeProblem.recompute: only the 3R stage inputs are stored and
the backward re-runs each stage's layer phases.  The recomputed activations are the forward's own
arithmetic, so the results must be bit-identical to the stored path -- and green vs the oracle."""
import pytest
import torch

from helpers import normwise_rel
from oracle.ude_oracle import OracleRHS, solve_and_grad

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [("FaFp", 1, [64, 64, 32], [64, 64], 37, 15, 7.0),
         ("Fp", 1, [32, 32], None, 300, 12, 7.0),
         ("FaFp", 10, [64, 64, 32], [64, 64], 40, 5, 1.0),
         ("FaFp", 49, [64, 64, 32], [64, 64], 35, 4, 1.0)]


def _solve(pkg, mod, y0, t, dl, budget):
    from ude_amd import fused, solvers
    solvers._PLAN_CACHE.clear()
    fused.ACT_BUDGET = budget
    try:
        mod.zero_grad(set_to_none=True)
        yg = y0.clone().requires_grad_(True)
        mod.clear_tracking()
        lat = pkg.odeint(mod, yg, t, method="rk4", options=dict(step_size=t[1] - t[0]))
        plan = next(reversed(solvers._PLAN_CACHE.values()))
        post = mod.posterior() if mod.ode_type != "Fa" else None
        loss = (lat * dl).sum()
        if post is not None:
            loss = loss + (post.loc * torch.tensor([0.3, -0.2], device=DEV)).sum() \
                + (post.scale * torch.tensor([0.5, 0.1], device=DEV)).sum()
        if mod.ode_type != "Fp":
            loss = loss + 0.1 * torch.norm(torch.stack(mod.tracker))
        loss.backward()
        return (plan.prob.recompute, plan.sizes.act_bytes, lat.detach(), yg.grad.clone(),
                [p.grad.clone() for p in mod.parameters()])
    finally:
        fused.ACT_BUDGET = None
        solvers._PLAN_CACHE.clear()


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}_R{c[1]}")
def test_recompute_bit_identical_and_vs_oracle(pkg, case):
    kind, R, net, aug, N, n_t, div = case
    torch.manual_seed(0)
    kw = {"net_sizes": net}
    if aug:
        kw["aug_net_sizes"] = aug
    mod = getattr(pkg, kind)(R, latent_dim=8, **kw)
    gen = torch.Generator().manual_seed(3)
    S = torch.rand(N, R, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, R, generator=gen) * 0.05
    y0 = torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, R, 5, generator=gen)], -1) + 1e-5
    t = torch.arange(n_t, dtype=torch.float32) / div
    dl = torch.randn((n_t, N, R, 8), generator=gen)
    mg = mod.to(DEV)
    a = _solve(pkg, mg, y0.to(DEV), t, dl.to(DEV), None)
    b = _solve(pkg, mg, y0.to(DEV), t, dl.to(DEV), 0)          # any stored activation exceeds 0 bytes
    assert a[0] == 0 and a[1] > 0, "default plan stores activations"
    assert b[0] == 1 and b[1] == 0, "a zero budget selects the recompute path"
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3]), "latent / dy0 differ"
    # weight gradients: bit-identical where both backwards accumulate them the same way (R = 49);
    # small records' stored path is the 8-wave split kernel, whose partner waves sum the bias rows
    # per trajectory first (a different fp32 summation order than the 4-wave recompute kernel)
    split = R <= 16
    for ga, gb in zip(a[4], b[4]):
        if split:
            assert normwise_rel(gb, ga) < 1e-6
        else:
            assert torch.equal(ga, gb)
    ref = solve_and_grad(OracleRHS.from_module(mod.cpu(), torch.float64), y0.double(), t, t[1] - t[0],
                         dl.double(), torch.tensor([0.3, -0.2], dtype=torch.float64),
                         torch.tensor([0.5, 0.1], dtype=torch.float64), 0.1 if kind != "Fp" else None)
    assert normwise_rel(b[2], ref.latent) < 1e-5
    assert normwise_rel(b[3], ref.grads["y0"]) < 2e-5


def test_query_reports_stored_activation_bytes(pkg):
    """ude_query's act_bytes: the stored-activation share of the checkpoint, 0 with recompute."""
    from ude_amd import _native, configs
    cfg = configs._c("FaFp", 1, 8, [64, 64, 32], [64, 64])
    lib = _native.library_for(cfg)
    desc = _native.make_desc(cfg)
    p = _native.UdeProblem()
    p.n_traj, p.n_steps, p.n_out, p.fa_w, p.recompute = 4096, 365, 365, 1.0, 0
    s0 = lib.query(desc, p, 0)
    p.recompute = 1
    s1 = lib.query(desc, p, 0)
    assert s0.act_bytes > 6e9 and s1.act_bytes == 0
    assert s0.ckpt_bytes - s1.ckpt_bytes == s0.act_bytes
    assert s1.ckpt_bytes == 256 * 365 * 4 * 3 * 16 * 4            # the 3R stage inputs only
