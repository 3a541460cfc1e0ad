"""HIP fused RK4 solve vs the golden fixtures and the fp64 CPU oracle (gfx950).

Parity bar (north_star: "trajectories within 1e-5 rel-err"): normwise relative
error of the fp32 kernel against the fp64 reference <= max(1e-5, 2x the
distance the reference's own fp32 run shows on the same case).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, solver_cases
from helpers import module_from_golden, normwise_rel, step_of, tol

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _run_case(pkg, g, want_grad=True):
    mod = module_from_golden(pkg, g, DEV)
    t, h = step_of(g)
    y0 = torch.from_numpy(g["y0"]).to(DEV).requires_grad_(want_grad)
    mod.clear_tracking()
    assert pkg.fusable(mod, y0)
    latent = pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=h))
    out = {"latent": latent}
    loss = (latent.double() * torch.from_numpy(g["dlatent"]).to(DEV)).sum()
    kind = g["meta"]["kind"]
    if kind in ("Fa", "FaFp"):
        norm = torch.norm(torch.stack(mod.tracker))
        out["fa_norm"] = norm.reshape(1)
        loss = loss + float(g["dnorm"][0]) * norm
    if kind in ("Fp", "FaFp"):
        post = mod.posterior()
        out["mean"], out["std"] = post.loc, post.scale
        loss = loss + (post.loc.double() * torch.from_numpy(g["dmean"]).to(DEV)).sum() \
                    + (post.scale.double() * torch.from_numpy(g["dstd"]).to(DEV)).sum()
    if want_grad:
        loss.backward()
        out["d_y0"] = y0.grad
        for name, p in mod.named_parameters():
            out["d_" + name] = p.grad
    return out


@pytest.mark.parametrize("case", solver_cases())
def test_fused_matches_golden(pkg, case):
    g = load_golden(case)
    out = _run_case(pkg, g)
    torch.cuda.synchronize()
    for key in ["latent", "mean", "std", "fa_norm"]:
        if "ref64_" + key in g:
            err = normwise_rel(out[key], g["ref64_" + key])
            assert err <= tol(g, key), f"{case} {key}: rel err {err:.3e} > {tol(g, key):.1e}"
    for key in [k for k in g if k.startswith("ref64_d_")]:
        k = key[len("ref64_"):]
        err = normwise_rel(out[k], g[key])
        assert err <= tol(g, k, 2e-5), f"{case} {k}: rel err {err:.3e}"


def test_deterministic(pkg):
    g = load_golden("fafp_r1_weekly")
    a = _run_case(pkg, g)
    b = _run_case(pkg, g)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_native_library_was_loaded(pkg):
    paths = pkg.ude_amd._native.loaded_paths()
    assert paths and all(p.endswith(".so") for p in paths)


# ---------------------------------------------------------------------------
# randomised cases vs the fp64 CPU oracle (ragged N, every RHS kind, R = 1/10/49)
# ---------------------------------------------------------------------------
from oracle.ude_oracle import OracleRHS, solve_and_grad  # noqa: E402

RANDOM_CASES = [
    # kind, R, L, net, aug, N, n_t, div, step
    ("FaFp", 1, 8, [64, 64, 32], [64, 64], 129, 30, 7.0, "t1-t0"),
    ("Fp", 1, 8, [32, 32], None, 200, 40, 7.0, "t1-t0"),
    ("Fa", 1, 8, None, [64, 64], 33, 9, 1.0, "t1-t0"),
    ("FaFp", 10, 8, [64, 64, 32], [64, 64], 50, 6, 1.0, "t1-t0"),
    ("Fp", 10, 8, [64, 64, 32], None, 17, 5, 1.0, "t1-t0"),
    ("Fa", 49, 8, None, [64, 64], 20, 4, 1.0, "t1-t0"),
    ("FaFp", 49, 8, [64, 64, 32], [64, 64], 35, 4, 1.0, "t1-t0"),
    ("FaFp", 1, 8, [64, 64, 32], [64, 64], 1, 12, 7.0, 1.0),        # N = 1, interpolated outputs
    ("FaFp", 2, 4, [12], [20, 8], 23, 7, 2.0, "t1-t0"),             # not prebuilt -> JIT build
]


def _random_case(pkg, kind, R, L, net, aug, N, n_t, div, step, seed=0):
    torch.manual_seed(seed)
    cls = getattr(pkg, kind)
    kw = {}
    if net is not None:
        kw["net_sizes"] = net
    if aug is not None:
        kw["aug_net_sizes"] = aug
    mod = cls(R, latent_dim=L, **kw)
    if kind == "FaFp":
        mod.Fa_w = 0.7
    gen = torch.Generator().manual_seed(seed + 1)
    S = torch.rand(N, R, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, R, generator=gen) * 0.05
    y0 = torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None],
                    torch.randn(N, R, L - 3, generator=gen)], -1) + 1e-5
    if step == "t1-t0":
        t = torch.arange(n_t, dtype=torch.float32) / div
        h = t[1] - t[0]
    else:
        t = torch.linspace(1, n_t, n_t) / div
        h = step
    dl = torch.randn((n_t, N, R, L), generator=gen, dtype=torch.float64)
    return mod, y0, t, h, dl


@pytest.mark.parametrize("case", RANDOM_CASES, ids=lambda c: f"{c[0]}_R{c[1]}_L{c[2]}_N{c[5]}_T{c[6]}")
def test_fused_matches_oracle_random(pkg, case):
    kind = case[0]
    mod, y0, t, h, dl = _random_case(pkg, *case)
    dm = torch.tensor([0.3, -0.2], dtype=torch.float64)
    ds = torch.tensor([0.5, 0.1], dtype=torch.float64)
    ref = solve_and_grad(OracleRHS.from_module(mod, torch.float64), y0.double(), t, h, dl, dm, ds, 0.1)
    mg = mod.to(DEV)
    yg = y0.to(DEV).requires_grad_(True)
    mg.clear_tracking()
    assert pkg.fusable(mg, yg)
    lat = pkg.odeint(mg, yg, t, method="rk4", options=dict(step_size=h))
    loss = (lat.double() * dl.to(DEV)).sum()
    if kind != "Fp":
        loss = loss + 0.1 * torch.norm(torch.stack(mg.tracker))
    if kind != "Fa":
        post = mg.posterior()
        assert normwise_rel(post.loc, ref.mean) < 1e-5 and normwise_rel(post.scale, ref.std) < 1e-5
        loss = loss + (post.loc.double() * dm.to(DEV)).sum() + (post.scale.double() * ds.to(DEV)).sum()
    loss.backward()
    assert normwise_rel(lat, ref.latent) < 1e-5
    assert normwise_rel(yg.grad, ref.grads["y0"]) < 2e-5
    lins = mg.ude_linears()
    names = [n for n in ref.grads if n != "y0"]
    params = []
    for lin in lins:
        params += [lin.weight, lin.bias]
    for n, p in zip(names, params):
        assert normwise_rel(p.grad, ref.grads[n]) < 5e-5, n


# ---------------------------------------------------------------------------
# full-size (BASELINE configs[1]: 20,480 trajectories, R = 49) properties
# ---------------------------------------------------------------------------
def _full_size(pkg):
    torch.manual_seed(0)
    mod = pkg.FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]).to(DEV)
    gen = torch.Generator().manual_seed(5)
    N = 20480
    S = torch.rand(N, 49, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, 49, generator=gen) * 0.05
    y0 = torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, 49, 5, generator=gen)], -1)
    t = torch.arange(9, dtype=torch.float32)
    dl = torch.randn((9, N, 49, 8), generator=gen)
    return mod, (y0 + 1e-5).to(DEV), t, dl.to(DEV)


def _vjp(pkg, mod, y0, t, dl, scale=1.0):
    yg = y0.clone().requires_grad_(True)
    mod.zero_grad(set_to_none=True)
    mod.clear_tracking()
    lat = pkg.odeint(mod, yg, t, method="rk4", options=dict(step_size=t[1] - t[0]))
    post = mod.posterior()
    nrm = torch.norm(torch.stack(mod.tracker))
    torch.autograd.backward([lat, post.loc, post.scale, nrm],
                            [dl * scale, torch.tensor([0.3, -0.2], device=DEV) * scale,
                             torch.tensor([0.5, 0.1], device=DEV) * scale, torch.tensor(0.1 * scale, device=DEV)])
    return lat.detach(), yg.grad, [p.grad.clone() for p in mod.parameters()]


def test_full_size_properties(pkg):
    mod, y0, t, dl = _full_size(pkg)
    lat, dy, dws = _vjp(pkg, mod, y0, t, dl)
    assert torch.isfinite(lat).all() and torch.isfinite(dy).all() and all(torch.isfinite(g).all() for g in dws)
    # bitwise reproducible (deterministic reductions, no float atomics)
    lat2, dy2, dws2 = _vjp(pkg, mod, y0, t, dl)
    assert torch.equal(lat, lat2) and torch.equal(dy, dy2) and all(torch.equal(a, b) for a, b in zip(dws, dws2))
    # the VJP is linear in the cotangents: x2 scaling is exact in fp32
    _, dy3, dws3 = _vjp(pkg, mod, y0, t, dl, scale=2.0)
    assert torch.equal(dy3, 2 * dy) and all(torch.equal(a, 2 * b) for a, b in zip(dws3, dws))
    # trajectories are independent: a 64-trajectory slice solved alone is bit-identical
    mod.clear_tracking()
    sub = pkg.odeint(mod, y0[:64].contiguous(), t, method="rk4", options=dict(step_size=t[1] - t[0]))
    assert torch.equal(sub, lat[:, :64])
    # static latent dims are carried unchanged
    assert torch.equal(lat[:, :, :, 3:], y0[None, :, :, 3:].expand_as(lat[:, :, :, 3:]))


@pytest.mark.gpu
def test_cached_grid_follows_inplace_updates(pkg):
    """The host-side t / plan caches must not serve a stale schedule when the same
    device tensor t is modified in place between solves."""
    mod, y0, t, h, dl = _random_case(pkg, "FaFp", 1, 8, [64, 64, 32], [64, 64], 16, 6, 7.0, "t1-t0")
    ref = OracleRHS.from_module(mod, torch.float64)
    mg = mod.to(DEV)
    td = t.to(DEV)
    for scale in (1.0, 2.0):
        if scale != 1.0:
            td.mul_(scale)                       # same tensor object, new values
        tc = td.cpu()
        want = solve_and_grad(ref, y0.double(), tc, tc[1] - tc[0]).latent
        mg.clear_tracking()
        with torch.no_grad():
            lat = pkg.odeint(mg, y0.to(DEV), td, method="rk4", options=dict(step_size=td[1] - td[0]))
        assert normwise_rel(lat, want) < 1e-5, scale


def test_weight_pack_not_reused_across_modules(pkg):
    """the weight pack is cached on the shared plan; a module freed and a new one of
    the same configuration built in its place (same allocator addresses, the same parameter version
    sequence: init + load_state_dict) must solve with ITS weights, not the freed module's pack."""
    import gc
    t = torch.arange(5, dtype=torch.float32)
    gen = torch.Generator().manual_seed(3)
    y0 = torch.cat([torch.rand(32, 1, 3, generator=gen) * 0.3 + 0.2, torch.randn(32, 1, 5, generator=gen)], -1).to(DEV)

    def build(seed):
        torch.manual_seed(seed)
        m = pkg.FaFp(1, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
        m2 = pkg.FaFp(1, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
        m2.load_state_dict(m.state_dict())       # one version bump per parameter, like a checkpoint load
        return m2.to(DEV)

    def solve(m):
        m.clear_tracking()
        with torch.no_grad():
            return pkg.odeint(m, y0, t, method="rk4", options=dict(step_size=1.0)).clone()

    a = build(1)
    lat_a = solve(a)
    del a
    gc.collect()
    b = build(2)                                  # different weights, very likely a's addresses
    lat_b = solve(b)
    fresh = build(2)
    pkg.ude_amd.fused.invalidate_packs()
    lat_ref = solve(fresh)
    assert not torch.equal(lat_a, lat_ref)
    assert torch.equal(lat_b, lat_ref)
