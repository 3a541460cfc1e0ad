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
