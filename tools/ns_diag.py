"""Diagnostic (GPU box): error growth of the fused RK4 VJP with the horizon, M1 FaFp R=1.

For T in a list of horizons, N trajectories: fused kernel, the per-evaluation kernels (eager
step loop, evaluation + VJP kernels), the fp32 and fp64 oracles (chunked).  Prints normwise
errors of the latent and of dy0 / every weight gradient against fp64."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import importlib
    pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
    from ude_amd.solvers import eager_fixed_grid
    from oracle.ude_oracle import OracleRHS, solve_and_grad_chunked
    from helpers import normwise_rel
    N = int(os.environ.get("DIAG_N", "512"))
    kind = os.environ.get("DIAG_KIND", "FaFp")
    horizons = [int(x) for x in os.environ.get("DIAG_T", "31,91,181,366").split(",")]
    print(f"N={N} kind={kind} stats={os.environ.get('DIAG_STATS', '0')}", flush=True)
    stats = os.environ.get("DIAG_STATS", "0") == "1"
    DM = torch.tensor([0.3, -0.2], dtype=torch.float64)
    DS = torch.tensor([0.5, 0.1], dtype=torch.float64)
    DN = 0.1
    torch.manual_seed(0)
    kw = dict(net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]) if kind == "FaFp" else dict(net_sizes=[32, 32])
    mod = getattr(pkg, kind)(1, latent_dim=8, **kw)
    gen = torch.Generator().manual_seed(11)
    S = torch.rand(N, 1, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, 1, generator=gen) * 0.05
    y0 = torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, 1, 5, generator=gen)], -1) + 1e-5
    dl_full = torch.randn((max(horizons), N, 1, 8), generator=gen, dtype=torch.float64)
    for T in horizons:
        t = torch.arange(T, dtype=torch.float32) / 7.0
        dl = dl_full[:T].contiguous()
        res = {}
        for name in ("fused", "eager"):
            mg = mod.to("cuda")
            mg.zero_grad(set_to_none=True)
            yg = y0.cuda().requires_grad_(True)
            mg.clear_tracking()
            if name == "fused":
                lat = pkg.odeint(mg, yg, t, method="rk4", options=dict(step_size=t[1] - t[0]))
            else:
                lat = eager_fixed_grid(mg, yg, t.cuda(), "rk4", t[1] - t[0])
            loss = (lat.double() * dl.cuda()).sum()
            if stats:
                if mg.ode_type != "Fp":
                    loss = loss + DN * torch.norm(torch.stack(mg.tracker))
                post = mg.posterior()
                loss = loss + (post.loc.double() * DM.cuda()).sum() + (post.scale.double() * DS.cuda()).sum()
            loss.backward()
            res[name] = {"latent": lat.detach().cpu(), "y0": yg.grad.cpu(),
                         "w0": mg.ude_linears()[0].weight.grad.cpu(), "wl": mg.ude_linears()[-1].weight.grad.cpu()}
            mod.cpu()
        for dt, nm in ((torch.float64, "o64"), (torch.float32, "o32")):
            r = solve_and_grad_chunked(OracleRHS.from_module(mod, dt), y0.to(dt), t, t[1] - t[0], dl.to(dt),
                                       *((DM.to(dt), DS.to(dt), DN) if stats else ()), chunk=64, workers=12)
            keys = [k for k in r.grads if k != "y0"]
            res[nm] = {"latent": r.latent, "y0": r.grads["y0"], "w0": r.grads[keys[0]], "wl": r.grads[keys[-2]]}
        ref = res["o64"]
        for nm in ("fused", "eager", "o32"):
            print(f"T={T:4d} {nm:6s} " + "  ".join(f"{k} {normwise_rel(res[nm][k], ref[k]):.2e}" for k in ref),
                  flush=True)
        print(f"T={T:4d} fused-vs-eager y0 {normwise_rel(res['fused']['y0'], res['eager']['y0']):.2e}", flush=True)


if __name__ == "__main__":
    main()
