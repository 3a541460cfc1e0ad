"""Generate the Bayesian-RHS golden fixtures under tests/golden/ (build container only).

Runs the reference's own ``lib/in_development/models_bayes.py`` classes
(Bayes_Fp / Bayes_Fa / Bayes_FaFp, read-only under /root/reference) through the
oracle's restatement of torchdiffeq's fixed-grid RK4 (torchdiffeq is absent, see
oracle/ude_oracle.py).  The only intervention: each ``Dense_Variational``
instance's ``make_z`` (:30-32) takes its ``z`` from a recorded standard-normal
stream instead of ``torch.randn_like``, so the fixture can replay the exact
draws -- ``eps[e]`` holds evaluation e's draws in the order the layers call
``make_z`` (torch parameter order: per layer w then b, rate net first).
``Dense_Variational.forward`` itself (:43-48: ``w_mean + z * |w_std|``) runs
unmodified.

Outputs (npz, no pickles): inputs, eps, weights, the fp64 reference outputs and
the VJP of a fixed linear functional w.r.t. y0 and every parameter (means and
stds), and the reference's own fp32-vs-fp64 distances.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_bayes.py [case names]
"""
from __future__ import annotations

import copy
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

import lib.in_development.models_bayes as ref_bayes  # noqa: E402  (reference, read-only)
from oracle.ude_oracle import odeint_rk4, normwise_rel  # noqa: E402

CASES = [
    # name, kind, R, L, net, aug, N, t-spec, step, fa_w
    ("bayes_fafp_r1_weekly", "FaFp", 1, 8, [64, 64, 32], [64, 64], 40, ("arange", 9, 1.0), "t1-t0", 1.0),
    ("bayes_fp_r1_daily", "Fp", 1, 8, [20, 20], None, 24, ("arange", 15, 7.0), "t1-t0", 1.0),
    ("bayes_fa_r1_weekly", "Fa", 1, 8, None, [32, 32], 20, ("arange", 6, 1.0), "t1-t0", 1.0),
    ("bayes_fafp_r1_interp", "FaFp", 1, 8, [64, 64, 32], [64, 64], 33, ("linspace", 12, 7.0), 0.25, 0.5),
    ("bayes_fafp_r10_weekly", "FaFp", 10, 8, [64, 64, 32], [64, 64], 18, ("arange", 4, 1.0), "t1-t0", 1.0),
    # the state model's size ('UONNb', run_ode.py): beyond the fused whole-solve kernel
    ("bayes_fafp_r49_weekly", "FaFp", 49, 8, [64, 64, 32], [64, 64], 10, ("arange", 3, 1.0), "t1-t0", 1.0),
]


def make_t(spec):
    kind, n, div = spec
    return torch.arange(n, dtype=torch.float32) / div if kind == "arange" else torch.linspace(1, n, n) / div


def make_y0(gen, N, R, L):
    S = torch.rand(N, R, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, R, generator=gen) * 0.05
    rest = torch.randn(N, R, L - 3, generator=gen)
    return (torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], rest], -1) + 1e-5).float()


def build(kind, R, L, net, aug):
    if kind == "FaFp":
        return ref_bayes.Bayes_FaFp(R, latent_dim=L, net_sizes=net, aug_net_sizes=aug, prior_std=0.05)
    if kind == "Fp":
        return ref_bayes.Bayes_Fp(R, latent_dim=L, net_sizes=net, prior_std=0.05)
    return ref_bayes.Bayes_Fa(R, latent_dim=L, aug_net_sizes=aug, prior_std=0.05)


def variational_layers(mod):
    out = []
    for name in ("Fp_net", "aug_net"):
        if hasattr(mod, name):
            out += [m for m in getattr(mod, name) if isinstance(m, ref_bayes.Dense_Variational)]
    return out


def inject(mod, eps):
    """Replace every layer's make_z by a replay of eps (one row per evaluation)."""
    layers = variational_layers(mod)
    state = {"ev": -1}
    off = 0
    for li, lay in enumerate(layers):
        nw, nb = lay.w_mean.numel(), lay.b_mean.numel()

        def make_z(lay=lay, li=li, ow=off, nw=nw, nb=nb):
            if li == 0:
                state["ev"] += 1
            row = eps[state["ev"]]
            lay.z = [row[ow:ow + nw].reshape(lay.w_mean.shape).to(lay.w_mean.dtype),
                     row[ow + nw:ow + nw + nb].reshape(lay.b_mean.shape).to(lay.b_mean.dtype)]
        lay.make_z = make_z
        off += nw + nb
    return state


def run(mod, eps, y0, t, step, dlatent, dmean, dstd, dnorm, dtype):
    mod = mod.to(dtype)
    state = inject(mod, eps.to(dtype))
    y0 = y0.to(dtype).clone().requires_grad_(True)
    h = t[1] - t[0] if step == "t1-t0" else step
    mod.clear_tracking()
    latent = odeint_rk4(mod, y0, t, h)
    assert state["ev"] + 1 == eps.shape[0], (state["ev"], eps.shape)
    loss = (latent * dlatent.to(dtype)).sum()
    out = {"latent": latent.detach()}
    if mod.ode_type in ("Fa", "FaFp"):                 # Bayes_Fp keeps no tracker
        norm = torch.norm(torch.stack(mod.tracker))
        loss = loss + dnorm * norm
        out["fa_norm"] = norm.detach().reshape(1)
    if mod.ode_type in ("Fp", "FaFp"):                 # Bayes_Fa records no rates
        post = mod.posterior()
        loss = loss + (post.loc * dmean.to(dtype)).sum() + (post.scale * dstd.to(dtype)).sum()
        out["mean"], out["std"] = post.loc.detach(), post.scale.detach()
    params = [p for _, p in mod.named_parameters()]
    grads = torch.autograd.grad(loss, [y0] + params)
    out["d_y0"] = grads[0]
    for (name, _), g in zip(mod.named_parameters(), grads[1:]):
        out["d_" + name] = g
    mod.clear_tracking()
    return out


def main(only=None):
    torch.set_num_threads(1)
    for ci, (name, kind, R, L, net, aug, N, tspec, step, fa_w) in enumerate(CASES):
        if only and name not in only:
            continue
        torch.manual_seed(3000 + ci)
        gen = torch.Generator().manual_seed(4000 + ci)
        mod = build(kind, R, L, net, aug)
        # std parameters of both signs and varied size (|std| and its sign matter)
        with torch.no_grad():
            for lay in variational_layers(mod):
                lay.w_std.copy_(0.1 * torch.randn(lay.w_std.shape, generator=gen))
                lay.b_std.copy_(0.1 * torch.randn(lay.b_std.shape, generator=gen))
        if kind == "FaFp":
            mod.Fa_w = fa_w
        t = make_t(tspec)
        h = t[1] - t[0] if step == "t1-t0" else step
        from oracle.ude_oracle import make_grid
        n_steps = len(make_grid(t, h)) - 1
        n_params = sum(p.numel() for p in mod.parameters()) // 2
        eps = torch.randn(4 * n_steps, n_params, generator=gen)
        y0 = make_y0(gen, N, R, L)
        dlatent = torch.randn(len(t), N, R, L, generator=gen, dtype=torch.float64)
        dmean = torch.tensor([0.3, -0.2], dtype=torch.float64)
        dstd = torch.tensor([0.5, 0.1], dtype=torch.float64)
        dnorm = 0.1
        sd32 = {k: v.detach().clone() for k, v in mod.state_dict().items()}
        o32 = run(copy.deepcopy(mod), eps, y0, t, step, dlatent, dmean, dstd, dnorm, torch.float32)
        o64 = run(copy.deepcopy(mod), eps, y0, t, step, dlatent, dmean, dstd, dnorm, torch.float64)
        arrs = {"y0": y0.numpy(), "t": t.numpy(), "eps": eps.numpy(), "dlatent": dlatent.numpy(),
                "dmean": dmean.numpy(), "dstd": dstd.numpy(), "dnorm": np.array([dnorm])}
        for k, v in sd32.items():
            arrs["w_" + k] = v.numpy()
        for k, v in o32.items():
            if k in ("latent", "mean", "std", "fa_norm"):
                arrs["ref32_" + k] = v.float().numpy()
        for k, v in o64.items():
            arrs["ref64_" + k] = v.double().numpy()
        dist = {k: normwise_rel(o32[k], o64[k]) for k in o64}
        meta = {"name": name, "kind": kind, "bayes": True, "n_regions": R, "latent_dim": L,
                "net_sizes": net, "aug_net_sizes": aug, "n_traj": N, "step": step, "fa_w": fa_w,
                "state_dict_keys": list(sd32.keys()), "ref32_vs_ref64": dist,
                "generator": "tests/golden/make_golden_bayes.py (reference models_bayes.py + oracle RK4, "
                             "eps replayed through Dense_Variational.make_z)"}
        arrs["meta_json"] = np.array(json.dumps(meta))
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **arrs)
        print(f"{name:20s} N={N:3d} evals={eps.shape[0]:3d} worst ref32-vs-ref64 rel={max(dist.values()):.2e}")


if __name__ == "__main__":
    main(sys.argv[1:])
