"""Generate the golden fixtures under tests/golden/ (run in the build container).

This is the ONLY place reference code runs.  It imports the reference's own RHS
classes (``lib/models.py`` Fp / Fa / FaFp under /root/reference) and integrates
them with the oracle's restatement of torchdiffeq's fixed-grid RK4 (torchdiffeq
itself is absent from the reference and the image; see oracle/ude_oracle.py).
The loss side-statistics are taken exactly as ``lib/VAE.py`` takes them:
``ode.posterior()`` (:173) and ``torch.norm(torch.stack(ode.tracker))`` (:180).

Outputs (npz, no pickles): inputs, reference-RHS outputs in fp32 and fp64, the
VJP of a fixed linear functional in fp64, and the fp32-vs-fp64 distances the
reference itself shows on each case (used to set the parity tolerance).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

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

import lib.models as ref_models  # noqa: E402  (reference, read-only)
from oracle.ude_oracle import odeint_rk4, normwise_rel  # noqa: E402

CASES = [
    # name, kind, R, L, net_sizes, aug_net_sizes, N, t-spec, step, fa_w, masked
    ("fafp_r1_weekly", "FaFp", 1, 8, [64, 64, 32], [64, 64], 48, ("arange", 9, 1.0), "t1-t0", 1.0, False),
    ("fp_r1_daily", "Fp", 1, 8, [32, 32], None, 40, ("arange", 29, 7.0), "t1-t0", 1.0, False),
    ("fa_r1_weekly", "Fa", 1, 8, None, [64, 64], 24, ("arange", 6, 1.0), "t1-t0", 1.0, False),
    ("fafp_r10_weekly", "FaFp", 10, 8, [64, 64, 32], [64, 64], 20, ("arange", 5, 1.0), "t1-t0", 1.0, False),
    ("fafp_r49_weekly", "FaFp", 49, 8, [64, 64, 32], [64, 64], 8, ("arange", 3, 1.0), "t1-t0", 1.0, False),
    ("fafp_r1_interp", "FaFp", 1, 8, [64, 64, 32], [64, 64], 24, ("linspace", 20, 7.0), 1.0, 0.05, False),
    ("fafp_r1_masked", "FaFp", 1, 8, [64, 64, 32], [64, 64], 32, ("arange", 9, 1.0), "t1-t0", 1.0, True),
    ("fafp_r1_defaults", "FaFp", 1, 8, [20, 20], [32, 32], 24, ("arange", 8, 7.0), "t1-t0", 1.0, False),
    ("fp_r1_onehidden", "Fp", 1, 6, [24], None, 24, ("arange", 6, 1.0), "t1-t0", 1.0, False),
    ("fafp_r3_l5_ragged", "FaFp", 3, 5, [40, 24], [36], 37, ("arange", 7, 3.0), "t1-t0", 0.5, False),
]


def make_t(spec):
    kind, n, div = spec
    if kind == "arange":
        return torch.arange(n, dtype=torch.float32) / div
    return torch.linspace(1, n, n) / div


def make_y0(gen, N, R, L, masked):
    S = torch.rand(N, R, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, R, generator=gen) * 0.05
    Rr = 1 - S - I
    rest = torch.randn(N, R, L - 3, generator=gen)
    y0 = torch.cat([S[..., None], I[..., None], Rr[..., None], rest], -1) + 1e-5
    if masked:
        # push some compartments outside [-1, 2] (the strict mask of lib/models.py:130)
        y0[0::4, :, 0] = 2.5
        y0[1::4, :, 1] = -1.5
        y0[2::4, :, 2] = 2.0      # exactly 2.0 is NOT masked
    return y0.float()


def build_module(kind, R, L, net, aug):
    if kind == "FaFp":
        return ref_models.FaFp(R, latent_dim=L, net_sizes=net, aug_net_sizes=aug)
    if kind == "Fp":
        return ref_models.Fp(R, latent_dim=L, net_sizes=net)
    return ref_models.Fa(R, latent_dim=L, aug_net_sizes=aug)


def run(mod, y0, t, step, dlatent, dmean, dstd, dnorm, dtype):
    mod = mod.to(dtype)
    y0 = y0.to(dtype).clone().requires_grad_(True)
    if step == "t1-t0":
        h = t[1] - t[0]
    else:
        h = step
    mod.clear_tracking()
    latent = odeint_rk4(mod, y0, t, h)
    loss = (latent * dlatent.to(dtype)).sum()
    out = {"latent": latent.detach()}
    if mod.ode_type in ("Fa", "FaFp"):
        norm = torch.norm(torch.stack(mod.tracker))          # lib/VAE.py:180
        loss = loss + dnorm * norm
        out["fa_norm"] = norm.detach().reshape(1)
    if mod.ode_type in ("Fp", "FaFp"):
        post = mod.posterior()                                # lib/VAE.py:173
        loss = loss + (post.loc * dmean.to(dtype)).sum() + (post.scale * dstd.to(dtype)).sum()
        out["mean"] = post.loc.detach()
        out["std"] = post.scale.detach()
    params = [p for _, p in mod.named_parameters()]
    grads = torch.autograd.grad(loss, [y0] + params)
    out["d_y0"] = grads[0]
    for (name, _), g in zip(mod.named_parameters(), grads[1:]):
        out["d_" + name] = g
    mod.clear_tracking()
    return out


def main():
    torch.set_num_threads(1)
    for ci, (name, kind, R, L, net, aug, N, tspec, step, fa_w, masked) in enumerate(CASES):
        torch.manual_seed(1000 + ci)
        gen = torch.Generator().manual_seed(2000 + ci)
        mod = build_module(kind, R, L, net, aug)
        if kind == "FaFp":
            mod.Fa_w = fa_w
        t = make_t(tspec)
        y0 = make_y0(gen, N, R, L, masked)
        dlatent = torch.randn(len(t), N, R, L, generator=gen, dtype=torch.float64)
        dmean = torch.tensor([0.3, -0.2], dtype=torch.float64)
        dstd = torch.tensor([0.5, 0.1], dtype=torch.float64)
        dnorm = 0.1
        sd32 = {k: v.detach().clone() for k, v in mod.state_dict().items()}
        import copy
        o32 = run(copy.deepcopy(mod), y0, t, step, dlatent, dmean, dstd, dnorm, torch.float32)
        o64 = run(copy.deepcopy(mod), y0, t, step, dlatent, dmean, dstd, dnorm, torch.float64)
        arrs = {
            "y0": y0.numpy(), "t": t.numpy(),
            "dlatent": dlatent.numpy(), "dmean": dmean.numpy(), "dstd": dstd.numpy(),
            "dnorm": np.array([dnorm]),
        }
        for k, v in sd32.items():
            arrs["w_" + k] = v.numpy()
        for k, v in o32.items():
            if k in ("latent", "mean", "std", "fa_norm"):
                arrs["ref32_" + k] = v.float().numpy()
        for k, v in o64.items():
            arrs["ref64_" + k] = v.double().numpy()
        dist = {k: normwise_rel(o32[k], o64[k]) for k in o64}
        meta = {
            "name": name, "kind": kind, "n_regions": R, "latent_dim": L,
            "net_sizes": net, "aug_net_sizes": aug, "n_traj": N,
            "step": step, "fa_w": fa_w, "masked": masked,
            "state_dict_keys": list(sd32.keys()),
            "ref32_vs_ref64": dist,
            "generator": "tests/golden/make_golden.py (reference lib/models.py + oracle RK4)",
        }
        arrs["meta_json"] = np.array(json.dumps(meta))
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **arrs)
        worst = max(dist.values())
        print(f"{name:22s} N={N:3d} T={len(t):3d} worst ref32-vs-ref64 rel={worst:.2e} -> {path}")

    # single-eval RHS fixtures, including states on/over the mask boundary
    torch.manual_seed(77)
    gen = torch.Generator().manual_seed(78)
    for kind in ("Fp", "Fa", "FaFp"):
        for R in (1, 4):
            mod = build_module(kind, R, 8, [16, 16, 8], [16, 12])
            x = torch.randn(33, R, 8, generator=gen) * 1.2
            x[0, 0, 0] = 2.0
            x[1, 0, 1] = -1.0
            x[2, 0, 2] = 2.0000002
            x[3, 0, 0] = -1.0000001
            mod.clear_tracking()
            res = mod(0.0, x.clone())
            arrs = {"x": x.numpy(), "res": res.detach().numpy()}
            if kind != "Fa":
                arrs["p"] = mod.params[0].detach().numpy()
            if kind != "Fp":
                arrs["fa"] = mod.tracker[0].detach().numpy()
            for k, v in mod.state_dict().items():
                arrs["w_" + k] = v.numpy()
            meta = {"kind": kind, "n_regions": R, "latent_dim": 8, "net_sizes": [16, 16, 8],
                    "aug_net_sizes": [16, 12], "state_dict_keys": list(mod.state_dict().keys())}
            arrs["meta_json"] = np.array(json.dumps(meta))
            np.savez_compressed(os.path.join(HERE, f"rhs_{kind.lower()}_r{R}.npz"), **arrs)
    print("rhs fixtures written")




def make_e2e():
    """End-to-end training-step fixture: the reference VAE (lib/VAE.py) with the
    reference Encoder / Decoder / FaFp, integrated by the oracle RK4 (injected as
    the `torchdiffeq` module the reference imports), one train-step loss + grads."""
    import types
    import torch.nn as nn
    td = types.ModuleType("torchdiffeq")

    def _odeint(func, y0, t, rtol=1e-7, atol=1e-9, method=None, options=None, event_fn=None):
        assert method == "rk4"
        return odeint_rk4(func, y0, t, (options or {}).get("step_size"))
    td.odeint = _odeint
    sys.modules["torchdiffeq"] = td
    import lib.VAE as ref_vae
    torch.manual_seed(4242)
    B, window, n_qs, S_ = 4, 6, 3, 5
    model = ref_vae.VAE(ref_models.Encoder_Back_GRU, ref_models.FaFp, ref_models.Decoder, n_qs, 8, 1,
                        ode_params={"net_sizes": [16, 16, 8], "aug_net_sizes": [16, 12], "prior_std": 0.05},
                        enc_params={"q_sizes": [16, 8], "ff_sizes": [8, 8], "SIR_scaler": [0.1, 0.05, 1.0]},
                        uncertainty=True, ode_kl_w=1 / 153)
    model.setup_training(lr=1e-3)
    gen = torch.Generator().manual_seed(99)
    x = torch.rand(B, window, n_qs + 1, generator=gen)
    gamma = 21
    t = torch.arange(window + gamma + 1, dtype=torch.float32) / 7
    eval_pts = np.arange(0, 22, 7)                      # run_ode.py curriculum stage [0, 7, 14, 21]
    y = torch.rand(B, len(t), 1, generator=gen) * 0.5
    y[0, 3, 0] = -1.0                                   # masked target (train_functions.nll_loss)
    losses = {"nll": True, "mse": False, "kl_z": True, "kl_p": True, "Fa_norm": 1e-1, "reg_loss": True, "anneal": True}
    sd = {"enc": {k: v.clone() for k, v in model.enc.state_dict().items()},
          "ode": {k: v.clone() for k, v in model.ode.state_dict().items()},
          "dec": {k: v.clone() for k, v in model.dec.state_dict().items()}}
    torch.manual_seed(7)
    eps = torch.randn(S_, B, 1, model.ld_enc)
    torch.manual_seed(7)                                # VAE.__call__ draws the same eps
    model.optimizer.zero_grad()
    y_pred = model(x, t[eval_pts], n_samples=S_, training=True)
    loss, data, names = model.calc_loss(y_pred, y[:, eval_pts, :], losses)
    loss.backward()
    arrs = {"x": x.numpy(), "y": y.numpy(), "t": t.numpy(), "eval_pts": eval_pts, "eps": eps.numpy(),
            "loss": np.array([float(loss)]), "y_pred": y_pred.detach().numpy(),
            "latent": model.latent.detach().numpy()}
    for part, mod in (("enc", model.enc), ("ode", model.ode), ("dec", model.dec)):
        for k, v in sd[part].items():
            arrs[f"w_{part}.{k}"] = v.numpy()
        for k, p in mod.named_parameters():
            arrs[f"g_{part}.{k}"] = p.grad.detach().numpy()
    meta = {"B": B, "window": window, "n_qs": n_qs, "n_samples": S_, "losses": losses,
            "loss_names": names, "loss_data": data,
            "ode_params": {"net_sizes": [16, 16, 8], "aug_net_sizes": [16, 12]},
            "enc_params": {"q_sizes": [16, 8], "ff_sizes": [8, 8], "SIR_scaler": [0.1, 0.05, 1.0]}}
    arrs["meta_json"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, "e2e_vae_step.npz"), **arrs)
    print("e2e fixture written, loss", float(loss), dict(zip(names, data)))


def make_e2e_case(name, R, n_qs, B, S_, window, gamma, ode_params, enc_params, seed, bayes=False):
    """End-to-end training step of the reference VAE at a given region count, run twice by the
    reference code itself: in fp32 (the reference's dtype) and in fp64 (the parity target; the
    fp32-vs-fp64 distance of the reference's own step sets the tolerance).  The eps draw of
    VAE.__call__ is pinned by replacing torch.randn for the duration of the call.  bayes: the ODE is
    the reference's Bayes_FaFp (lib/in_development/models_bayes.py, run_ode.py:99 'UONNb'); every
    RHS evaluation's weight draws replay the stream ``ode_eps`` through Dense_Variational.make_z
    (tests/golden/make_golden_bayes.py inject) and the loss gains the reference's ode_kl term."""
    import copy
    import types
    td = types.ModuleType("torchdiffeq")

    def _odeint(func, y0, t, rtol=1e-7, atol=1e-9, method=None, options=None, event_fn=None):
        assert method == "rk4"
        return odeint_rk4(func, y0, t, (options or {}).get("step_size"))
    td.odeint = _odeint
    sys.modules["torchdiffeq"] = td
    import lib.VAE as ref_vae
    torch.manual_seed(seed)
    ode_cls = ref_models.FaFp
    if bayes:
        import lib.in_development.models_bayes as ref_bayes
        ode_cls = ref_bayes.Bayes_FaFp
    model = ref_vae.VAE(ref_models.Encoder_Back_GRU, ode_cls, ref_models.Decoder, n_qs, 8, R,
                        ode_params=dict(ode_params, prior_std=0.05), enc_params=enc_params,
                        uncertainty=True, ode_kl_w=1 / 153)
    gen = torch.Generator().manual_seed(seed + 1)
    x = torch.rand(B, window, R * (n_qs + 1), generator=gen)
    t = torch.arange(window + gamma + 1, dtype=torch.float32) / 7
    eval_pts = np.arange(0, gamma + 1, 7)                # run_ode.py's longest curriculum stage
    y = torch.rand(B, len(t), R, generator=gen) * 0.5
    y[0, 7, 0] = -1.0                                    # masked targets (train_functions.nll_loss)
    y[-1, 14, R - 1] = -1.0
    eps = torch.randn(S_, B, R, model.ld_enc, generator=gen)
    losses = {"nll": True, "mse": False, "kl_z": True, "kl_p": True, "Fa_norm": 1e-1, "reg_loss": True,
              "anneal": True}
    sd = {part: {k: v.clone() for k, v in getattr(model, part).state_dict().items()}
          for part in ("enc", "ode", "dec")}
    ode_eps = None
    if bayes:
        n_steps = len(eval_pts) - 1                      # weekly outputs, step = t[1] - t[0]: grid = outputs
        n_par = sum(p.numel() for p in model.ode.parameters()) // 2
        ode_eps = torch.randn(4 * n_steps, n_par, generator=gen)

    def step(dtype):
        m = copy.deepcopy(model)
        for part in ("enc", "ode", "dec"):
            getattr(m, part).to(dtype)
        m.dtype = dtype
        m.enc.scaler = m.enc.scaler.to(dtype)
        m.setup_training(lr=1e-3)
        if bayes:
            from make_golden_bayes import inject
            inject(m.ode, ode_eps.to(dtype))
        real_randn = torch.randn
        torch.randn = lambda *a, **k: eps.to(dtype).clone()
        try:
            y_pred = m(x.to(dtype), t[eval_pts].to(dtype), n_samples=S_, training=True)
        finally:
            torch.randn = real_randn
        loss, data, names = m.calc_loss(y_pred, y[:, eval_pts, :].to(dtype), losses)
        loss.backward()
        out = {"loss": loss.detach().reshape(1), "y_pred": y_pred.detach(), "latent": m.latent.detach()}
        for part in ("enc", "ode", "dec"):
            for k, p in getattr(m, part).named_parameters():
                out[f"g_{part}.{k}"] = p.grad.detach()
        return out, names, data

    o32, names, data = step(torch.float32)
    o64, _, _ = step(torch.float64)
    dist_b = None
    if bayes:
        # a second fp32 run of the same reference step with every Linear's products summed in another
        # order (blocks of 4 along K, last block first): a second sample of fp32 rounding for the
        # ill-conditioned terms (the decoder gradients through nll_loss's per-window sample std)
        lin = torch.nn.functional.linear

        def rev4(h, w, b=None):
            K = h.shape[-1]
            acc = None if b is None else b.expand(h.shape[:-1] + (w.shape[0],))
            for k0 in reversed(range(0, K, 4)):
                part = h[..., k0:k0 + 4] @ w[:, k0:k0 + 4].T
                acc = part if acc is None else acc + part
            return acc
        torch.nn.functional.linear = rev4
        try:
            o32b, _, _ = step(torch.float32)
        finally:
            torch.nn.functional.linear = lin
        dist_b = {k: normwise_rel(o32b[k], o64[k]) for k in o64}
    arrs = {"x": x.numpy(), "y": y.numpy(), "t": t.numpy(), "eval_pts": eval_pts, "eps": eps.numpy()}
    if bayes:
        arrs["ode_eps"] = ode_eps.numpy()
    for part in ("enc", "ode", "dec"):
        for k, v in sd[part].items():
            arrs[f"w_{part}.{k}"] = v.numpy()
    for k, v in o64.items():
        # the (T, N, R, L) latent is kept at fp32 precision (6e-8 rounding, far under every bar)
        arrs["ref64_" + k] = v.float().numpy() if k == "latent" else v.numpy()
    arrs["ref32_loss"] = o32["loss"].numpy()
    dist = {k: normwise_rel(o32[k], o64[k]) for k in o64}
    meta = {"B": B, "window": window, "gamma": gamma, "n_qs": n_qs, "n_regions": R, "n_samples": S_, "bayes": bayes,
            "losses": losses, "loss_names": names, "loss_data": data, "ode_params": ode_params,
            "enc_params": enc_params, "ref32_vs_ref64": dist, "ref32b_vs_ref64": dist_b,
            "generator": "tests/golden/make_golden.py make_e2e_case (reference lib/VAE.py + lib/models.py, "
                         "oracle RK4 as torchdiffeq), fp32 and fp64 runs of the reference step"}
    arrs["meta_json"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
    print(f"{name}: loss32 {float(o32['loss'])} loss64 {float(o64['loss'])}, worst ref32-vs-ref64 "
          f"{max(dist.values()):.2e}", dict(zip(names, data)))


def make_e2e_state49():
    # configs[3]: the reference's state model (run_ode.py:41-49: R = 49, L = 8, FaFp net [64, 64, 32],
    # aug [64, 64], n_qs 8), 64 MC samples (run_ode.py:37), 9 weekly outputs (gamma 56); the GRU
    # encoder (out of scope, plain PyTorch) is narrowed to keep the fixture small
    make_e2e_case("e2e_vae_state49", R=49, n_qs=8, B=2, S_=64, window=8, gamma=56,
                  ode_params={"net_sizes": [64, 64, 32], "aug_net_sizes": [64, 64]},
                  enc_params={"q_sizes": [32, 16], "ff_sizes": [16, 16], "SIR_scaler": [0.1, 0.05, 1.0]},
                  seed=4949)


def make_e2e_us():
    # the reference's US model (run_ode.py:59-66: R = 1, L = 8, FaFp [64, 64, 32] / [64, 64]) at
    # run_ode.py's training batch shape (64 MC samples), narrowed encoder as above
    make_e2e_case("e2e_vae_us", R=1, n_qs=90, B=8, S_=64, window=8, gamma=56,
                  ode_params={"net_sizes": [64, 64, 32], "aug_net_sizes": [64, 64]},
                  enc_params={"q_sizes": [32, 16], "ff_sizes": [16, 16], "SIR_scaler": [0.1, 0.05, 1.0]},
                  seed=1111)


def make_e2e_us_bayes():
    # the US model as run_ode.py's 'UONNb' (Bayes_FaFp, fresh weight sample per RHS evaluation) in the
    # VAE training step, with the reference's ode_kl term (lib/VAE.py:191-195)
    make_e2e_case("e2e_vae_us_bayes", R=1, n_qs=90, B=8, S_=64, window=8, gamma=56,
                  ode_params={"net_sizes": [64, 64, 32], "aug_net_sizes": [64, 64]},
                  enc_params={"q_sizes": [32, 16], "ff_sizes": [16, 16], "SIR_scaler": [0.1, 0.05, 1.0]},
                  seed=2222, bayes=True)


def make_e2e_toy64():
    # the toy shapes of e2e_vae_step (S = 5, masked target), with the fp64 parity target
    make_e2e_case("e2e_vae_toy64", R=1, n_qs=3, B=4, S_=5, window=6, gamma=21,
                  ode_params={"net_sizes": [16, 16, 8], "aug_net_sizes": [16, 12]},
                  enc_params={"q_sizes": [16, 8], "ff_sizes": [8, 8], "SIR_scaler": [0.1, 0.05, 1.0]},
                  seed=4242)


if __name__ == "__main__":
    torch.set_num_threads(1)
    if len(sys.argv) > 1 and sys.argv[1] == "e2e_state49":
        make_e2e_state49()
    elif len(sys.argv) > 1 and sys.argv[1] == "e2e_us":
        make_e2e_us()
    elif len(sys.argv) > 1 and sys.argv[1] == "e2e_us_bayes":
        make_e2e_us_bayes()
    elif len(sys.argv) > 1 and sys.argv[1] == "e2e_toy64":
        make_e2e_toy64()
    else:
        if len(sys.argv) == 1:
            main()
        make_e2e()
