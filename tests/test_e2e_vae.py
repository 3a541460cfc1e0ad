"""End-to-end caller contract: one VAE training step of the
drop-in lib/VAE.py (encoder -> reparam -> odeint -> decoder -> calc_loss ->
backward) against the reference VAE's own step (tests/golden/e2e_vae_step.npz,
reference lib/VAE.py + lib/models.py with the oracle RK4 as torchdiffeq).
CPU: the eager solver path; GPU: the fused kernel."""
import importlib
import sys

import numpy as np
import pytest
import torch

from conftest import load_golden
from helpers import normwise_rel


def _build(pkg, g, device):
    import lib.VAE as vae_mod
    import lib.models as models
    m = g["meta"]
    model = vae_mod.VAE(models.Encoder_Back_GRU, models.FaFp, models.Decoder, m["n_qs"], 8, 1,
                        ode_params=dict(m["ode_params"], prior_std=0.05), enc_params=m["enc_params"],
                        uncertainty=True, ode_kl_w=1 / 153)
    for part in ("enc", "ode", "dec"):
        mod = getattr(model, part)
        sd = {k[len(part) + 3:]: torch.from_numpy(g[k]) for k in g if k.startswith(f"w_{part}.")}
        mod.load_state_dict(sd, strict=True)
    model.to(device)
    model.setup_training(lr=1e-3)
    return model


def _step(pkg, g, device, monkeypatch):
    model = _build(pkg, g, device)
    eps = torch.from_numpy(g["eps"]).to(device)
    monkeypatch.setattr(torch, "randn", lambda *a, **k: eps.clone())
    x = torch.from_numpy(g["x"]).to(device)
    y = torch.from_numpy(g["y"]).to(device)
    t = torch.from_numpy(g["t"])
    ev = g["eval_pts"]
    model.optimizer.zero_grad()
    y_pred = model(x, t[ev], n_samples=g["meta"]["n_samples"], training=True)
    loss, data, names = model.calc_loss(y_pred, y[:, ev, :], g["meta"]["losses"])
    loss.backward()
    monkeypatch.undo()
    return model, loss, y_pred, names, data


def _check(g, model, loss, y_pred, names, tol):
    assert names == g["meta"]["loss_names"]
    assert abs(float(loss.detach()) - float(g["loss"][0])) <= tol * abs(float(g["loss"][0]))
    assert normwise_rel(y_pred, g["y_pred"]) < tol
    assert normwise_rel(model.latent, g["latent"]) < tol
    for part in ("enc", "ode", "dec"):
        for k, p in getattr(model, part).named_parameters():
            ref = g[f"g_{part}.{k}"]
            assert normwise_rel(p.grad, ref) < 20 * tol, (part, k, normwise_rel(p.grad, ref))


def test_vae_step_cpu_matches_reference(pkg, monkeypatch):
    g = load_golden("e2e_vae_step")
    model, loss, y_pred, names, data = _step(pkg, g, "cpu", monkeypatch)
    _check(g, model, loss, y_pred, names, 1e-5)  # fp32 CPU reductions differ across host ISAs (AVX2 vs AVX-512)


@pytest.mark.gpu
def test_vae_step_fused_matches_reference(pkg, monkeypatch):
    g = load_golden("e2e_vae_step")
    model, loss, y_pred, names, data = _step(pkg, g, "cuda", monkeypatch)
    assert pkg.fusable(model.ode, torch.zeros(1, 1, 8, device="cuda"))
    _check(g, model, loss, y_pred, names, 2e-5)
