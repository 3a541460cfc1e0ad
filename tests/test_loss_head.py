"""Fused loss head (csrc/ude_loss.h): decoder + nll_loss + latent_init_loss, forward and
backward, against fixtures made by the reference's own code in fp64
(tests/golden/make_golden_loss.py: lib/models.py:27-51 Decoder, lib/VAE.py:138 reshape /
permute, lib/train_functions.py:81-90 nll_loss, :116-126 latent_init_loss).

Tolerance: normwise relative 1e-5 for the loss values and the gradients (fp32 kernel vs
fp64 reference; the sample mean / std are fp32 sums over S <= 128 terms).  Cases include
S = 128 (the kernel's largest sample tile, ~157 KiB of LDS at R = 49) and ragged S."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from helpers import normwise_rel

sys.path.insert(0, GOLDEN)
import make_golden_loss as mgl  # noqa: E402  (input recipe only; runs no reference code)

DEV = "cuda"


def test_loss_fixture_inputs_regenerate():
    """The seeded input recipe reproduces the inputs the fixtures were made from."""
    for case in mgl.CASES:
        g = load_golden(mgl.case_name(case))
        assert np.allclose(mgl.checksum(*mgl.inputs(case)), g["meta"]["checksum"], rtol=0, atol=0)


def _ode_for(pkg, R, L):
    net, aug = ([40, 24], [36]) if R == 3 else ([64, 64, 32], [64, 64])     # prebuilt configurations
    return pkg.FaFp(R, latent_dim=L, net_sizes=net, aug_net_sizes=aug).to(DEV)


@pytest.mark.gpu
@pytest.mark.parametrize("case", mgl.CASES, ids=mgl.case_name)
def test_fused_loss_head_matches_reference(pkg, case):
    from ude_amd import loss_head
    R, L, T, S, B = case
    g = load_golden(mgl.case_name(case))
    latent, W, b, y = mgl.inputs(case)
    ode = _ode_for(pkg, R, L)
    lin = torch.nn.Linear(3 * R, R).to(DEV)
    with torch.no_grad():
        lin.weight.copy_(W)
        lin.bias.copy_(b)
    lat = latent.to(DEV).requires_grad_(True)
    assert loss_head.eligible(ode, lat, lin, S, B)
    nll, reg = loss_head.fused_loss_head(ode, lat, lin, y.to(DEV), S, B)
    (g["meta"]["g_nll"] * nll + g["meta"]["g_reg"] * reg).backward()
    assert normwise_rel(nll, g["nll"]) < 1e-5 and normwise_rel(reg, g["reg"]) < 1e-5
    assert normwise_rel(lat.grad[..., :3], g["dlat3"]) < 1e-5
    assert int(torch.count_nonzero(lat.grad[..., 3:])) == 0
    assert normwise_rel(lin.weight.grad, g["dW"]) < 1e-5 and normwise_rel(lin.bias.grad, g["db"]) < 1e-5


@pytest.mark.gpu
def test_loss_head_rejects_oversized_sample_tile(pkg):
    """S = 129 exceeds the kernel's sample tile: not eligible, so VAE.calc_loss takes the
    reference's own ops (it used to raise from the C-ABI)."""
    from ude_amd import loss_head
    R, L, T, S, B = 1, 8, 3, 129, 2
    ode = _ode_for(pkg, R, L)
    lin = torch.nn.Linear(3, 1).to(DEV)
    lat = torch.rand(T, S * B, R, L, device=DEV)
    assert not loss_head.eligible(ode, lat, lin, S, B)
    assert not loss_head.eligible(ode, lat[..., 1:], lin, S, B)              # not the model's L


def _vae_step(S, fused_ok, monkeypatch, mse=False, epilogue=False):
    """One VAE calc_loss + backward.  fused_ok: the fused loss head over a written latent may run;
    epilogue: the decoder-epilogue solve (y_hat from the forward kernel, no latent) may run."""
    import lib.VAE as vae_mod
    import lib.models as models
    from ude_amd import decoder_head, loss_head
    torch.manual_seed(3)
    model = vae_mod.VAE(models.Encoder_Back_GRU, models.FaFp, models.Decoder, 4, 8, 1,
                        ode_params={"net_sizes": [64, 64, 32], "aug_net_sizes": [64, 64]},
                        enc_params={"q_sizes": [16, 8], "ff_sizes": [8], "SIR_scaler": [0.1, 0.05, 1.0]})
    model.to(DEV)
    model.setup_training()
    gen = torch.Generator().manual_seed(5)
    x = torch.rand(3, 6, 5, generator=gen).to(DEV)
    y = (torch.rand(3, 3, 1, generator=gen) * 0.5).to(DEV)
    t = torch.arange(3, dtype=torch.float32)
    eps = torch.randn(S, 3, 1, 7, generator=gen).to(DEV)
    if not fused_ok:
        monkeypatch.setattr(loss_head, "eligible", lambda *a, **k: False)
    if not epilogue:
        monkeypatch.setattr(decoder_head, "eligible", lambda *a, **k: False)
    real_randn = torch.randn
    monkeypatch.setattr(torch, "randn", lambda *a, **k: eps.clone())
    y_pred = model(x, t, n_samples=S, training=True)
    monkeypatch.setattr(torch, "randn", real_randn)
    losses = {"nll": True, "mse": mse, "kl_z": True, "kl_p": True, "Fa_norm": 0.1, "reg_loss": True,
              "anneal": True}
    took_fused = model._fused_head(y_pred, y, losses) is not None
    loss, data, names = model.calc_loss(y_pred, y, losses)
    loss.backward()
    monkeypatch.undo()
    grads = {f"{part}.{k}": p.grad.detach().clone() for part in ("enc", "ode", "dec")
             for k, p in getattr(model, part).named_parameters()}
    return took_fused, loss.detach(), grads


@pytest.mark.gpu
def test_vae_calc_loss_fused_head_matches_eager(pkg, monkeypatch):
    """One batch through VAE.calc_loss with the fused head and with the reference's ops
    (loss_head disabled): the loss to 1e-5, every gradient to 5e-5 (the decoder gradients are
    sums with cancellation, where two fp32 summation orders differ by ~3e-5)."""
    f_on, loss_f, g_f = _vae_step(64, True, monkeypatch)
    f_off, loss_e, g_e = _vae_step(64, False, monkeypatch)
    assert f_on and not f_off
    assert normwise_rel(loss_f, loss_e) < 1e-5
    for k in g_e:
        assert normwise_rel(g_f[k], g_e[k]) < 5e-5, (k, normwise_rel(g_f[k], g_e[k]))


@pytest.mark.gpu
@pytest.mark.parametrize("mse", [False, True], ids=["nll_reg", "with_mse"])
def test_vae_calc_loss_decoder_epilogue_matches_eager(pkg, monkeypatch, mse):
    """the training step with the decoder epilogue (y_hat + latent_init_loss from the
    solve's forward kernel, no latent written; nll kernels; decoder backward from the checkpoint
    store) against the reference's own ops over a written latent: loss to 1e-5, every gradient to
    5e-5; with mse the prediction also feeds torch ops (d y_hat from two consumers)."""
    f_on, loss_f, g_f = _vae_step(64, False, monkeypatch, mse=mse, epilogue=True)
    f_off, loss_e, g_e = _vae_step(64, False, monkeypatch, mse=mse)
    assert f_on and not f_off
    assert normwise_rel(loss_f, loss_e) < 1e-5
    for k in g_e:
        assert normwise_rel(g_f[k], g_e[k]) < 5e-5, (k, normwise_rel(g_f[k], g_e[k]))


@pytest.mark.gpu
def test_decoder_epilogue_latent_materialised_on_read(pkg):
    """VAE.latent after a decoder-epilogue training call is rebuilt from the training store on
    first read: equal to the latent a plain solve writes, and differentiable (its cotangent
    reaches y0 / the weights through the solve's backward)."""
    import lib.VAE as vae_mod
    import lib.models as models
    from ude_amd.decoder_head import LazyLatent
    torch.manual_seed(3)
    model = vae_mod.VAE(models.Encoder_Back_GRU, models.FaFp, models.Decoder, 4, 8, 1,
                        ode_params={"net_sizes": [64, 64, 32], "aug_net_sizes": [64, 64]},
                        enc_params={"q_sizes": [16, 8], "ff_sizes": [8], "SIR_scaler": [0.1, 0.05, 1.0]})
    model.to(DEV)
    model.setup_training()
    gen = torch.Generator().manual_seed(5)
    x = torch.rand(3, 6, 5, generator=gen).to(DEV)
    t = torch.arange(4, dtype=torch.float32)
    model(x, t, n_samples=8, training=True)
    lazy = model.__dict__["_latent"]
    assert isinstance(lazy, LazyLatent) and not lazy.materialized
    lat = model.latent
    assert lazy.materialized and lat.shape == (4, 24, 1, 8)
    z = lat[0].detach()
    model.ode.clear_tracking()
    with torch.no_grad():
        ref = pkg.odeint(model.ode, z, t.to(DEV), method="rk4", options=dict(step_size=t[1] - t[0]))
    assert torch.equal(lat.detach(), ref)
    (lat[..., 1] * 0.5).sum().backward()                  # a loss built on the materialised latent
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in model.ode.parameters())


@pytest.mark.gpu
def test_vae_calc_loss_large_sample_count_runs_eager(pkg, monkeypatch):
    """n_samples = 129 (> the kernel's 128 tile): calc_loss takes the reference's ops, no error."""
    took_fused, loss, grads = _vae_step(129, True, monkeypatch)
    assert not took_fused and torch.isfinite(loss)


@pytest.mark.gpu
def test_compact_sir_cotangent_matches_full(pkg, monkeypatch):
    """the fused loss head hands the solve's backward only the S, I, R
    cotangents (ude_loss_head_backward_sir -> ude_rk4_backward_sir) instead of a full
    (T, N, R, L) d latent that is 5/8 zeros.  Same step with the hand-off disabled: identical
    loss and bit-identical gradients (the compact path adds the same values in the same order)."""
    from ude_amd import _native, loss_head
    calls = []
    real = _native.NativeLib.loss_backward_sir
    monkeypatch.setattr(_native.NativeLib, "loss_backward_sir",
                        lambda self, *a: (calls.append("sir"), real(self, *a))[1])
    f1, loss_c, g_c = _vae_step(64, True, monkeypatch)
    assert calls == ["sir"], calls
    calls.clear()
    monkeypatch.setattr(loss_head, "COMPACT", False)
    f2, loss_f, g_f = _vae_step(64, True, monkeypatch)
    assert f1 and f2 and not calls
    assert torch.equal(loss_c, loss_f)
    for k in g_f:
        assert torch.equal(g_c[k], g_f[k]), (k, normwise_rel(g_c[k], g_f[k]))


@pytest.mark.gpu
def test_compact_sir_cotangent_with_other_consumers(pkg, monkeypatch):
    """The latent also feeds the mse term (through the decoder): the solve's backward gets the
    full cotangent of that path plus the loss head's compact deposit, merged once."""
    from ude_amd import loss_head
    f1, loss_c, g_c = _vae_step(64, True, monkeypatch, mse=True)
    monkeypatch.setattr(loss_head, "COMPACT", False)
    f2, loss_f, g_f = _vae_step(64, True, monkeypatch, mse=True)
    assert f1 and f2 and torch.equal(loss_c, loss_f)
    for k in g_f:
        assert torch.equal(g_c[k], g_f[k]), (k, normwise_rel(g_c[k], g_f[k]))


@pytest.mark.gpu
def test_compact_sir_cotangent_retain_graph(pkg):
    """A backward that reaches the loss head but not the solve (decoder grads only, retain_graph)
    must not leak its S, I, R cotangent into a later backward through the solve: the compact
    cotangent travels on an autograd edge (the solve's sir_token output), not in shared state."""
    from ude_amd import loss_head
    torch.manual_seed(0)
    R, L, T, S, B = 1, 8, 5, 8, 4
    ode = pkg.FaFp(R, latent_dim=L, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]).to(DEV)
    dec = torch.nn.Linear(3 * R, R).to(DEV)
    gen = torch.Generator().manual_seed(1)
    Sv = torch.rand(S * B, R, generator=gen) * 0.4 + 0.5
    Iv = torch.rand(S * B, R, generator=gen) * 0.05
    y0 = torch.cat([Sv[..., None], Iv[..., None], (1 - Sv - Iv)[..., None], torch.randn(S * B, R, L - 3,
                                                                                        generator=gen)], -1)
    y0 = (y0 + 1e-5).to(DEV).requires_grad_(True)
    y = torch.rand(B, T, R, generator=gen).to(DEV)
    t = torch.arange(T, dtype=torch.float32).to(DEV)

    def run():
        ode.clear_tracking()
        lat = pkg.odeint(ode, y0, t, method="rk4", options=dict(step_size=t[1] - t[0]))
        assert loss_head.eligible(ode, lat, dec, S, B)
        nll, reg = loss_head.fused_loss_head(ode, lat, dec, y, S, B)
        return nll + 0.1 * reg

    loss = run()
    g_ref = torch.autograd.grad(loss, [y0], retain_graph=True)[0]
    loss2 = run()
    torch.autograd.grad(loss2, [dec.weight], retain_graph=True)     # reaches the head only
    g2 = torch.autograd.grad(loss2, [y0])[0]
    assert torch.equal(g_ref, g2)
