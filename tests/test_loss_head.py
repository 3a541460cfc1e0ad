"""Fused loss head (csrc/ude_loss.h): decoder + nll_loss + latent_init_loss, forward and
backward, against the same terms computed with the reference's formulas in fp64
(lib/models.py:27-51 Decoder, lib/VAE.py:138 reshape/permute,
lib/train_functions.py:81-90 nll_loss, :116-126 latent_init_loss).

Tolerance: normwise relative 1e-5 for the loss values and the gradients (fp32 kernel vs
fp64 reference; the sample mean / std are fp32 sums over S <= 64 terms)."""
import pytest
import torch

from helpers import normwise_rel

DEV = "cuda"


def _reference(latent, W, b, y, S, B, g_nll, g_reg):
    import lib.train_functions as tf
    lat = latent.detach().double().requires_grad_(True)
    Wd = W.detach().double().requires_grad_(True)
    bd = b.detach().double().requires_grad_(True)
    T, N, R, L = lat.shape
    x = lat[..., :3]
    dec = torch.nn.functional.linear(x.reshape(-1, R * 3), Wd, bd).reshape(T, N, R)
    y_pred = dec.reshape((-1, S, B, R)).permute(2, 1, 0, 3)
    nll = tf.nll_loss(y_pred, y.double())
    reg = tf.latent_init_loss(x)
    (g_nll * nll + g_reg * reg).backward()
    return nll.detach(), reg.detach(), lat.grad, Wd.grad, bd.grad


CASES = [  # R, L, T, S, B
    (1, 8, 9, 64, 32), (10, 8, 5, 64, 8), (49, 8, 3, 64, 6), (1, 8, 4, 5, 4), (3, 5, 6, 17, 3),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "R{}_L{}_T{}_S{}_B{}".format(*c))
def test_fused_loss_head_matches_reference(pkg, case):
    from ude_amd import loss_head
    R, L, T, S, B = case
    torch.manual_seed(R * 100 + S)
    net, aug = ([40, 24], [36]) if R == 3 else ([64, 64, 32], [64, 64])     # prebuilt configurations
    ode = pkg.FaFp(R, latent_dim=L, net_sizes=net, aug_net_sizes=aug).to(DEV)
    gen = torch.Generator().manual_seed(7)
    latent = (torch.rand(T, S * B, R, L, generator=gen) * 2.0 - 0.5)
    W = torch.randn(R, 3 * R, generator=gen) * 0.3
    b = torch.randn(R, generator=gen) * 0.1
    y = torch.rand(B, T, R, generator=gen)
    y[0, 0, 0] = -1.0
    y[-1, -1, -1] = -1.0
    lin = torch.nn.Linear(3 * R, R).to(DEV)
    with torch.no_grad():
        lin.weight.copy_(W)
        lin.bias.copy_(b)
    lat = latent.to(DEV).requires_grad_(True)
    assert loss_head.eligible(ode, lat, lin, S, B)
    nll, reg = loss_head.fused_loss_head(ode, lat, lin, y.to(DEV), S, B)
    g_nll, g_reg = 0.7, 0.1
    (g_nll * nll + g_reg * reg).backward()
    rn, rr, rl, rW, rb = _reference(latent, W, b, y, S, B, g_nll, g_reg)
    assert normwise_rel(nll, rn) < 1e-5 and normwise_rel(reg, rr) < 1e-5
    assert normwise_rel(lat.grad, rl) < 1e-5
    assert torch.equal(lat.grad[..., 3:].cpu(), torch.zeros_like(rl[..., 3:]).float())
    assert normwise_rel(lin.weight.grad, rW) < 1e-5 and normwise_rel(lin.bias.grad, rb) < 1e-5
