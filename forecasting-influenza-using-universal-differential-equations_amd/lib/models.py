"""Drop-in for lib/models.py.

The ODE right-hand sides (Fp, Fa, FaFp -- the hot path) come from ude_amd and
run on the fused gfx950 RK4 kernel inside ``odeint``; the encoder / decoder and
the reparameterisation helpers around them stay plain PyTorch (they are outside
the accelerated path).
"""
import torch
from torch import nn
from torch.distributions import Normal

from ude_amd.rhs import Fp, Fa, FaFp  # noqa: F401
import lib.utils as utils


def make_prior(mean, z_prior=torch.tensor([0.1, 0.01]), device="cpu", latent_dim=8):
    """Prior over the encoder latent (lib/models.py:9-14): N([S0, I0, 0...], [0.1, 0.01, 1...])."""
    z_prior = z_prior.to(device)
    loc = torch.cat((mean[..., :2], torch.zeros_like(mean[..., 2:], device=device)), dim=-1)
    tail = torch.ones(latent_dim - len(z_prior) - 1, device=device)
    scale = torch.cat([z_prior[:1], z_prior[1:2], tail], 0).expand_as(loc)
    return Normal(loc, torch.abs(scale))


def reparam(eps, std, mean, n_samples, batch_size, uncertainty=True):
    """SIR simplex y0 from encoder samples (lib/models.py:16-24), shape (S*B, R, L)."""
    z = eps * std + mean if uncertainty else mean
    si = torch.abs(z[..., :2])
    z = torch.concat([si, (1 - si.sum(-1)).unsqueeze(-1), z[..., 2:]], -1)
    return z.reshape((n_samples * batch_size,) + z.shape[2:])


class Decoder(nn.Module):
    """Linear map from the S, I, R compartments to ILI per region (lib/models.py:26-51)."""

    def __init__(self, n_regions, latent_dim, input_dim, Fp=True, device=torch.device("cpu"),
                 dtype=torch.float32, **kwargs):
        super().__init__()
        self.Fp = Fp
        self.n_regions = n_regions
        self.input_dim = input_dim
        self.latent_dim = 3 if Fp else latent_dim
        self.decoder = nn.Sequential(nn.Flatten(), nn.Linear(n_regions * self.latent_dim, n_regions * input_dim))
        self.decoder.to(device=device, dtype=dtype)
        utils.init_network_weights(self.decoder)

    def forward(self, data):
        data = data[..., :self.latent_dim]
        lead = data.shape[:2]
        out = self.decoder(data.reshape((-1,) + tuple(data.shape[2:])))
        return out.reshape(tuple(lead) + (-1,))


class Encoder_Back_GRU(nn.Module):
    """Time-reversed stacked GRU -> MLP -> (mean, |std| * scaler) (lib/models.py:53-107)."""

    def __init__(self, n_regions, n_qs=9, latent_dim=6, q_sizes=[128, 64], ff_sizes=[32],
                 SIR_scaler=[0.1, 0.05, 1.0], uncertainty=True, device="cpu", dtype=torch.float32, **kwargs):
        super().__init__()
        self.latent_dim = latent_dim
        self.n_regions = n_regions
        self.device, self.dtype = device, dtype
        self.uncertainty = uncertainty
        sc = torch.tensor(SIR_scaler, dtype=dtype, device=device)
        if latent_dim > len(sc):
            sc = torch.cat([sc, sc[-1].repeat(latent_dim - len(sc))])
        self.scaler = sc.view(1, -1)
        widths = [n_regions * (n_qs + 1)] + list(q_sizes)
        self.rnn_layers = nn.ModuleList(nn.GRU(a, b, batch_first=True) for a, b in zip(widths[:-1], widths[1:]))
        ff = nn.ModuleList([nn.Linear(q_sizes[-1], ff_sizes[0])])
        for a, b in zip(ff_sizes[:-1], ff_sizes[1:]):
            ff.extend([nn.ReLU(), nn.Linear(a, b)])
        n_out = n_regions * latent_dim * (2 if uncertainty else 1)
        ff.append(nn.Linear(ff_sizes[-1] if len(ff_sizes) > 1 else ff_sizes[0], n_out))
        self.ff_layers = ff

    def forward(self, x):
        h = x.flip(1)
        for gru in self.rnn_layers:
            h, _ = gru(h)
        h = h[:, -1, :]
        for layer in self.ff_layers:
            h = layer(h)
        shape = (-1, self.n_regions, self.latent_dim)
        if not self.uncertainty:
            return h.reshape(shape)
        mean, raw_std = torch.split(h, h.size(-1) // 2, dim=-1)
        return mean.reshape(shape), torch.abs(raw_std.reshape(shape)) * self.scaler
