"""Drop-in for lib/train_functions.py: the loss helpers lib/VAE.py composes around
the ODE solve (KL_annealing :17-44, get_kl_params :77-80, nll_loss :81-90,
make_prior / reparam :92-102, latent_init_loss :116-126, history :142-176,
kl_div :178-179, make_file :12-15) with the reference's signatures."""
import os
import subprocess

import numpy as np
import torch
from torch.distributions import Normal, kl_divergence  # noqa: F401  (re-exported, lib/VAE.py:167)

from lib.models import make_prior, reparam  # noqa: F401


def make_file(prefix):
    folder = "/".join(prefix.split("/")[:-1])
    if folder and not os.path.exists(folder):
        os.makedirs(folder)


def KL_annealing(step, anneal_params):
    """KL weight schedule: linear / sigmoid / cosine ramp over reset_pos*split steps, then flat."""
    if not anneal_params.get("anneal", True):
        return 1
    period = anneal_params.get("reset_pos", 10000)
    split = anneal_params.get("split", 0.5)
    lo, hi = anneal_params.get("lower", 0.0), anneal_params.get("upper", 1.0)
    kind = anneal_params.get("type", "linear")
    while step > period:
        step -= period
    ramp = int(period * split)
    if step >= ramp:
        return hi
    frac = step / ramp
    if kind == "linear":
        return lo + frac * (hi - lo)
    if kind == "sigmoid":
        return lo + (hi - lo) / (1 + np.exp(-10 * (frac - 0.5)))
    if kind == "cosine":
        return lo + 0.5 * (1 - np.cos(np.pi * frac)) * (hi - lo)
    return None


def get_kl_params(epoch, Q, means=[0.8, 0.55], stds=[0.2, 0.2], device="cpu", limit=1e10):
    """KL(N(means, stds) || Q).mean() -- Q is ode.posterior() (lib/VAE.py:173)."""
    if epoch >= limit:
        return torch.tensor(0)
    prior = Normal(torch.tensor(means, device=device), torch.tensor(stds, device=device))
    return kl_divergence(prior, Q).mean()


def nll_loss(y_pred, y, mean=True):
    """Gaussian NLL of y under the MC-sample mean/std (dim 1); entries with y == -1 are masked."""
    dist = Normal(torch.mean(y_pred, 1), torch.std(y_pred, 1))
    out = -dist.log_prob(y) * (y != -1).float()
    return out.mean() if mean else out


def latent_init_loss(x):
    """sum over entries of (|x| where x < 0) + (|1 - x| where x > 1)."""
    zero = torch.zeros_like(x)
    return (torch.where(x < 0, abs(x), zero) + torch.where(x > 1, abs(1 - x), zero)).sum()


def kl_div(Q_mu, Q_std, P_mu, P_std):
    return torch.sum(kl_divergence(Normal(Q_mu, Q_std), Normal(P_mu, P_std)), -1)


def get_free_gpu():
    """Index of the GPU with the most free memory (rocm-smi on ROCm)."""
    try:
        import torch.cuda as tc
        free = [tc.mem_get_info(i)[0] for i in range(tc.device_count())]
        return int(np.argmax(free)) if free else 0
    except Exception:
        out = subprocess.run(["rocm-smi", "--showmeminfo", "vram", "--csv"], capture_output=True, text=True).stdout
        rows = [r.split(",") for r in out.strip().splitlines()[1:]]
        free = [int(r[1]) - int(r[2]) for r in rows if len(r) >= 3]
        return int(np.argmax(free)) if free else 0


class history:
    """Per-batch loss records -> per-epoch means (lib/train_functions.py:142-176)."""

    def __init__(self):
        self.batches = []
        self.batch_history = []
        self.epoch_history = []

    def batch(self, data=None, names=None, batch=None):
        if batch is None:
            batch = dict(zip(names, data))
        for k, v in list(batch.items()):
            if torch.is_tensor(v):
                batch[k] = v.detach().cpu().numpy()
        self.batches.append(batch)

    def epoch(self):
        return {k: np.asarray([b[k] for b in self.batches]).mean() for k in self.batches[0]}

    def reset(self):
        self.batch_history.append(self.batches)
        self.epoch_history.append(self.epoch())
        self.batches = []
