"""Drop-in for lib/Metrics.py (forecast scoring used by VAE.evaluate / validate)."""
import numpy as np
from scipy.stats import norm


def _unpack(true, mean, std):
    if hasattr(true, "columns"):
        return true["True"], true["Pred"], true["Std"]
    return true, mean, std


def nll(true, mean=None, std=None, bins=False):
    true, mean, std = _unpack(true, mean, std)
    return -np.mean(norm.logpdf(true, loc=mean, scale=std))


def mae(true, mean=None, std=None, bins=False):
    true, mean, std = _unpack(true, mean, std)
    return np.mean(np.abs(true - mean))


def mb_log(true, mean=None, std=None, bins=False):
    """log probability mass of [true - 0.5, true + 0.6] (CDC-style), floored at e^-10."""
    true, mean, std = _unpack(true, mean, std)
    d = norm(loc=mean, scale=std)
    mass = np.asarray(d.cdf(true + 0.6) - d.cdf(true - 0.5))
    mass = np.where(mass == 0, 4.5399929762484854e-05, mass)
    return np.log(mass)


def skill(true, mean=None, std=None, bins=False):
    return np.exp(mb_log(true, mean, std, bins).mean())
