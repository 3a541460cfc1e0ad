"""Synthetic stand-in for lib/regional_data_builder.py (DataConstructor :162-274,
convert_to_torch :276-284).

The reference builds its windows from CSVs under ``Data/`` (Google query frequencies and
CDC ILI rates), which are not part of the repository (``.gitignore:2``) and not available
here.  This stand-in keeps the class, its constructor / call signature and the exact
window shapes and layout, and fills them with seeded synthetic seasons instead:

* one daily ILI curve per region per season: an SIR epidemic (random R0, peak timing and
  amplitude), normalised per region by its maximum as the reference does (:210-211), with
  ``scaler = max * 13`` (:209) as a pandas Series over the regions;
* ``n_queries`` query series per region: noisy, lagged copies of that region's ILI curve,
  each divided by its own maximum (:199);
* windows exactly as :216-246: inputs ``(window_size + lag, R * n_queries + R)`` = every
  region's queries then the ILI columns, the last ``lag`` ILI rows set to -1; outputs
  ``(window_size + gamma + 1, R)`` with ``run_backward`` and ``no_qs_in_output`` (the call
  run_ode.py:141 makes), else ``(gamma, ...)`` from the window end;
* the test split is the windows starting in the last season (``test_season``), the train
  split every earlier window (the reference reads the split dates from Data/Dates.csv).

It exists so that run_ode.py's flow (data -> VAE -> curriculum training -> utils.test) runs
end to end on synthetic data of the reference's shapes; it is not a data pipeline.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.utils.data import DataLoader, TensorDataset

_N_REGIONS = {"hhs": 10, "state": 49}
SEASON_DAYS = 365


def _sir_curve(rng, n_days):
    """Daily infected fraction of one SIR season (forward Euler on a daily grid)."""
    r0 = rng.uniform(1.3, 2.2)
    gamma = 1.0 / rng.uniform(3.0, 6.0)
    beta = r0 * gamma
    s, i = 1.0 - 1e-4, 1e-4 * rng.uniform(0.5, 2.0)
    start = int(rng.integers(40, 120))
    out = np.zeros(n_days)
    for d in range(start, n_days):
        inf = beta * s * i
        s, i = s - inf, i + inf - gamma * i
        out[d] = i
    return out * rng.uniform(0.5, 1.5) + 0.002 * rng.uniform(0.5, 1.5)


class DataConstructor:
    def __init__(self, test_season, region="hhs", n_queries=10, gamma=28, window_size=28, lag=14, n_regions=10,
                 fill_1=False, root="checkpoints/HHS_SIR_Big_new/", n_seasons=4, seed=0):
        self.lag = lag
        self.window_size = window_size
        self.root = root
        self.test_season = test_season
        self.region = region
        self.n_queries = n_queries
        self.gamma = gamma
        self.fill_1 = fill_1
        self.n_regions = _N_REGIONS.get(region, 1)      # as :178-183: US (anything else) -> 1
        self.n_seasons = n_seasons
        self.seed = seed

    def _series(self):
        rng = np.random.default_rng([self.seed, int(self.test_season), self.n_regions, self.n_queries])
        n_days = self.n_seasons * SEASON_DAYS
        ili = np.stack([np.concatenate([_sir_curve(rng, SEASON_DAYS) for _ in range(self.n_seasons)])
                        for _ in range(self.n_regions)], -1)                       # (days, R)
        qs = []
        for r in range(self.n_regions):
            q = np.empty((n_days, self.n_queries))
            for k in range(self.n_queries):
                shift = int(rng.integers(-7, 8))
                q[:, k] = np.roll(ili[:, r], shift) * rng.uniform(0.5, 2.0) \
                    + rng.normal(0.0, 0.05 * ili[:, r].max(), n_days)
            q = np.clip(q, 0.0, None)
            qs.append(q / q.max(0, keepdims=True))                                # :199
        return ili, qs

    def __call__(self, run_backward=False, no_qs_in_output=False):
        import pandas as pd
        ili, qs = self._series()
        R = self.n_regions
        scaler = pd.Series(ili.max(0) * 13, index=[f"region {r + 1}" for r in range(R)])   # :209
        ili = ili / np.nanmax(ili, axis=0)                                               # :210
        w, lag, gamma = self.window_size, self.lag, self.gamma
        inputs, outputs, starts = [], [], []
        for batch in range(w + 1, ili.shape[0] - gamma):                                 # :216
            t_ili = ili[batch - w - 1: batch + lag - 1].copy()
            t_ili[-lag:, :] = -1
            x = np.concatenate([q[batch - w - 1: batch + lag - 1] for q in qs] + [t_ili], -1)
            if run_backward:
                lo, hi = batch - w - 1, batch + gamma
            else:
                lo, hi = batch, batch + gamma
            y = np.concatenate([q[lo:hi] for q in qs] + [ili[lo:hi]], -1)
            if no_qs_in_output:
                y = y[..., -R:]
            inputs.append(x)
            outputs.append(y)
            starts.append(batch)
        starts = np.asarray(starts)
        test_from = (self.n_seasons - 1) * SEASON_DAYS                                  # the test season
        tr = starts < test_from - gamma
        te = starts >= test_from
        x_all, y_all = np.asarray(inputs), np.asarray(outputs)
        return x_all[tr], y_all[tr], x_all[te], y_all[te], scaler


def convert_to_torch(x_train, y_train, x_test, y_test, batch_size=32, shuffle=True, dtype=torch.float32):
    """Tensors + a DataLoader over the training windows (reference :276-284)."""
    x_train = torch.tensor(x_train, dtype=dtype)
    y_train = torch.tensor(y_train, dtype=dtype)
    x_test = torch.tensor(x_test, dtype=dtype)
    y_test = torch.tensor(y_test, dtype=dtype)
    train_loader = DataLoader(dataset=TensorDataset(x_train, y_train), batch_size=batch_size, shuffle=shuffle)
    return train_loader, x_test, y_test
