"""Drop-in for lib/utils.py host helpers (test :20-56, append_to_line :58-67,
init_network_weights :69-73, update_learning_rate :75-79, make_file :81-84)."""
import os

import numpy as np
import torch.nn as nn

import lib.Metrics as Metrics


def _np(x):
    return x.detach().cpu().numpy()


def test(model, scaler, x_test, y_test, t, test_season, window_size=1, variables={"ode_name": "CONN"},
         n_samples=128, file_name="results_table"):
    """Forward-only forecast of the test windows at n_samples MC samples (run_ode.py:166 calls it
    with 128), scored per horizon (7/14/21/28 days after the window) with Metrics.nll / skill
    into ``<file_name>.csv`` under a FileLock: the row whose ``variables`` all match is updated,
    else a new row is appended.  The forecast runs wherever the model lives (the fused solve on
    a HIP device); the scoring reads it back to the host."""
    import pandas as pd
    from filelock import FileLock
    y_pred = model(x_test, t, n_samples=n_samples, training=False)
    s = scaler.values if hasattr(scaler, "values") else np.asarray(scaler)
    y_pr = _np(y_pred) * s[np.newaxis, np.newaxis, np.newaxis, :]
    y_te = _np(y_test) * s[np.newaxis, np.newaxis, :]
    pred_mean = y_pr.mean(1)
    pred_std = y_pr.std(1)
    with FileLock(file_name + ".lock"):
        results_df = pd.read_csv(file_name + ".csv", index_col=0)
        common = None
        for key, value in variables.items():
            if key not in results_df.columns:
                continue
            idx = np.where(results_df[key] == value)[0]
            common = idx if common is None else np.intersect1d(common, idx)
        if common is not None and len(common) > 0:
            row = np.min(common)
        else:
            row = (np.max(results_df.index) + 1) if len(results_df.index) else 0
        for key, value in variables.items():
            results_df.loc[row, key] = value
        for col, g in zip([7, 14, 21, 28], [window_size + 6, window_size + 13, window_size + 20, window_size + 27]):
            results_df.loc[row, f"{test_season} {g}"] = Metrics.nll(y_te[:, g, :], pred_mean[:, g, :],
                                                                    pred_std[:, g, :])
            results_df.loc[row, f"skill {test_season} {col}"] = Metrics.skill(y_te[:, g, :], pred_mean[:, g, :],
                                                                              pred_std[:, g, :])
        results_df.to_csv(file_name + ".csv")


def init_network_weights(net, std=0.1):
    """N(0, std) weights, zero biases for every nn.Linear in ``net``."""
    for m in net.modules():
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0, std=std)
            nn.init.constant_(m.bias, val=0)


def update_learning_rate(optimizer, decay_rate=0.999, lowest=1e-3):
    for group in optimizer.param_groups:
        group["lr"] = max(group["lr"] * decay_rate, lowest)


def make_file(prefix):
    folder = os.path.dirname(prefix)
    if folder and not os.path.exists(folder):
        os.makedirs(folder)


def append_to_line(file_path, line_prefix, append="finished"):
    from filelock import FileLock
    with FileLock(file_path + ".lock"):
        with open(file_path) as f:
            rows = f.readlines()
        with open(file_path, "w") as f:
            for row in rows:
                f.write(row.rstrip("\n") + " " + append + "\n" if row.startswith(line_prefix) else row)
