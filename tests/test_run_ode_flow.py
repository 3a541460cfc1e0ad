"""run_ode.py's flow against the drop-in lib/ (BASELINE configs[0]: a single US-region SIR-UDE
with the 32-hidden rate MLP, fixed-step RK4, one test season, CPU PyTorch).

The sequence of calls is the reference driver's (run_ode.py:125-167), on the synthetic
DataConstructor stand-in (Data/ is absent): make folders, build the windows, convert to
torch, construct the VAE from region_info['US'] with the ODE class Fp and net_sizes [32, 32],
setup_training, the gamma curriculum of model.train calls (eval_pts grown by a week at a
time, :147-164, with checkpointing, grad-norm tracking and validation), save, utils.test
into a results CSV under a FileLock, and append_to_line into the started file.  Shrunk
only in epochs / sample counts so it runs in seconds.
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch


def _run_ode_flow(tmp_path, device, region="US", ode_name="CONN", n_samples=8, test_n_samples=16):
    from torchdiffeq import odeint  # noqa: F401  (the import run_ode.py:24 makes)
    import lib.utils as utils
    from lib.regional_data_builder import DataConstructor, convert_to_torch
    from lib.models import Encoder_Back_GRU, Decoder, Fa, Fp, FaFp
    from lib.in_development.models_bayes import Bayes_Fa, Bayes_Fp, Bayes_FaFp
    from lib.VAE import VAE

    dtype = torch.float32
    region_info = {"US": {"n_regions": 1, "latent_dim": 8, "n_qs": 9,
                          "ode_params": {"net_sizes": [32, 32], "aug_net_sizes": [32, 32], "prior_std": 0.05},
                          "dec_params": {}, "enc_params": {"q_sizes": [16, 8], "ff_sizes": [8, 8],
                                                           "SIR_scaler": [0.1, 0.05, 1.0]}},
                   "hhs": {"n_regions": 10, "latent_dim": 8, "n_qs": 3,
                           "ode_params": {"net_sizes": [16, 16], "aug_net_sizes": [16, 16], "prior_std": 0.05},
                           "dec_params": {}, "enc_params": {"q_sizes": [16, 8], "ff_sizes": [8, 8],
                                                            "SIR_scaler": [0.1, 0.05, 1.0]}}}
    training_info = {"CONN": {"nll": True, "mse": False, "kl_z": True, "kl_p": True, "Fa_norm": False,
                              "reg_loss": True, "anneal": True},
                     "UONN": {"nll": True, "mse": False, "kl_z": True, "kl_p": True, "Fa_norm": 1e-1,
                              "reg_loss": True, "anneal": True}}
    ode = {"CONN": Fp, "UONN": FaFp, "SONN": Fa, "CONNb": Bayes_Fp, "UONNb": Bayes_FaFp, "SONNb": Bayes_Fa}[ode_name]
    epochs, window_size, gamma, latent_dim, num, test_season = 4, 8, 28, 8, 15, 2016
    os.chdir(tmp_path)
    started = "started.txt"
    common_prefix = f"{region}/{ode_name}/{test_season}_e{epochs}_g{gamma}_w{window_size}_{num}_"
    file_prefix, norm_prefix, chkpt_prefix = (f"weights/{common_prefix}", f"norms/{common_prefix}",
                                              f"chkpts/{common_prefix}")
    with open(started, "w") as f:
        f.write(file_prefix + "\n")
    pd.DataFrame({"epochs": [0]}).to_csv("results_table_server.csv")
    for p in (chkpt_prefix, file_prefix, norm_prefix):
        utils.make_file(p)

    t = torch.arange(window_size + gamma + 1, dtype=dtype) / 7
    losses = training_info[ode_name]
    ri = region_info[region]
    _data = DataConstructor(test_season=test_season, region=region, window_size=window_size,
                            n_queries=ri["n_qs"], gamma=gamma, n_seasons=2)
    x_train, y_train, x_test, y_test, scaler = _data(run_backward=True, no_qs_in_output=True)
    R = ri["n_regions"]
    assert x_train.shape[1:] == (window_size + 14, R * (ri["n_qs"] + 1))
    assert y_train.shape[1:] == (window_size + gamma + 1, R) and y_test.shape[1:] == y_train.shape[1:]
    # keep the loop short: a few training windows, a few test windows
    x_train, y_train, x_test, y_test = x_train[:40], y_train[:40], x_test[:6], y_test[:6]
    train_loader, x_test, y_test = convert_to_torch(x_train, y_train, x_test, y_test, batch_size=32,
                                                    shuffle=True, dtype=dtype)
    model = VAE(Encoder_Back_GRU, ode, Decoder, ri["n_qs"], latent_dim, R, file_prefix=file_prefix,
                chkpt_prefix=chkpt_prefix, ode_params=ri["ode_params"], enc_params=ri["enc_params"],
                dec_params=ri["dec_params"], uncertainty=True, ode_kl_w=1 / 153)
    if device != "cpu":
        model.to(device)
        train_loader = [(x.to(device), y.to(device)) for x, y in train_loader]
        x_test, y_test = x_test.to(device), y_test.to(device)
    model.setup_training(lr=1e-3)
    eval_all = list(np.linspace(0, gamma, int((gamma / 7) + 1), dtype=int))
    epochs_per_cycle = int(epochs / (len(eval_all) - 1))
    for i in range(2, len(eval_all) + 1):
        eval_pts = eval_all[:i]
        time_steps = t[:(eval_pts[-1] + 1)]
        model.train(train_loader, time_steps, epochs_per_cycle, losses, eval_pts, n_samples=n_samples,
                    grad_lim=5000, checkpoint=True, track_norms=True, norm_file=f"{norm_prefix}norms.txt",
                    disable=True, validate={"x_test": x_test, "y_test": y_test, "t": t, "scaler": scaler,
                                            "n_samples": 4})
    model.save()
    variables = {"epochs": epochs, "gamma": gamma, "ode_name": ode_name, "region": region,
                 "latent_dim": latent_dim, "window_size": window_size, "num": num}
    utils.test(model, scaler, x_test, y_test, t, test_season=test_season, window_size=window_size,
               variables=variables, n_samples=test_n_samples, file_name="results_table_server")
    utils.append_to_line(started, file_prefix, append="finished")
    return model, epochs, window_size, test_season, file_prefix


def _check_outputs(model, epochs, window_size, test_season, file_prefix):
    hist = model._history.epoch_history
    assert len(hist) == epochs and all(np.isfinite(h["loss"]) for h in hist)
    assert all("forecast_nll" in h for h in hist)
    for part in ("enc", "ode", "dec"):
        assert os.path.exists(f"{file_prefix}{part}.pth")
    res = pd.read_csv("results_table_server.csv", index_col=0)
    row = res[res["ode_name"] == "CONN"] if "ode_name" in res else res
    cols = [f"{test_season} {window_size + 6}", f"skill {test_season} 28"]
    assert all(c in res.columns for c in cols)
    assert np.isfinite(row[cols].values.astype(float)).all()
    with open("started.txt") as f:
        assert f.read().strip().endswith("finished")
    # the saved ODE weights load back into the reference-named module
    sd = torch.load(f"{file_prefix}ode.pth", weights_only=True)
    assert set(sd) == set(model.ode.state_dict())


def test_run_ode_flow_us_fp32_cpu(pkg, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    torch.manual_seed(0)
    _check_outputs(*_run_ode_flow(tmp_path, "cpu"))


@pytest.mark.gpu
def test_run_ode_flow_us_fp32_gpu(pkg, tmp_path, monkeypatch):
    """The same flow with the model on the MI355X: every solve (training, validation, test)
    runs on the fused kernels."""
    monkeypatch.chdir(tmp_path)
    torch.manual_seed(0)
    _check_outputs(*_run_ode_flow(tmp_path, "cuda"))
