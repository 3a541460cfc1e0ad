"""Drop-in for lib/VAE.py: the VAE whose forward calls the hot path.

``VAE.__call__`` (reference :118-140) draws eps, encodes, builds
``y0 = reparam(...) + 1e-5`` and calls ``odeint(ode, y0, t, method='rk4',
options=dict(step_size=t[1]-t[0]))`` -- here served by the fused gfx950 kernel
when the model lives on a HIP device -- then decodes ``latent[..., :3]``.
``calc_loss`` (:142-198) reads the solver's side outputs exactly as the
reference does (``ode.posterior()``, ``torch.norm(torch.stack(ode.tracker))``,
``self.latent``) and ``train_step`` (:200-223) back-propagates through the solve.
On a HIP device the ``nll`` and ``reg_loss`` terms of the model's own training
prediction come from the fused loss head (ude_amd/loss_head.py: decoder +
nll_loss + latent_init_loss, forward and backward in one kernel pass each).
"""
from itertools import chain

import numpy as np
import torch
import tqdm
from torch.distributions import Normal
from torch.optim.lr_scheduler import LambdaLR
from torchdiffeq import odeint

import lib.Metrics as Metrics
import lib.models as models
import lib.train_functions as train_functions
from lib.in_development.models_bayes import Dense_Variational
from ude_amd import loss_head


def warm_up_lr(epoch):
    return 1e-3 * (epoch + 1) / 10 if epoch < 10 else 1e-3


def print_rounded_dict(dictionary, decimals=3):
    print({k: round(v, decimals) if isinstance(v, (int, float)) else v for k, v in dictionary.items()})


def _scale_forecast(y_pred, y_test, scaler):
    s = scaler.values if hasattr(scaler, "values") else np.asarray(scaler)
    return y_pred.detach().cpu().numpy() * s[None, None, None, :], y_test.detach().cpu().numpy() * s[None, None, :]


def evaluate(model, x_test, y_test, t, scaler, n_samples=128):
    y_pr, y_te = _scale_forecast(model(x_test, t, n_samples=n_samples), y_test, scaler)
    mu, sd = y_pr.mean(1), y_pr.std(1)
    nlls = [Metrics.nll(y_te[:, g, :], mu[:, g, :], sd[:, g, :]) for g in range(57)]
    return {"forecast_nll": np.mean(nlls[-28:]), "all_nll": np.mean(nlls)}


class VAE:
    def __init__(self, enc, ode, dec, n_qs, latent_dim, n_regions=1, ode_type="Fp", len_tr=130,
                 file_prefix=None, chkpt_prefix=None, prior_params={"means": [0.8, 0.55], "stds": [0.2, 0.2]},
                 device="cpu", ode_params={}, enc_params={}, dec_params={}, kl_w=1, ode_kl_w=1,
                 uncertainty=True, dtype=torch.float32):
        self.kl_w, self.ode_kl_w = kl_w, ode_kl_w
        self.dtype, self.device = dtype, device
        self.tr_step = 0
        self.n_regions = n_regions
        self.len_tr = len_tr
        self.ld_ode = latent_dim
        self.uncertainty = uncertainty
        self.ode = ode(n_regions, latent_dim=self.ld_ode, **ode_params)
        self.file_prefix, self.chkpt_prefix = file_prefix, chkpt_prefix
        self.ode_type = getattr(self.ode, "ode_type", ode_type)
        if ode_type == "Fa":
            self.ld_enc = latent_dim
        else:
            self.ld_enc = latent_dim - 1
            self.ld_dec = 3
        self.enc = enc(n_regions, n_qs=n_qs, latent_dim=self.ld_enc, device=device, dtype=dtype,
                       uncertainty=uncertainty, **enc_params)
        self.dec = dec(n_regions, latent_dim=self.ld_dec, input_dim=1, **dec_params)
        self.anneal_params = {"anneal": True, "reset_pos": 10000, "split": 0.5, "lower": 0.0, "upper": 1.0,
                              "type": "cosine"}
        self.batch_grad_norms = []
        self.prior_params = prior_params
        self.started = False
        self.skip_count = 0

    def to(self, device):
        """Move encoder / ODE / decoder (the reference pins 'cpu'; here a HIP device runs the fused solve)."""
        self.device = device
        for m in (self.enc, self.ode, self.dec):
            m.to(device)
        self.enc.scaler = self.enc.scaler.to(device)
        return self

    def update_priors(self, new_std=0.1):
        for net_name in ("aug_net", "Fp_net"):
            net = getattr(self.ode, net_name, None)
            if net is not None:
                for layer in net.modules():
                    if isinstance(layer, Dense_Variational):
                        layer.prior_std = new_std

    def parameters(self):
        return chain(self.enc.parameters(), self.ode.parameters(), self.dec.parameters())

    def setup_training(self, lr=1e-3):
        self.optimizer = torch.optim.Adam(self.parameters(), lr=lr)
        self._history = train_functions.history()

    def __call__(self, x, t, n_samples=32, training=False):
        B = x.shape[0]
        eps = torch.randn(n_samples, B, self.n_regions, self.ld_enc, dtype=self.dtype, device=self.device)
        self.ode.clear_tracking()
        if training:
            self.optimizer.zero_grad()
        step = t[1] - t[0]
        with torch.set_grad_enabled(training):
            if self.uncertainty:
                self.mean, self.std = self.enc(x)
                z = models.reparam(eps, self.std, self.mean, n_samples, B, uncertainty=True) + 1e-5
            else:
                n_samples = 1
                self.mean = self.enc(x)
                z = (models.reparam(eps, None, self.mean, n_samples, B, uncertainty=False) + 1e-5).unsqueeze(1)
            self.latent = odeint(self.ode, z, t, method="rk4", options=dict(step_size=step))
            decoded = self.dec(self.latent[..., :3])
            y_pred = decoded.reshape((-1, n_samples, B, self.n_regions)).permute(2, 1, 0, 3)
        # calc_loss may take nll / reg from the fused loss head when handed this prediction
        self._pred_src = (y_pred, n_samples, B) if training else None
        return y_pred

    def _fused_head(self, y_pred, y_true, losses):
        """(nll, reg) from the fused gfx950 loss head (ude_amd/loss_head.py), or None when
        y_pred is not this model's latest training prediction or the shapes do not fit."""
        src = getattr(self, "_pred_src", None)
        if not (losses.get("nll", True) or losses.get("reg_loss", True)) or src is None or src[0] is not y_pred:
            return None
        lin = self.dec.decoder[-1]
        if getattr(self.dec, "latent_dim", None) != 3 or not hasattr(self.ode, "ude_config"):
            return None
        if not loss_head.eligible(self.ode, self.latent, lin, src[1], src[2]):
            return None
        return loss_head.fused_loss_head(self.ode, self.latent, lin, y_true, src[1], src[2], group_stats=True)

    @staticmethod
    def _validate_normals(checks):
        """The Normal argument checks the reference's nll_loss / posterior() get from
        torch.distributions (scale > 0, finite loc), for parameters that live on a HIP device:
        one batched read-back (calc_loss reads its loss terms back anyway) instead of one per
        Normal; raises ValueError as torch's validation does."""
        if not checks:
            return
        flags = torch.stack([((~(scale > 0)).any() | (loc != loc).any()) for _, loc, scale in checks]).cpu()
        for (what, loc, scale), bad in zip(checks, flags.tolist()):
            if bad:
                raise ValueError(f"Expected parameters loc / scale of distribution Normal ({what}) to satisfy the "
                                 "constraints Real() / GreaterThan(lower_bound=0.0), but found invalid values")

    def calc_loss(self, y_pred, y_true, losses):
        terms = {}
        if losses.get("anneal", True):
            self.tr_step += 1
            self.kl_w = train_functions.KL_annealing(self.tr_step, self.anneal_params)
        if losses.get("mse", True):
            terms["mse"] = torch.mean(torch.square(y_pred - y_true.unsqueeze(1)))
        fused = self._fused_head(y_pred, y_true, losses)
        checks = []
        if fused is not None:
            checks.append(("nll_loss prediction mean / std", fused[2][..., 0], fused[2][..., 1]))
        if losses.get("nll", True):
            terms["nll"] = fused[0] if fused is not None else train_functions.nll_loss(y_pred, y_true)
        if losses.get("kl_z", True):
            prior = models.make_prior(self.mean, latent_dim=self.ld_ode, device=self.device)
            kl = train_functions.kl_divergence(prior, Normal(self.mean, self.std)).sum(-1).mean()
            terms["kl_latent"] = self.kl_w * kl / self.len_tr
        if losses.get("kl_p", True):
            post = self.ode.posterior()
            if post.loc.is_cuda:
                checks.append(("ode.posterior()", post.loc, post.scale))
            terms["kl_params"] = train_functions.get_kl_params(
                1, post, means=self.prior_params["means"], stds=self.prior_params["stds"],
                limit=1e6, device=self.device)
        norm = None
        if losses.get("Fa_norm", 0) > 0:
            norm = torch.norm(torch.stack(self.ode.tracker))
            terms["Fa_norm"] = losses["Fa_norm"] * norm
        if losses.get("reg_loss", True):
            terms["reg_loss"] = 0.1 * (fused[1] if fused is not None
                                       else train_functions.latent_init_loss(self.latent[..., :3]))
        if self.ode.uncertainty == "bayes":
            terms["ode_kl"] = self.ode_kl_w * self.ode.get_kl()
        self._validate_normals(checks)
        loss = torch.tensor(0.0, requires_grad=True)
        for v in terms.values():
            loss = loss + v
        names, data = ["loss"], [round(loss.cpu().item(), 3)]
        if losses.get("anneal", True):
            names.append("kl_w"); data.append(round(self.kl_w, 3))
        for k, v in terms.items():
            names.append(k)
            data.append(round((norm if k == "Fa_norm" else v).cpu().item(), 3))
        return loss, data, names

    def train_step(self, x, y, t, epoch, losses, eval_pts, grad_lim=300, n_samples=32, track_norms=False,
                   norm_file="grad_norms.txt"):
        y_pred = self(x, t[eval_pts], n_samples=n_samples, training=True)
        loss, data, names = self.calc_loss(y_pred, y[:, eval_pts, :], losses=losses)
        loss.backward()
        grad_norm = torch.norm(torch.cat([p.grad.reshape(-1) for p in self.parameters() if p.grad is not None]), 2).item()
        self.batch_grad_norms.append(grad_norm)
        if grad_norm < grad_lim or self.skip_count >= 4 or epoch <= 3:
            self.optimizer.step()
            self.skip_count = 0
        else:
            self.skip_count += 1
        data.append(round(grad_norm, 1)); names.append("grad_norm")
        if track_norms:
            if not self.started:
                open(norm_file, "w").close()
                self.started = True
            self.norms.append(round(grad_norm, 1))
        return data, names

    def pre_train(self, train_loader, epochs=3, lr=1e-3, disable=False):
        opt = torch.optim.Adam(self.enc.parameters(), lr=lr)
        for epoch in range(1, epochs + 1):
            kls = []
            for x_batch, _ in tqdm.tqdm(train_loader, desc="Training", leave=True, disable=disable):
                opt.zero_grad()
                mean, std = self.enc(x_batch)
                prior = models.make_prior(mean, latent_dim=self.ld_ode, device=self.device)
                kl = train_functions.kl_divergence(prior, Normal(mean, std)).sum(-1).mean() / self.len_tr
                kl.backward()
                opt.step()
                kls.append(kl.detach().cpu().numpy())
            if disable:
                print(f"{'Epoch':<8}: {epoch:.3f}, {'KL_z':<8}: {np.mean(kls):.3f}")

    def train(self, train_loader, t, epochs, losses, eval_pts, grad_lim=300, n_samples=32, checkpoint=False,
              track_norms=False, norm_file="grad_norms.txt", disable=False, warmup=False, validate=None):
        self.best_loss = 1e9
        self.skip_count = 0
        start = len(self._history.epoch_history)
        sched = LambdaLR(self.optimizer, lr_lambda=warm_up_lr) if warmup else None
        for e in range(epochs):
            epoch = start + e
            self.norms = []
            bar = tqdm.tqdm(train_loader, desc="Training " + str(epoch + 1), leave=True, disable=disable)
            for x, y in bar:
                data, names = self.train_step(x, y, t, epoch, losses, eval_pts, grad_lim=grad_lim,
                                              n_samples=n_samples, track_norms=track_norms, norm_file=norm_file)
                self._history.batch(data, names)
                bar.set_postfix(self._history.epoch())
            if sched is not None:
                sched.step()
            self._history.reset()
            if validate is not None:
                y_pred = self(validate["x_test"], validate["t"], n_samples=validate["n_samples"], training=False)
                y_pr, y_te = _scale_forecast(y_pred, validate["y_test"], validate["scaler"])
                mu, sd = y_pr.mean(1), y_pr.std(1)
                nlls = [Metrics.nll(y_te[:, g, :], mu[:, g, :], sd[:, g, :]) for g in range(len(validate["t"]))]
                self._history.epoch_history[-1]["forecast_nll"] = np.mean(nlls[-28:])
                self._history.epoch_history[-1]["all_nll"] = np.mean(nlls)
            if disable:
                print(epoch + 1, end=" ")
                print_rounded_dict(self._history.epoch_history[-1], decimals=3)
            with open(norm_file, "a") as f:
                f.write(",".join(map(str, self.norms)) + "\n")
            if checkpoint:
                self.checkpoint()

    def _files(self, prefix, tag=""):
        return [f"{prefix}{tag}{part}.pth" for part in ("enc", "ode", "dec")]

    def checkpoint(self):
        if self.chkpt_prefix is None:
            self.chkpt_prefix = self.file_prefix
        if self._history.epoch_history[-1]["loss"] < self.best_loss:
            self.best_loss = self._history.epoch_history[-1]["loss"]
            for m, f in zip((self.enc, self.ode, self.dec), self._files(self.chkpt_prefix, "chkpt_")):
                torch.save(m.state_dict(), f)

    def save(self):
        for m, f in zip((self.enc, self.ode, self.dec), self._files(self.file_prefix)):
            torch.save(m.state_dict(), f)

    def load(self, checkpoint=False, file_prefix=None):
        if self.chkpt_prefix is None:
            self.chkpt_prefix = self.file_prefix
        files = self._files(self.chkpt_prefix, "chkpt_") if checkpoint else self._files(file_prefix or self.file_prefix)
        for m, f in zip((self.enc, self.ode, self.dec), files):
            m.load_state_dict(torch.load(f, weights_only=True), strict=False)
