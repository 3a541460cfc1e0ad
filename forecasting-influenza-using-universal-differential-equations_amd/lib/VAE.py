"""Drop-in for lib/VAE.py: the VAE whose forward calls the hot path.

``VAE.__call__`` (reference :118-140) draws eps, encodes, builds
``y0 = reparam(...) + 1e-5`` and calls ``odeint(ode, y0, t, method='rk4',
options=dict(step_size=t[1]-t[0]))`` -- here served by the fused gfx950 kernel
when the model lives on a HIP device -- then decodes ``latent[..., :3]``.
``calc_loss`` (:142-198) reads the solver's side outputs exactly as the
reference does (``ode.posterior()``, ``torch.norm(torch.stack(ode.tracker))``,
``self.latent``) and ``train_step`` (:200-223) back-propagates through the solve.
Under ``torch.distributed`` (one process per GPU, ``VAE.enable_data_parallel()`` or a process
group of more than one rank at ``setup_training``) ``train_step`` runs data-parallel (BASELINE
configs[4]): each rank takes a contiguous shard of the batch's windows, the
posterior / |Fa| side statistics are made global before ``calc_loss``
(``ude_amd.distributed.sync_side_stats``), every loss term is weighted by its share of the
global batch, and one bucketed all-reduce of the encoder + ODE + decoder gradients precedes
the grad-norm gate, so every rank takes the identical Adam step the single-process run takes.
On a HIP device a training call runs the solve with the decoder epilogue
(ude_amd/decoder_head.py): the forward kernel emits the decoder output
y_hat = Decoder(latent[..., :3]) and latent_init_loss(latent[..., :3]) at every output time and
writes no (T, N, R, L) latent -- ``self.latent`` is rebuilt from the training store only when it
is read -- and calc_loss takes nll_loss of that prediction from the gfx950 nll kernels.  The
Bayesian RHS (models_bayes.py, run_ode.py's ``*b`` models) takes the same epilogue
(``fused.FusedBayesRK4Dec``: each evaluation's weight sample through the decoder forward).  When
the epilogue does not apply (output times between grid points, a non-reference decoder) the latent
is written and the fused loss head (ude_amd/loss_head.py: decoder + nll_loss + latent_init_loss in
one kernel pass each) serves the same terms.
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
from ude_amd import decoder_head
from ude_amd import distributed as udist
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
        self._dp = None            # data-parallel state (enable_data_parallel)
        self._dp_eps = None        # (full window count, lo, hi) while a sharded step draws eps

    # ``latent``: a tensor, or (decoder-epilogue training solve) rebuilt on first read
    @property
    def latent(self):
        v = self.__dict__.get("_latent")
        if isinstance(v, decoder_head.LazyLatent):
            return v.get()
        return v

    @latent.setter
    def latent(self, value):
        self.__dict__["_latent"] = value

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
        if self._dp is None and udist.world_size() > 1:
            self.enable_data_parallel()
        self.optimizer = torch.optim.Adam(self.parameters(), lr=lr)
        self._history = train_functions.history()

    def enable_data_parallel(self, group=None):
        """Data-parallel training steps over the default (or given) process group: rank 0's
        weights are broadcast so every replica starts identical; ``train_step`` then shards
        each batch's windows over the ranks (see the module docstring)."""
        self._dp = {"group": group, "world": udist.world_size(group), "rank": udist.rank(group)}
        udist.broadcast_parameters(self.parameters(), group=group)
        # every rank then draws the same full-batch eps each step (__call__ slices its shard)
        udist.broadcast_rng_state(self.device, group=group)
        return self

    def _shard(self, B):
        """This rank's contiguous window range [lo, hi) of a B-window batch."""
        world, rank = self._dp["world"], self._dp["rank"]
        if B < world:
            # an empty shard would reach the solve with no trajectories while the peers wait in
            # the statistics / gradient all-reduces
            raise ValueError(f"data-parallel train_step: a batch of {B} windows cannot be sharded over "
                             f"{world} ranks (need at least one window per rank)")
        base, rem = divmod(B, world)
        lo = rank * base + min(rank, rem)
        return lo, lo + base + (1 if rank < rem else 0)
    def __call__(self, x, t, n_samples=32, training=False):
        B = x.shape[0]
        # release the previous call's training store (LazyLatent keeps the stage checkpoints and
        # stored activations alive) before this call's solve allocates its own
        self.__dict__["_latent"] = None
        self._pred_src = None
        if self._dp_eps is not None:
            # sharded step: the full batch's eps sliced to this shard.  Every rank's generator
            # holds rank 0's state (enable_data_parallel) and draws the same count per step, so
            # the draw is the same on every rank and equals the single-process step's samples
            b_full, lo, hi = self._dp_eps
            eps = torch.randn(n_samples, b_full, self.n_regions, self.ld_enc, dtype=self.dtype,
                              device=self.device)[:, lo:hi]
        else:
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
            dec = None
            if training and decoder_head.eligible(self.ode, z, decoder_head.decoder_linear(self.dec)):
                dec = decoder_head.solve_decode(self.ode, z, t, step, decoder_head.decoder_linear(self.dec))
            if dec is not None:
                # y_hat (T, N, R) == self.dec(latent[..., :3]) (lib/models.py:45-51), no latent written
                yhat, reg, lazy, _ = dec
                self.latent = lazy
                y_pred = yhat.reshape((-1, n_samples, B, self.n_regions)).permute(2, 1, 0, 3)
                self._pred_src = (y_pred, n_samples, B, yhat, reg)
                return y_pred
            self.latent = odeint(self.ode, z, t, method="rk4", options=dict(step_size=step))
            decoded = self.dec(self.latent[..., :3])
            y_pred = decoded.reshape((-1, n_samples, B, self.n_regions)).permute(2, 1, 0, 3)
        # calc_loss may take nll / reg from the fused loss head when handed this prediction
        self._pred_src = (y_pred, n_samples, B, None, None) if training else None
        return y_pred

    def _fused_head(self, y_pred, y_true, losses):
        """(nll, reg, per-group prediction mean / std) for this model's latest training prediction:
        from the decoder-epilogue solve (reg) and the gfx950 nll kernels, or from the fused loss
        head over the written latent (ude_amd/loss_head.py); None when y_pred is not that
        prediction or the shapes do not fit."""
        src = getattr(self, "_pred_src", None)
        if not (losses.get("nll", True) or losses.get("reg_loss", True)) or src is None or src[0] is not y_pred:
            return None
        if src[3] is not None:
            yhat, reg = src[3], src[4]
            if losses.get("nll", True) and src[1] >= 2:
                nll, musd = decoder_head.nll_head(self.ode, yhat, y_true, src[1], src[2])
            elif losses.get("nll", True):
                return None
            else:
                nll, musd = None, None
            return nll, reg, musd
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
        """The reference's loss composition (:142-198).  In a data-parallel step
        (``self._dp_w``) each term is weighted by this rank's share of the global loss -- batch
        means by the window fraction, sums by 1, terms of the (already global) side statistics and
        of the parameters by 1/world -- and the reported values are the all-reduced global ones."""
        dpw = getattr(self, "_dp_w", None)
        terms = {}
        if losses.get("anneal", True):
            self.tr_step += 1
            self.kl_w = train_functions.KL_annealing(self.tr_step, self.anneal_params)
        if losses.get("mse", True):
            terms["mse"] = torch.mean(torch.square(y_pred - y_true.unsqueeze(1)))
        fused = self._fused_head(y_pred, y_true, losses)
        checks = []
        if fused is not None and losses.get("nll", True):
            # nll_loss builds Normal(y_mean, y_std) only when the nll term is on (ref :160-161)
            checks.append(("nll_loss prediction mean / std", fused[2][..., 0], fused[2][..., 1]))
        if fused is None and losses.get("reg_loss", True) and getattr(self, "_pred_src", None) is not None \
                and self._pred_src[0] is y_pred and self._pred_src[4] is not None:
            fused = (None, self._pred_src[4], None)     # reg of the decoder-epilogue solve (nll eager)
        if losses.get("nll", True):
            terms["nll"] = fused[0] if (fused is not None and fused[0] is not None) \
                else train_functions.nll_loss(y_pred, y_true)
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
        if dpw is not None:
            frac, glob = dpw
            kind = {"mse": frac, "nll": frac, "kl_latent": frac, "reg_loss": 1.0}
            terms = {k: v * kind.get(k, glob) for k, v in terms.items()}
        loss = torch.tensor(0.0, requires_grad=True)
        for v in terms.values():
            loss = loss + v
        shown = {k: (norm if k == "Fa_norm" else v) for k, v in terms.items()}
        if dpw is not None:
            # global values for the history: one all-reduce of the weighted terms (the Fa norm
            # is already global)
            keys = list(terms)
            vec = torch.stack([loss.detach().reshape(()).to(torch.float64)] +
                              [terms[k].detach().reshape(()).to(torch.float64) for k in keys]).to(self.device)
            vec = udist.all_reduce_values(vec, group=self._dp["group"])
            loss_val = vec[0]
            shown = {k: (norm if k == "Fa_norm" else vec[1 + i]) for i, k in enumerate(keys)}
        else:
            loss_val = loss
        names, data = ["loss"], [round(loss_val.cpu().item(), 3)]
        if losses.get("anneal", True):
            names.append("kl_w"); data.append(round(self.kl_w, 3))
        for k, v in shown.items():
            names.append(k)
            data.append(round(v.cpu().item(), 3))
        return loss, data, names

    def train_step(self, x, y, t, epoch, losses, eval_pts, grad_lim=300, n_samples=32, track_norms=False,
                   norm_file="grad_norms.txt"):
        if self._dp is not None and self._dp["world"] > 1:
            B = x.shape[0]
            lo, hi = self._shard(B)
            self._dp_eps = (B, lo, hi)
            try:
                y_pred = self(x[lo:hi], t[eval_pts], n_samples=n_samples, training=True)
            finally:
                self._dp_eps = None
            udist.sync_side_stats(self.ode, group=self._dp["group"])
            self._dp_w = ((hi - lo) / B, 1.0 / self._dp["world"])
            try:
                loss, data, names = self.calc_loss(y_pred, y[lo:hi][:, eval_pts, :], losses=losses)
            finally:
                self._dp_w = None
            if "reducer" not in self._dp:
                # one bucket group per stage, in registration order: autograd produces the decoder's
                # gradients first, then the ODE's (the fused solve's tail hands them over at once),
                # then the encoder's -- the decoder / ODE buckets are in flight while the encoder's
                # backward still runs (a single 4 MB bucket would go out only after the last hook)
                self._dp["reducer"] = udist.GradReducer(
                    average=False, group=self._dp["group"],
                    groups=[list(self.enc.parameters()), list(self.ode.parameters()), list(self.dec.parameters())])
            self._dp["reducer"].arm()
            loss.backward()
            # encoder + ODE + decoder gradients summed over the ranks, each bucket's all-reduce issued
            # during the backward as soon as its gradients exist (ref :205 then sees the global
            # gradient on every rank: same gate, same Adam step)
            self._dp["reducer"].finish()
        else:
            y_pred = self(x, t[eval_pts], n_samples=n_samples, training=True)
            loss, data, names = self.calc_loss(y_pred, y[:, eval_pts, :], losses=losses)
            loss.backward()
        # every parameter must have a gradient (the reference's p.grad.data raises otherwise, :205)
        grad_norm = torch.norm(torch.cat([p.grad.reshape(-1) for p in self.parameters()]), 2).item()
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
                # the reference scores range(len(t)) with the TRAINING grid t (ref lib/VAE.py:278)
                nlls = [Metrics.nll(y_te[:, g, :], mu[:, g, :], sd[:, g, :]) for g in range(len(t))]
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
