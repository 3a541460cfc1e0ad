#!/usr/bin/env python3
"""Benchmark of the hot path: fused RK4 solve of the SIR-UDE + VJP through it.

Metric (BASELINE.json): UDE trajectories x steps / s (fwd+bwd), batch = states x
seasons, whole job over all ranks.  One "step" = one forward solve of the
trajectory batch (all RK4 steps, all 4 stages, outputs at every grid point) plus
the VJP w.r.t. y0 and every RHS weight given d latent and d (posterior mean,
std, |Fa|), plus -- with N > 1 ranks -- the side-statistic all-reduce and the
parameter-gradient all-reduce (RCCL).

Workload (per rank, weak scaling): BASELINE configs[1] "50 states x 10 seasons
x 28-day windows": the reference's state model (run_ode.py:41-49, R = 49 regions
flattened jointly into the FaFp MLPs, latent_dim 8, net [64,64,32], aug
[64,64]) on 64 MC samples x 10 seasons x 32 windows = 20,480 trajectories, 8
weekly RK4 steps (dt = 1 week, the longest training curriculum of run_ode.py
:147-152, gamma = 56).  Synthetic inputs, default nn.Linear init, seed 0.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "forecasting-influenza-using-universal-differential-equations_amd"

METRIC = "UDE trajectories×steps/sec (fwd+bwd), batch=states×seasons, at 1/2/4/8 MI355X"
PEAK_FP32_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector == FP32 MFMA dense peak
PEAK_HBM_GBS = 8000.0

_US = dict(kind="FaFp", R=1, L=8, net=[64, 64, 32], aug=[64, 64])
_STATE = dict(kind="FaFp", R=49, L=8, net=[64, 64, 32], aug=[64, 64])
WORKLOADS = {
    "state49": dict(_STATE, n_traj=64 * 10 * 32, t=("arange", 9, 1.0),
                    desc="state model R=49 (joint), 64 MC samples x 10 seasons x 32 windows, 8 weekly RK4 steps"),
    "state49_n2048": dict(_STATE, n_traj=2048, t=("arange", 9, 1.0),
                          desc="state model R=49 (joint), the reference's own batch: 64 MC samples x 32 windows, "
                               "8 weekly RK4 steps (SURVEY 8d M2 variant)"),
    "state49_n2560": dict(_STATE, n_traj=2560, t=("arange", 9, 1.0),
                          desc="state model R=49 (joint), 2,560 trajectories = the per-GPU shard of the 20,480 "
                               "batch strong-scaled over 8 MI355X (BASELINE configs[4]), 8 weekly RK4 steps"),
    "m3_states_r1": dict(_US, n_traj=64 * 50 * 10 * 32, t=("arange", 9, 1.0),
                         desc="50 independent states as R=1 US-architecture models: 64 samples x 50 states x "
                              "10 seasons x 32 windows = 1,024,000 trajectories, 8 weekly RK4 steps (SURVEY 8d M3)"),
    "us_northstar": dict(_US, n_traj=4096, t=("arange", 366, 7.0),
                         desc="US model R=1, 4096 trajectories x 365 daily RK4 steps (north-star M1)"),
    "us_fp32": dict(kind="Fp", R=1, L=8, net=[32, 32], aug=None, n_traj=4096, t=("arange", 366, 7.0),
                    desc="US Fp [32, 32] ('32-hidden' north-star model), R=1, 4096 trajectories x 365 daily "
                         "RK4 steps (north-star M1)"),
    "bayes_us": dict(_US, kind="Bayes_FaFp", n_traj=4096, t=("arange", 366, 7.0),
                     desc="Bayesian US model (models_bayes.py Bayes_FaFp, fresh weight sample per RHS "
                          "evaluation), R=1, 4096 trajectories x 365 daily RK4 steps"),
    "bayes_state49": dict(_STATE, kind="Bayes_FaFp", n_traj=64 * 10 * 32, t=("arange", 9, 1.0),
                          desc="Bayesian state model (models_bayes.py Bayes_FaFp, run_ode.py 'UONNb'), R=49, "
                               "64 MC samples x 10 seasons x 32 windows, 8 weekly RK4 steps"),
    "state49_fp": dict(kind="Fp", R=49, L=8, net=[64, 64, 32], aug=None, n_traj=64 * 10 * 32, t=("arange", 9, 1.0),
                       desc="state model R=49, rate net only (run_ode.py 'Fp' variant), 20,480 trajectories, "
                            "8 weekly RK4 steps (development line: --workload)"),
    "state49_fa": dict(kind="Fa", R=49, L=8, net=None, aug=[64, 64], n_traj=64 * 10 * 32, t=("arange", 9, 1.0),
                       desc="state model R=49, augmentation net only (run_ode.py 'Fa' variant), 20,480 "
                            "trajectories, 8 weekly RK4 steps (development line: --workload)"),
    "tiny": dict(_US, n_traj=64, t=("arange", 5, 1.0),
                 desc="plumbing rehearsal only (CPU / gloo): US model, 64 trajectories, 4 weekly steps"),
}


def macs_per_eval(w):
    """Multiply-adds of one RHS evaluation with the full R*L layer-0 input."""
    R, L = w["R"], w["L"]
    tot = 0
    for sizes, out in ((w["net"], 2 * R), (w["aug"], 3 * R)):
        if sizes is None:
            continue
        dims = [R * L] + list(sizes) + [out]
        tot += sum(a * b for a, b in zip(dims[:-1], dims[1:]))
    return tot


def executed_macs_per_eval(w):
    """Multiply-adds the MFMA tiles actually issue per evaluation: every layer padded to 16 rows /
    16 input columns, layer 0 over the 3R dynamic features only for the deterministic kernels (the
    static latent dims' contribution is hoisted once per tile, ude_kernels.h static_hoist), over
    [dynamic | static] for the Bayesian ones."""
    R, L = w["R"], w["L"]
    p16 = lambda x: (x + 15) // 16 * 16
    in0 = p16(3 * R) + (p16(R * (L - 3)) if w["kind"].startswith("Bayes_") else 0)
    tot = 0
    for sizes, out in ((w["net"], 2 * R), (w["aug"], 3 * R)):
        if sizes is None:
            continue
        dims = [in0] + [p16(x) for x in sizes] + [p16(out)]
        tot += sum(a * b for a, b in zip(dims[:-1], dims[1:]))
    return tot


def make_t(spec):
    kind, n, div = spec
    return torch.arange(n, dtype=torch.float32) / div


def synthetic_y0(gen, N, R, L):
    S = torch.rand(N, R, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, R, generator=gen) * 0.05
    rest = torch.randn(N, R, L - 3, generator=gen)
    return torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], rest], -1) + 1e-5


def build(pkg, w, device, seed):
    torch.manual_seed(0)                         # identical weights on every rank
    if w["kind"].startswith("Bayes_"):
        from ude_amd import bayes
        cls = getattr(bayes, w["kind"])
    else:
        cls = getattr(pkg, w["kind"])
    kw = {}
    if w["net"] is not None:
        kw["net_sizes"] = w["net"]
    if w["aug"] is not None:
        kw["aug_net_sizes"] = w["aug"]
    mod = cls(w["R"], latent_dim=w["L"], **kw).to(device)
    gen = torch.Generator().manual_seed(seed)
    y0 = synthetic_y0(gen, w["n_traj"], w["R"], w["L"]).to(device).requires_grad_(True)
    t = make_t(w["t"])
    dlat = torch.randn((len(t),) + tuple(y0.shape), generator=gen).to(device)
    return mod, y0, t, dlat


_COTS = {}


def _cot(vals, device):
    """Fixed loss cotangents (created once: they stand for upstream gradients)."""
    key = (tuple(vals) if isinstance(vals, (list, tuple)) else vals, str(device))
    if key not in _COTS:
        _COTS[key] = torch.tensor(vals, device=device)
    return _COTS[key]


def one_step(pkg, udist, mod, y0, t, dlat, world):
    mod.clear_tracking()
    mod.zero_grad(set_to_none=True)
    y0.grad = None
    latent = pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=t[1] - t[0]))
    if world > 1:
        udist.sync_side_stats(mod)
    outs, cots = [latent], [dlat]
    if mod.ode_type in ("Fp", "FaFp"):
        post = mod.posterior()
        outs += [post.loc, post.scale]
        cots += [_cot([0.3, -0.2], y0.device), _cot([0.5, 0.1], y0.device)]
    if mod.ode_type in ("Fa", "FaFp"):
        outs.append(torch.norm(torch.stack(mod.tracker)))
        cots.append(_cot(0.1, y0.device))
    if world > 1 and getattr(mod, "_ude_reducer", None) is None:
        # the gradient all-reduce issued from autograd hooks as soon as the solve's backward has
        # written the gradients, on a side stream (ude_amd.distributed.GradReducer)
        mod._ude_reducer = udist.GradReducer(mod.parameters())
    if world > 1:
        mod._ude_reducer.arm()
    torch.autograd.backward(outs, cots)
    if world > 1:
        mod._ude_reducer.finish()


def time_steps(pkg, udist, mod, y0, t, dlat, world, steps, warmup, barrier, dev):
    from ude_amd import fused
    for _ in range(warmup):
        one_step(pkg, udist, mod, y0, t, dlat, world)
    _sync(dev)
    fused.EVENTS = [] if dev.type == "cuda" else None
    barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        one_step(pkg, udist, mod, y0, t, dlat, world)
    barrier()
    _sync(dev)
    el = time.perf_counter() - t0
    evs = fused.EVENTS or []
    fused.EVENTS = None
    k_ms = {"fwd": [], "bwd": []}
    for kind, e0, e1 in evs:
        k_ms[kind].append(e0.elapsed_time(e1))
    return el, {k: (sum(v) / len(v) if v else None) for k, v in k_ms.items()}


# host threads of the CPU baseline: the GPU box's CPU share per GPU (OMP_NUM_THREADS there)
CPU_THREADS = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)


def cpu_baseline(w, mod_gpu, budget_s=10.0, threads=1):
    """The oracle (PyTorch CPU restatement, fp32, autograd) on a bounded sample."""
    from oracle.ude_oracle import OracleRHS, solve_and_grad
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)              # 1 = the reference's own setting (run_ode.py:28)
    rhs = OracleRHS.from_module(_cpu_copy(mod_gpu))
    n = 1024 if w["R"] > 10 else 4096
    steps_cap = 8 if w["R"] > 10 else 40
    tt = make_t(w["t"])[: steps_cap + 1]
    gen = torch.Generator().manual_seed(123)
    y0 = synthetic_y0(gen, n, w["R"], w["L"])
    dl = torch.randn((len(tt),) + tuple(y0.shape), generator=gen)
    dm, ds = torch.tensor([0.3, -0.2]), torch.tensor([0.5, 0.1])
    best = None
    t_start = time.perf_counter()
    reps = 0
    while reps < 5 and (reps < 2 or time.perf_counter() - t_start < budget_s):
        a = time.perf_counter()
        solve_and_grad(rhs, y0, tt, tt[1] - tt[0], dl, dm, ds, 0.1)
        d = time.perf_counter() - a
        best = d if best is None else min(best, d)
        reps += 1
    torch.set_num_threads(prev)
    units = n * (len(tt) - 1)
    return {"value": units / best, "unit": "traj*steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ude_oracle.py (PyTorch CPU fp32 + autograd, torch.set_num_threads({threads}); "
                      f"the reference runs 1 thread, run_ode.py:28) on {n} trajectories x {len(tt) - 1} steps of "
                      f"the same model, fwd+bwd incl. posterior/|Fa| terms, best of {reps}",
            "host_cpus_visible": os.cpu_count()}


def dopri5_line(pkg, w, dev, reps=3):
    """BASELINE configs[2] forward: the same batch solved by the fused adaptive dopri5
    (torchdiffeq defaults rtol 1e-7, atol 1e-9; evaluation path, no autograd)."""
    mod, y0, t, _ = build(pkg, w, dev, seed=77)
    y0 = y0.detach()
    td = t.to(dev)
    with torch.no_grad():
        mod.clear_tracking()
        pkg.odeint(mod, y0, td, method="dopri5")                 # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            mod.clear_tracking()
            pkg.odeint(mod, y0, td, method="dopri5")
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / reps
    info = mod.last_solve_info
    evals = info["n_evals"] * w["n_traj"]
    return {"workload": "state49 batch, method='dopri5' (rtol 1e-7, atol 1e-9), forward only",
            "ms_per_solve": el * 1e3, "n_steps": info["n_steps"], "n_accepted": info["n_accepted"],
            "n_evals": info["n_evals"], "rhs_evals_per_s": evals / el,
            "traj_accepted_steps_per_s": info["n_accepted"] * w["n_traj"] / el}


def loss_head_line(pkg, w, dev, reps=20):
    """the training loss head over the state49 solve's latent (T = 9 outputs,
    64 MC samples x 320 windows, R = 49, L = 8): Decoder(latent[..., :3]) + nll_loss +
    latent_init_loss, forward and backward, fused (csrc/ude_loss.h) vs the reference's own
    torch ops on the same GPU.  HBM roofline: the fused pass reads the latent once (forward)
    and reads it + writes d latent once (backward)."""
    import lib.models as models
    import lib.train_functions as tf
    from ude_amd import fused, loss_head
    T, S, B, R, L = 9, 64, w["n_traj"] // 64, w["R"], w["L"]
    gen = torch.Generator(device=dev).manual_seed(5)
    lat = torch.rand(T, S * B, R, L, device=dev, generator=gen).requires_grad_(True)
    dec = models.Decoder(R, L, 1).to(dev)
    y = torch.rand(B, T, R, device=dev, generator=gen)
    ode, _, _, _ = build(pkg, w, dev, seed=3)
    lin = dec.decoder[-1]

    def fused_step():
        nll, reg = loss_head.fused_loss_head(ode, lat, lin, y, S, B)
        (nll + 0.1 * reg).backward()

    def ref_step():
        yp = dec(lat[..., :3]).reshape((-1, S, B, R)).permute(2, 1, 0, 3)
        (tf.nll_loss(yp, y) + 0.1 * tf.latent_init_loss(lat[..., :3])).backward()

    def run(fn, ev):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        fused.EVENTS = [] if ev else None
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / reps
        evs, fused.EVENTS = fused.EVENTS, None
        k = {}
        for kind, e0, e1 in evs or []:
            k.setdefault(kind, []).append(e0.elapsed_time(e1))
        return el, {kk: sum(v) / len(v) for kk, v in k.items()}

    el_f, k = run(fused_step, True)
    el_r, _ = run(ref_step, False)
    lat_bytes = lat.numel() * 4
    fwd_gbs = lat_bytes / (k["loss_fwd"] * 1e-3) / 1e9
    bwd_gbs = 2 * lat_bytes / (k["loss_bwd"] * 1e-3) / 1e9
    return {"workload": f"state49 latent (T={T}, S={S}, B={B}, R={R}, L={L}) -> Decoder + nll_loss + "
                        "latent_init_loss, fwd+bwd",
            "fused_ms_per_step": el_f * 1e3, "reference_torch_gpu_ms_per_step": el_r * 1e3,
            "speedup_vs_reference_ops": el_r / el_f,
            "fwd_kernel_ms": k["loss_fwd"], "bwd_kernel_ms": k["loss_bwd"],
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": PEAK_HBM_GBS,
                         "fwd_achieved": fwd_gbs, "fwd_frac": fwd_gbs / PEAK_HBM_GBS,
                         "bwd_achieved": bwd_gbs, "bwd_frac": bwd_gbs / PEAK_HBM_GBS,
                         "algorithmic_bytes": {"fwd": lat_bytes, "bwd": 2 * lat_bytes}}}


def adjoint_line(pkg, w, dev, T=2, rtol=1e-5, atol=1e-7, seminorm=True, reps=2):
    """BASELINE configs[2] forward + adjoint backward on the state49 batch: odeint_adjoint
    (torchdiffeq semantics) -- forward = the fused dopri5 solve, backward = the augmented
    dopri5 solve whose every evaluation is the gfx950 evaluation + VJP kernels."""
    from torchdiffeq import odeint_adjoint
    mod, y0, t, _ = build(pkg, w, dev, seed=78)
    td = t[:T].to(dev)
    dl = torch.randn((T,) + tuple(y0.shape), device=dev, generator=torch.Generator(device=dev).manual_seed(2))
    y0 = y0.detach().requires_grad_(True)

    def step():
        mod.clear_tracking()
        mod.zero_grad(set_to_none=True)
        y0.grad = None
        lat = odeint_adjoint(mod, y0, td, rtol=rtol, atol=atol,
                             adjoint_options=dict(norm="seminorm") if seminorm else None)
        info = dict(mod.last_solve_info)
        (lat * dl).sum().backward()
        info.update(mod.last_adjoint_info)
        return info

    step()                              # warm-up: evaluation plans, kernel attributes, allocator
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        info = step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    return {"workload": f"state49 batch ({w['n_traj']} trajectories, R=49), t = {T - 1} weekly interval(s), "
                        f"odeint_adjoint dopri5 rtol {rtol:g} atol {atol:g}"
                        f"{' adjoint_options norm=seminorm' if seminorm else ''}, forward + adjoint backward",
            "ms_per_step": el * 1e3, "forward_steps": info["n_steps"], "forward_evals": info["n_evals"],
            "adjoint_evals": info["augmented_evals"],
            "ms_per_adjoint_eval": el * 1e3 / max(info["augmented_evals"], 1),
            "rhs_evals_per_s_incl_vjp": (info["n_evals"] + info["augmented_evals"]) * w["n_traj"] / el}


def bayes_large_line(pkg, dev, steps=3):
    """SURVEY 8f row 1 at the state model's size: Bayes_FaFp R=49 (run_ode.py 'UONNb'), 20,480
    trajectories x 8 weekly RK4 steps, fwd+bwd; every RHS evaluation draws its own weight sample
    (models_bayes.py:43-48).  Whole-solve kernels (Model::GST): the training forward stores each
    stage's layer inputs, the backward the layer-output gradients, and ude_gst_dw_kernel forms every
    evaluation's weight gradient as one GEMM over the batch, eps-weighted by a fixed-order reduce."""
    w = dict(WORKLOADS["state49"], kind="Bayes_FaFp")
    mod, y0, t, dlat = build(pkg, w, dev, seed=21)
    el, k = time_steps(pkg, None, mod, y0, t, dlat, 1, steps, 1, lambda: None, dev)
    v = w["n_traj"] * (len(t) - 1) * steps / el
    return {"workload": "Bayes_FaFp R=49, 20480 trajectories x 8 weekly RK4 steps (whole-solve GST kernels)",
            "traj_steps_per_s": v, "ms_per_step": el / steps * 1e3}


def train_head_line(pkg, w, dev, reps=10):
    """one training step of the state49 workload (64 MC samples x 320 windows,
    9 weekly outputs) through the loss terms that read the latent -- y_pred = Decoder(latent[..., :3]),
    nll_loss, 0.1 latent_init_loss -- plus the posterior / |Fa| terms, backward into the solve:
    (a) the decoder epilogue (ude_rk4_forward_dec: y_hat and reg from the forward kernel, no latent
    written; nll kernels; decoder backward from the checkpoint store), the path lib/VAE.py takes;
    (b) the solve writing the latent + the fused loss head over it (the r02 path)."""
    import lib.models as models
    from ude_amd import decoder_head, fused, loss_head
    mod, y0, t, _ = build(pkg, w, dev, seed=31)
    S, B, R = 64, w["n_traj"] // 64, w["R"]
    dec = models.Decoder(R, w["L"], 1).to(dev)
    y = torch.rand(B, len(t), R, device=dev, generator=torch.Generator(device=dev).manual_seed(4))
    lin = dec.decoder[-1]
    h = t[1] - t[0]

    def stats_terms():
        post = mod.posterior()
        return post.loc.sum() + post.scale.sum() + 0.1 * torch.norm(torch.stack(mod.tracker))

    def step_epilogue():
        mod.clear_tracking()
        mod.zero_grad(set_to_none=True)
        y0.grad = None
        yhat, reg, lazy, _ = decoder_head.solve_decode(mod, y0, t, h, lin)
        nll, _ = decoder_head.nll_head(mod, yhat, y, S, B)
        (nll + 0.1 * reg + stats_terms()).backward()

    def step_latent():
        mod.clear_tracking()
        mod.zero_grad(set_to_none=True)
        y0.grad = None
        lat = pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=h))
        nll, reg = loss_head.fused_loss_head(mod, lat, lin, y, S, B)
        (nll + 0.1 * reg + stats_terms()).backward()

    out = {}
    for name, fn in (("decoder_epilogue", step_epilogue), ("latent_loss_head", step_latent)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        fused.EVENTS = []
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        out["ms_per_step_" + name] = (time.perf_counter() - t0) / reps * 1e3
        k = {}
        for kind, e0, e1 in fused.EVENTS:
            k.setdefault(kind, []).append(e0.elapsed_time(e1))
        fused.EVENTS = None
        out["kernel_ms_" + name] = {kk: sum(v) / len(v) for kk, v in k.items()}
    n = w["n_traj"] * len(t) * R
    return dict(workload="state49 training step: fused RK4 solve + decoder / nll_loss / latent_init_loss + "
                         "posterior / |Fa| terms, fwd+bwd", **out,
                latent_bytes_not_written=n * w["L"] * 4, yhat_bytes=n * 4)


def _cpu_copy(mod):
    import copy
    mod.clear_tracking()
    return copy.deepcopy(mod).cpu()


PMC_SOURCE = {}


def read_pmc(name):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary (or None).  rocprofv3 cannot
    collect counters inside this process, so the value comes from the committed profile; the
    profile's file and the commit it was measured at go into roofline.traffic_source."""
    p = os.path.join(REPO, "profiles", "pmc_" + name + ".json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        PMC_SOURCE[name] = {"file": os.path.relpath(p, REPO), "measured_at_commit": d.get("commit"),
                            "kernel_avg_ms": d.get("kernel_avg_ms")}
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


def read_roofline_rocprof(name):
    """The committed recomputation of the line's roofline from a rocprofv3 kernel trace of the same
    command over the same timed calls (tools/roofline_trace.py), or None."""
    p = os.path.join(REPO, "profiles", "roofline_rocprof_" + name + ".json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        return {"file": os.path.relpath(p, REPO), "measured_at_commit": d["source"].get("commit"),
                "rocprof_bwd_call_ms": d["rocprof_bwd_call_ms"], "rocprof_bwd_kernel_ms": d["rocprof_bwd_kernel_ms"],
                "rocprof_frac": d["rocprof_frac"], "timed_calls": d["timed_calls"]}
    except Exception:
        return None


def _launch_workers(n):
    """`bench.py --gpus N` run without a launcher: start N ranks under torch.distributed.run
    as a child process (before this process touches the GPU) and exit with its code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, UDE_BENCH_LAUNCHED="1")
    return subprocess.call(cmd, env=env)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def measure(pkg, udist, w, n_traj, dev, rank, world, steps, warmup, barrier):
    """Time `steps` fwd+bwd steps of workload w with n_traj trajectories on this rank;
    returns (max-over-ranks seconds, HIP-event kernel averages)."""
    import torch.distributed as dist
    w = dict(w, n_traj=n_traj)
    mod, y0, t, dlat = build(pkg, w, dev, seed=1000 + rank)
    el, kms = time_steps(pkg, udist, mod, y0, t, dlat, world, steps, warmup, barrier, dev)
    if world > 1:
        x = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x)
    return el, kms, mod, len(t) - 1


def time_steps_graphed(pkg, udist, mod, y0, t, dlat, steps, warmup, dev):
    """The same step replayed as a HIP graph (ude_amd/graphs.py GraphedStep: the pack, the fused
    forward, the backward and its tail, the gradient accumulation -- one host call per step)."""
    from ude_amd.graphs import GraphedStep
    gs = GraphedStep(lambda: one_step(pkg, udist, mod, y0, t, dlat, 1), warmup=max(warmup, 1))
    for _ in range(max(warmup, 1)):
        gs.replay()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        gs.replay()
    _sync(dev)
    return time.perf_counter() - t0


def extra_line(pkg, udist, name, dev, barrier, steps=3, graphed=False):
    """graphed: ms_per_step from HIP-graph replays of the step (the small-batch lines, host-bound when
    eager); the eager step's time and its HIP-event kernel times are reported beside it."""
    w = WORKLOADS[name]
    m, y, t, d = build(pkg, w, dev, seed=7)
    el, k = time_steps(pkg, udist, m, y, t, d, 1, steps, 1, barrier, dev)
    el_eager = el
    if graphed:
        el = time_steps_graphed(pkg, udist, m, y, t, d, steps, 3, dev)
    n_rk = len(t) - 1
    v = w["n_traj"] * n_rk * steps / el
    macs = macs_per_eval(w)
    out = {"workload": name, "description": w["desc"], "traj_steps_per_s": v, "rhs_evals_per_s": 4 * v,
           "ms_per_step": el / steps * 1e3, "fwd_ms": k["fwd"], "bwd_ms": k["bwd"]}
    if graphed:
        out["step_mode"] = "HIP graph replay (ude_amd.graphs.GraphedStep)"
        out["ms_per_step_eager"] = el_eager / steps * 1e3
    if k["bwd"] and not w["kind"].startswith("Bayes_"):
        bwd_flop = 4 * 4 * macs * w["n_traj"] * n_rk
        fwd_flop = 4 * 2 * macs * w["n_traj"] * n_rk
        out["bwd_tflops"] = bwd_flop / (k["bwd"] * 1e-3) / 1e12
        out["bwd_frac"] = out["bwd_tflops"] / PEAK_FP32_TFLOPS
        out["fwd_tflops"] = fwd_flop / (k["fwd"] * 1e-3) / 1e12
        out["fwd_frac"] = out["fwd_tflops"] / PEAK_FP32_TFLOPS
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="state49", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="weak: every rank solves the workload's batch; strong: the batch is split over ranks")
    ap.add_argument("--n-traj", type=int, default=None,
                    help="development: override the workload's trajectory count (not a benchmark line)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--lines", default=None, help="comma-separated subset of the extra lines (development)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) for runs; gloo only to rehearse N>1")
    ap.add_argument("--rehearse-cpu", action="store_true",
                    help="plumbing rehearsal on the host (gloo, eager solver): checks ranks / batch accounting")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(_launch_workers(args.gpus))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report a mislabelled number",
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    if args.rehearse_cpu:
        dev = torch.device("cpu")
        backend = "gloo"
    else:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local % max(ndev, 1))
        torch.cuda.set_device(dev)
        backend = args.dist_backend
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()                 # n_gpus comes from the process group
        rank = dist.get_rank()
        barrier = lambda: dist.barrier()
    else:
        barrier = lambda: None

    pkg = importlib.import_module(PKG)
    from ude_amd import distributed as udist

    w = WORKLOADS[args.workload]
    if args.n_traj:
        w = dict(w, n_traj=args.n_traj, desc=w["desc"] + f" [n_traj overridden: {args.n_traj}]")
    per_rank = w["n_traj"] if args.scaling == "weak" else w["n_traj"] // world
    if args.scaling == "strong" and per_rank * world != w["n_traj"]:
        raise SystemExit(f"strong scaling: {w['n_traj']} trajectories do not split over {world} ranks")
    el, kms, mod, n_steps_rk = measure(pkg, udist, w, per_rank, dev, rank, world, args.steps, args.warmup, barrier)
    units = world * per_rank * n_steps_rk * args.steps
    value = units / el
    macs = macs_per_eval(w)
    flop_unit = 4 * 6 * macs                                  # fwd + dX + dW per traj*step
    bwd_flop_launch = 4 * 4 * macs * per_rank * n_steps_rk    # dX + dW only (recompute not counted)
    fwd_flop_launch = 4 * 2 * macs * per_rank * n_steps_rk

    # strong-scaling companion (N > 1, weak headline): the same global batch split over the ranks
    strong = None
    if world > 1 and args.scaling == "weak" and not args.no_extra and w["n_traj"] % world == 0:
        el_s, kms_s, _, _ = measure(pkg, udist, w, w["n_traj"] // world, dev, rank, world, args.steps,
                                    args.warmup, barrier)
        strong = {"scaling": "strong", "global_batch": w["n_traj"], "traj_per_gpu": w["n_traj"] // world,
                  "value": w["n_traj"] * n_steps_rk * args.steps / el_s, "unit": "traj*steps/s",
                  "ms_per_step": el_s / args.steps * 1e3, "bwd_ms": kms_s["bwd"]}

    res = None
    if rank == 0:
        achieved = bwd_flop_launch / (kms["bwd"] * 1e-3) / 1e12 if kms["bwd"] else None
        pmc = read_pmc(args.workload + "_bwd")
        res = {
            "metric": METRIC, "value": value, "unit": "traj*steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded y0 per SURVEY 8d, default nn.Linear init, N(0,1) d latent)",
            "config": {"workload": args.workload, "description": w["desc"], "model": w["kind"],
                       "n_regions": w["R"], "latent_dim": w["L"], "net_sizes": w["net"],
                       "aug_net_sizes": w["aug"], "traj_per_gpu": per_rank, "global_batch": world * per_rank,
                       "rk4_steps": n_steps_rk, "parallelism": f"dp{world}",
                       "device": "cpu-rehearsal" if args.rehearse_cpu else "MI355X"},
            # avg_launch_ms: HIP events on the launch stream around one ude_rk4_backward_ex call = the
            # ude_bwd_kernel launch and its ude_bwd_tail_kernel (rocprof lists the two separately)
            "roofline": {"kernel": "ude_bwd_kernel + ude_bwd_tail_kernel", "bound": "mfma",
                         "achieved": achieved, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": (achieved / PEAK_FP32_TFLOPS) if achieved else None,
                         "traffic": pmc, "traffic_source": PMC_SOURCE.get(args.workload + "_bwd"),
                         "avg_launch_ms": kms["bwd"],
                         # the same span from a committed rocprofv3 trace of this command (timed calls only)
                         "rocprof": read_roofline_rocprof(args.workload),
                         "algorithmic_flop_per_launch": bwd_flop_launch,
                         # the MFMA work the kernel issues (padded tiles, hoisted static features) per
                         # algorithmic MAC, and the MFMA pipe's busy fraction that implies
                         "executed_per_algorithmic_mac": executed_macs_per_eval(w) / macs_per_eval(w),
                         "executed_mac_frac": ((achieved / PEAK_FP32_TFLOPS) * executed_macs_per_eval(w)
                                               / macs_per_eval(w)) if achieved else None},
            "kernels": {"fwd_ms": kms["fwd"], "bwd_ms": kms["bwd"],
                        "fwd_tflops": fwd_flop_launch / (kms["fwd"] * 1e-3) / 1e12 if kms["fwd"] else None,
                        "step_tflops_algorithmic": value * flop_unit / 1e12,
                        "rhs_evals_per_s": 4 * value},
        }
        if strong is not None:
            res["strong_scaling"] = strong
    extra = rank == 0 and world == 1 and not args.no_extra and args.workload == "state49" and not args.rehearse_cpu
    if extra:
        lines = [("north_star_M1", lambda: dict(extra_line(pkg, udist, "us_northstar", dev, barrier),
                                                target_rhs_evals_per_s=1e7)),
                 ("north_star_M1_fp32", lambda: extra_line(pkg, udist, "us_fp32", dev, barrier)),
                 ("M2_state49_n2048", lambda: extra_line(pkg, udist, "state49_n2048", dev, barrier, steps=20,
                                                         graphed=True)),
                 ("state49_n2560_strong8_shard", lambda: extra_line(pkg, udist, "state49_n2560", dev, barrier,
                                                                    steps=20, graphed=True)),
                 ("M3_states_r1", lambda: extra_line(pkg, udist, "m3_states_r1", dev, barrier)),
                 ("bayes_M1", lambda: extra_line(pkg, udist, "bayes_us", dev, barrier)),
                 ("dopri5_state49", lambda: dopri5_line(pkg, w, dev)),
                 ("dopri5_adjoint_state49", lambda: adjoint_line(pkg, w, dev)),
                 ("bayes_state49", lambda: bayes_large_line(pkg, dev)),
                 ("loss_head_state49", lambda: loss_head_line(pkg, w, dev)),
                 ("train_step_head_state49", lambda: train_head_line(pkg, w, dev))]
        if args.lines:
            keep = set(args.lines.split(","))
            lines = [(n, f) for n, f in lines if n in keep]
        for name, fn in lines:
            t0 = time.perf_counter()
            res[name] = fn()
            torch.cuda.empty_cache()
            print(f"[bench] {name}: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.rehearse_cpu:
        print("[bench] cpu baselines", file=sys.stderr, flush=True)
        res["cpu_baseline"] = cpu_baseline(w, mod, threads=CPU_THREADS)
        res["cpu_baseline_1thread"] = cpu_baseline(w, mod, threads=1)
        # BASELINE.md section 3 / SURVEY 8d: the north-star M1 models too (FaFp and Fp [32, 32], R = 1)
        for name, wl in (("cpu_baseline_M1", "us_northstar"), ("cpu_baseline_M1_fp32", "us_fp32")):
            wm = WORKLOADS[wl]
            m_cpu, _, _, _ = build(pkg, wm, torch.device("cpu"), seed=1000)
            res[name] = {"workload": wl, "threads_16": cpu_baseline(wm, m_cpu, threads=CPU_THREADS),
                         "threads_1": cpu_baseline(wm, m_cpu, threads=1)}
        # (the box's usable host share is OMP_NUM_THREADS = 16 per GPU: no line above it -- VERDICT r4 item 8)
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
