"""torch.autograd.Function over the C-ABI: one fused RK4 solve (+ its VJP).

Forward : pack weights -> ude_rk4_forward (latent, stage checkpoints, side stats)
Backward: ude_rk4_backward (dy0, every weight/bias gradient) -> split into the
          parameters' shapes.
PyTorch only provides device memory and the current HIP stream here.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple
import weakref

import torch

from . import _native
from .schedule import Schedule


@dataclass
class Plan:
    lib: "_native.NativeLib"
    desc: "_native.UdeModelDesc"
    prob: "_native.UdeProblem"
    sizes: "_native.UdeSizes"
    sched_dev: torch.Tensor
    n_times: int
    n_eval: int
    param_shapes: List[torch.Size]
    # grid point of every output time when each one is an exact grid hit (decoder epilogue), else None
    out_k: Optional[List[int]] = None
    n_regions: int = 0
    latent_dim: int = 0
    # control words of the *_ex calls, one zeroed buffer per stream (include/ude_rk4.h: zero on entry,
    # left zero by every call; calls sharing one are stream ordered)
    ctl: Dict[int, torch.Tensor] = field(default_factory=dict)
    # packed weights of the last forward and (weak reference, storage, version) of every parameter
    # they were packed from (``packed_weights``)
    pack_key: Optional[tuple] = None
    pack: Optional[torch.Tensor] = None


# Stored-activation budget (bytes) of one training solve: above it the training forward stores only
# the stage inputs and the backward recomputes each stage's layers (UdeProblem.recompute; same
# results bit for bit).  None: half of the device's free memory when the plan is made.
ACT_BUDGET = None


def act_budget(device: torch.device) -> int:
    import os
    env = os.environ.get("UDE_ACT_BUDGET_BYTES")
    if env is not None:
        return int(float(env))
    if ACT_BUDGET is not None:
        return int(ACT_BUDGET)
    free, _ = torch.cuda.mem_get_info(device)
    return free // 2


def make_plan(cfg, schedule: Schedule, n_traj: int, fa_w: float, device: torch.device,
              param_shapes: List[torch.Size]) -> Plan:
    lib = _native.library_for(cfg)
    desc = _native.make_desc(cfg)
    prob = _native.UdeProblem()
    prob.n_traj = int(n_traj)
    prob.n_steps = schedule.n_steps
    prob.n_out = schedule.n_out
    prob.fa_w = float(fa_w)
    prob.recompute = 0
    dev_index = device.index if device.index is not None else torch.cuda.current_device()
    sizes = lib.query(desc, prob, dev_index)
    if sizes.act_bytes > 0 and sizes.act_bytes > act_budget(device):
        prob.recompute = 1                      # memory fallback: recompute each stage's layers
        rsizes = lib.query(desc, prob, dev_index)
        if rsizes.act_bytes < sizes.act_bytes:
            sizes = rsizes
        else:
            # no Recompute view for this model (the Bayesian GST kernels store every stage's
            # layer inputs for the per-evaluation weight-gradient GEMM): say so, keep the store
            import warnings
            prob.recompute = 0
            warnings.warn(f"{cfg}: the training store ({sizes.act_bytes / 2**30:.2f} GiB of activations) "
                          f"exceeds the stored-activation budget ({act_budget(device) / 2**30:.2f} GiB) and "
                          "this model has no recompute path; allocating it anyway", ResourceWarning)
    sched = torch.from_numpy(schedule.to_bytes()).to(device, non_blocking=False)
    n_eval = 4 * schedule.n_steps * n_traj * cfg[1]
    out_k = None
    if schedule.n_steps >= 1 and all(int(m) == 1 for m in schedule.out_mode):
        out_k = [0]
        for n in range(schedule.n_steps):
            out_k += [n + 1] * int(schedule.out_start[n + 1] - schedule.out_start[n])
    return Plan(lib, desc, prob, sizes, sched, schedule.n_times, n_eval, param_shapes, out_k, cfg[1], cfg[2])


# Optional HIP-event instrumentation (bench.py): when a list, every forward /
# backward C-ABI call appends (kind, start_event, end_event) recorded on the
# stream the kernels are launched on.
EVENTS = None


def _ev(dev):
    return torch.cuda.Event(enable_timing=True)


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _ctl(plan: Plan, dev) -> torch.Tensor:
    if _capturing():
        # HIP-graph capture (ude_amd/graphs.py): the graph's own zeroed word (a memset node, re-zeroed
        # every replay), not cached -- it lives in the graph's memory pool
        return torch.zeros(max(int(plan.sizes.ctl_bytes) // 4, 1), dtype=torch.int32, device=dev)
    stream = _stream(dev)
    c = plan.ctl.get(stream)
    if c is None:
        c = plan.ctl[stream] = torch.zeros(max(int(plan.sizes.ctl_bytes) // 4, 1), dtype=torch.int32, device=dev)
    return c


def _stats_out(plan: Plan, dev):
    """Fresh (mean (2), std (2), fa_norm (1)) outputs + fp64 totals (5) of one solve: separate views
    of one buffer, so posterior() and the tracker read them without a split (and their cotangents
    reach the kernel without a concatenation); written by the forward kernel's last workgroup.  The
    kernel skips the statistics of a net the model lacks (mean / std of an Fa-only model, |Fa| of an
    Fp-only one): those outputs are zero-filled, so no uninitialised value reaches autograd (their
    zero cotangent terms, e.g. 2 g |Fa| in ``_StatSums``, stay zero)."""
    kind = int(plan.desc.kind) & 3
    buf = (torch.empty if kind == 3 else torch.zeros)(5, dtype=torch.float32, device=dev)
    mean, std, norm = buf[0:2], buf[2:4], buf[4:5]
    sums = (torch.empty if kind == 3 else torch.zeros)(5, dtype=torch.float64, device=dev)
    st = _native.UdeSideStats(mean.data_ptr(), std.data_ptr(), norm.data_ptr(), sums.data_ptr())
    return (mean, std, norm), sums, st


def _stats_in(stats) -> "_native.UdeSideStats":
    return _native.UdeSideStats(stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(), None)


def _dstats(*grads):
    """(UdeSideStatsGrad, the tensors it points into): absent / placeholder cotangents -> NULL."""
    keep = []
    for g in grads:
        if g is None or _is_placeholder(g):
            keep.append(None)
        else:
            keep.append(g.contiguous().to(torch.float32))
    return _native.UdeSideStatsGrad(*[_ptr(g) for g in keep]), keep


def _pack_key_matches(key, params) -> bool:
    if key is None or len(key) != len(params):
        return False
    for (ref, ptr, ver), p in zip(key, params):
        # the very tensor object (a weak reference: a freed module's parameters never match, even
        # when the allocator hands a new module the same addresses and its version counters run
        # through the same sequence), at the same storage, unmodified since the pack
        if ref() is not p or ptr != p.data_ptr() or ver != p._version:
            return False
    return True


def packed_weights(plan: Plan, params, dev) -> torch.Tensor:
    """The fragment-order pack of a deterministic model's weights, re-packed only when the parameters
    are not the very tensors of this plan's last pack (plans are shared by every module of the same
    configuration), or one's storage or version counter changed since then (an optimizer step, or any
    in-place update through the parameter, bumps it).  Like autograd's own saved-tensor check, an
    in-place write through ``param.data`` is not seen by the version counter: call
    ``invalidate_packs()`` after such an edit."""
    capturing = _capturing()
    if not capturing and plan.pack is not None and _pack_key_matches(plan.pack_key, params):
        return plan.pack
    key = tuple((weakref.ref(p), p.data_ptr(), p._version) for p in params)
    ws = [p.contiguous() for p in params[0::2]]
    bs = [p.contiguous() for p in params[1::2]]
    pack = torch.empty(plan.sizes.pack_bytes // 4, dtype=torch.float32, device=dev)
    plan.lib.pack(plan.desc, [w.data_ptr() for w in ws], [b.data_ptr() for b in bs], pack.data_ptr(), _stream(dev))
    if capturing:
        # a captured step packs on every replay (the parameters may be updated in place between
        # replays, e.g. by an optimizer step); the graph-pool pack is not cached
        return pack
    plan.pack_key, plan.pack = key, pack
    return pack


def invalidate_packs() -> None:
    """Drop every cached weight pack (after editing parameters through ``.data``)."""
    from . import solvers
    for plan in list(solvers._PLAN_CACHE.values()):
        plan.pack_key, plan.pack = None, None


_ZEROS = {}


def zero_grad_like(t: torch.Tensor, device=None) -> torch.Tensor:
    """A stride-0 zero tensor of t's shape (no memory), on t's device (or ``device``)."""
    dev = torch.device(device) if device is not None else t.device
    key = (str(dev), t.dtype)
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros((), dtype=t.dtype, device=dev)
    return z.expand(t.shape)


def _is_placeholder(g: torch.Tensor) -> bool:
    z = _ZEROS.get((str(g.device), g.dtype))
    return z is not None and g.data_ptr() == z.data_ptr() and all(st == 0 for st in g.stride())


def _d_std(d_abs: torch.Tensor, sds) -> torch.Tensor:
    """d/d std from the kernel's flat d/d |std| (torch's abs backward: times sign(std)) for every std
    tensor at once -- three device operators instead of two per tensor."""
    return d_abs * torch.sign(torch.cat([s.reshape(-1) for s in sds]))


def sir_token_like(latent: torch.Tensor) -> torch.Tensor:
    """Stride-0 (T, N, R, 3) placeholder output of a fused solve: a consumer that reads only
    latent[..., :3] (the fused loss head) takes it as an input and returns its compact S, I, R
    cotangent as the token's gradient, so the cotangent reaches the solve's backward through a
    real autograd edge (correct under retain_graph / partial backward passes)."""
    key = (str(latent.device), latent.dtype)
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros((), dtype=latent.dtype, device=latent.device)
    return z.expand(tuple(latent.shape[:3]) + (3,))


class FusedRK4(torch.autograd.Function):
    """Returns (latent, mean, std, fa_norm, ckpt, sir_token, sums): mean / std (2 each) / fa_norm (1)
    the solve's side statistics as separate differentiable outputs (posterior() and the tracker read
    them as they are; their cotangents go to ude_rk4_backward_ex as three pointers); sums = the solve's
    fp64 totals (``stat_sums`` makes them differentiable); ckpt (the stage inputs of every step) is only
    a real output when keep_ckpt is set (materialised tracking), else an empty tensor; sir_token
    (``sir_token_like``) receives compact S, I, R cotangents."""

    @staticmethod
    def forward(ctx, plan: Plan, y0: torch.Tensor, keep_ckpt: bool, *params: torch.Tensor):
        dev = y0.device
        stream = _stream(dev)
        sz = plan.sizes
        pack = packed_weights(plan, params, dev)
        latent = torch.empty((plan.n_times,) + tuple(y0.shape), dtype=torch.float32, device=dev)
        need_grad = any(ctx.needs_input_grad[1:])
        ckpt = torch.empty(max(sz.ckpt_bytes // 4, 1), dtype=torch.float32, device=dev) \
            if (need_grad or keep_ckpt) else None
        stats_slab = torch.empty(max(sz.stats_slab_bytes // 8, 1), dtype=torch.float64, device=dev)
        stats, sums, st = _stats_out(plan, dev)
        if EVENTS is not None:
            e0 = _ev(dev); e0.record()
        plan.lib.forward_ex(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                            latent.data_ptr(), _ptr(ckpt), stats_slab.data_ptr(), _ctl(plan, dev).data_ptr(), st,
                            stream)
        if EVENTS is not None:
            e1 = _ev(dev); e1.record(); EVENTS.append(("fwd", e0, e1))
        ctx.plan = plan
        ctx.set_materialize_grads(False)
        if need_grad:
            ctx.save_for_backward(y0, pack, ckpt, *stats)
        out_ck = ckpt if keep_ckpt else torch.empty(0, dtype=torch.float32, device=dev)
        ctx.mark_non_differentiable(out_ck, sums)
        return (latent,) + stats + (out_ck, sir_token_like(latent), sums)

    @staticmethod
    def backward(ctx, dlatent, dmean, dstd, dnorm, _dckpt=None, dl3=None, _dsums=None):
        plan: Plan = ctx.plan
        y0, pack, ckpt, *stats = ctx.saved_tensors
        dev = y0.device
        stream = _stream(dev)
        if dl3 is not None and _is_placeholder(dl3):
            dl3 = None
        if dl3 is not None:
            dl3 = dl3.contiguous().to(torch.float32)
        if dlatent is not None and _is_placeholder(dlatent):
            dlatent = None
        if dlatent is None and dl3 is None:
            dlatent = torch.zeros((plan.n_times,) + tuple(y0.shape), dtype=torch.float32, device=dev)
        if dlatent is not None:
            dlatent = dlatent.contiguous().to(torch.float32)
            if dl3 is not None:                     # other consumers too: one full cotangent
                dlatent = dlatent.clone()
                dlatent[..., :3] += dl3
                dl3 = None
        dst, _keep = _dstats(dmean, dstd, dnorm)
        dy0 = torch.empty_like(y0)
        slab = torch.empty(max(plan.sizes.grad_slab_bytes // 4, 1), dtype=torch.float32, device=dev)
        dparams = torch.empty(plan.sizes.n_params, dtype=torch.float32, device=dev)
        if EVENTS is not None:
            e0 = _ev(dev); e0.record()
        plan.lib.backward_ex(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                             ckpt.data_ptr(), _ptr(dlatent), _ptr(dl3), _stats_in(stats), dst, dy0.data_ptr(),
                             slab.data_ptr(), _ctl(plan, dev).data_ptr(), dparams.data_ptr(), stream)
        if EVENTS is not None:
            e1 = _ev(dev); e1.record(); EVENTS.append(("bwd", e0, e1))
        return (None, dy0, None) + tuple(_split(dparams, plan.param_shapes))


class FusedRK4Dec(torch.autograd.Function):
    """Training solve with the decoder epilogue (lib/VAE.py:138, :186): the
    forward kernel emits y_hat (T, N, R) = Decoder(latent[..., :3]) and reg =
    latent_init_loss(latent[..., :3]) at the output times and writes no latent.  Returns
    (y_hat, reg, mean, std, fa_norm, latent_token, ckpt, sums): latent_token is a stride-0 (T, N, R, L) placeholder
    (``materialize_latent`` turns it into the real latent on demand, its cotangent flowing back
    through the token); ckpt is the training store the latent is rebuilt from.
    Backward: ude_decoder_backward (d y_hat, d reg -> the compact S, I, R cotangent, d W_dec,
    d b_dec, every output state read from the checkpoint) then ude_rk4_backward_sir."""

    @staticmethod
    def forward(ctx, plan: Plan, y0: torch.Tensor, Wd: torch.Tensor, bd: torch.Tensor, *params: torch.Tensor):
        dev = y0.device
        pack = packed_weights(plan, params, dev)
        yhat, reg, stats, ckpt, sums = _dec_forward(plan, y0, pack, Wd, bd)
        ctx.plan = plan
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(y0, pack, ckpt, Wd.contiguous(), *stats)
        ctx.mark_non_differentiable(ckpt, sums)
        token = zero_grad_like(torch.empty((plan.n_times,) + tuple(y0.shape), device="meta"), dev)
        return (yhat, reg[0]) + stats + (token, ckpt, sums)

    @staticmethod
    def backward(ctx, dyhat, dreg, dmean, dstd, dnorm, dlatent, _dckpt=None, _dsums=None):
        plan: Plan = ctx.plan
        y0, pack, ckpt, Wd, *stats = ctx.saved_tensors
        dy0, dWd, dbd, dparams = _dec_backward(plan, y0, pack, ckpt, stats, Wd, dyhat, dreg, (dmean, dstd, dnorm),
                                               dlatent)
        return (None, dy0, dWd, dbd) + tuple(_split(dparams, plan.param_shapes))


class FusedBayesRK4Dec(torch.autograd.Function):
    """``FusedRK4Dec`` for the Bayesian RHS (lib/in_development/models_bayes.py; run_ode.py:99
    ``*b`` models in the VAE, lib/VAE.py:137-138): every evaluation's weight sample w_e = mean +
    eps_e |std| packed as in ``FusedBayesRK4``, the decoder epilogue as in ``FusedRK4Dec``.
    Inputs: plan, y0, eps, W_dec, b_dec, then the means and the raw stds (torch order)."""

    @staticmethod
    def forward(ctx, plan: Plan, y0: torch.Tensor, eps: torch.Tensor, Wd: torch.Tensor, bd: torch.Tensor,
                *params: torch.Tensor):
        dev = y0.device
        stream = _stream(dev)
        sz = plan.sizes
        k = len(params) // 2
        mus = [p.contiguous() for p in params[:k]]
        sds = [p.contiguous() for p in params[k:]]
        eps = eps.contiguous()
        pack = torch.empty(max(sz.pack_bytes // 4, 1), dtype=torch.float32, device=dev)
        plan.lib.pack_bayes(plan.desc, plan.prob, [w.data_ptr() for w in mus[0::2]], [b.data_ptr() for b in mus[1::2]],
                            [w.data_ptr() for w in sds[0::2]], [b.data_ptr() for b in sds[1::2]], eps.data_ptr(),
                            pack.data_ptr(), stream)
        yhat, reg, stats, ckpt, sums = _dec_forward(plan, y0, pack, Wd, bd)
        ctx.plan = plan
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(y0, pack, ckpt, Wd.contiguous(), *stats, *sds)
        ctx.mark_non_differentiable(ckpt, sums)
        token = zero_grad_like(torch.empty((plan.n_times,) + tuple(y0.shape), device="meta"), dev)
        return (yhat, reg[0]) + stats + (token, ckpt, sums)

    @staticmethod
    def backward(ctx, dyhat, dreg, dmean, dstd, dnorm, dlatent, _dckpt=None, _dsums=None):
        plan: Plan = ctx.plan
        y0, pack, ckpt, Wd, *rest = ctx.saved_tensors
        stats, sds = rest[:3], rest[3:]
        dy0, dWd, dbd, dparams = _dec_backward(plan, y0, pack, ckpt, stats, Wd, dyhat, dreg, (dmean, dstd, dnorm),
                                               dlatent)
        n = plan.sizes.n_params // 2
        d_mu = _split(dparams[:n], plan.param_shapes)
        d_sd = _split(_d_std(dparams[n:], sds), plan.param_shapes)
        return (None, dy0, None, dWd, dbd) + tuple(d_mu) + tuple(d_sd)


def _dec_forward(plan: Plan, y0: torch.Tensor, pack: torch.Tensor, Wd: torch.Tensor, bd: torch.Tensor):
    """ude_rk4_forward_dec on a packed model: (y_hat, reg, stats, training store, fp64 sums)."""
    dev = y0.device
    stream = _stream(dev)
    sz = plan.sizes
    Wd, bd = Wd.contiguous(), bd.contiguous()
    dec_pack = torch.empty(sz.dec_pack_bytes // 4, dtype=torch.float32, device=dev)
    plan.lib.pack_decoder(plan.desc, Wd.data_ptr(), bd.data_ptr(), dec_pack.data_ptr(), stream)
    N, R, L = y0.shape
    yhat = torch.empty((plan.n_times, N, R), dtype=torch.float32, device=dev)
    ckpt = torch.empty((sz.ckpt_bytes + sz.ckpt_final_bytes) // 4, dtype=torch.float32, device=dev)
    stats_slab = torch.empty(max(sz.stats_slab_bytes // 8, 1), dtype=torch.float64, device=dev)
    reg_slab = torch.empty(max(sz.grid_fwd, 1), dtype=torch.float64, device=dev)
    stats, sums, st = _stats_out(plan, dev)
    reg = torch.empty(1, dtype=torch.float32, device=dev)
    if EVENTS is not None:
        e0 = _ev(dev); e0.record()
    plan.lib.forward_dec_ex(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                            dec_pack.data_ptr(), yhat.data_ptr(), ckpt.data_ptr(), stats_slab.data_ptr(),
                            reg_slab.data_ptr(), _ctl(plan, dev).data_ptr(), st, reg.data_ptr(), stream)
    if EVENTS is not None:
        e1 = _ev(dev); e1.record(); EVENTS.append(("fwd_dec", e0, e1))
    return yhat, reg, stats, ckpt, sums


def _dec_backward(plan: Plan, y0, pack, ckpt, stats, Wd, dyhat, dreg, dstats, dlatent):
    """ude_decoder_backward then ude_rk4_backward_sir: (dy0, d W_dec, d b_dec, flat d params)."""
    dev = y0.device
    stream = _stream(dev)
    sz = plan.sizes
    N, R, L = y0.shape
    T = plan.n_times
    if dyhat is None or _is_placeholder(dyhat):
        dyhat = torch.zeros((T, N, R), dtype=torch.float32, device=dev)
    dyhat = dyhat.contiguous().to(torch.float32)
    g_reg = torch.zeros(1, dtype=torch.float32, device=dev) if dreg is None else dreg.reshape(1).float()
    dl3 = torch.empty((T, N, R, 3), dtype=torch.float32, device=dev)
    dWd = torch.empty_like(Wd)
    dbd = torch.empty(R, dtype=torch.float32, device=dev)
    dec_ws = torch.empty(max(sz.dec_ws_bytes // 4, 1), dtype=torch.float32, device=dev)
    if EVENTS is not None:
        e0 = _ev(dev); e0.record()
    plan.lib.decoder_backward(plan.desc, plan.prob, plan.sched_dev.data_ptr(), ckpt.data_ptr(), dyhat.data_ptr(),
                              Wd.data_ptr(), g_reg.data_ptr(), dec_ws.data_ptr(), dl3.data_ptr(), dWd.data_ptr(),
                              dbd.data_ptr(), stream)
    if EVENTS is not None:
        e1 = _ev(dev); e1.record(); EVENTS.append(("dec_bwd", e0, e1))
    full = None
    if dlatent is not None and not _is_placeholder(dlatent):
        # the materialised latent was used too: one full cotangent
        full = dlatent.contiguous().to(torch.float32).clone()
        full[..., :3] += dl3
        dl3 = None
    dst, _keep = _dstats(*dstats)
    dy0 = torch.empty_like(y0)
    slab = torch.empty(max(sz.grad_slab_bytes // 4, 1), dtype=torch.float32, device=dev)
    dparams = torch.empty(sz.n_params, dtype=torch.float32, device=dev)
    if EVENTS is not None:
        e0 = _ev(dev); e0.record()
    plan.lib.backward_ex(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                         ckpt.data_ptr(), _ptr(full), _ptr(dl3), _stats_in(stats), dst, dy0.data_ptr(),
                         slab.data_ptr(), _ctl(plan, dev).data_ptr(), dparams.data_ptr(), stream)
    if EVENTS is not None:
        e1 = _ev(dev); e1.record(); EVENTS.append(("bwd", e0, e1))
    return dy0, dWd, dbd, dparams


class _LatentFromStore(torch.autograd.Function):
    """The (T, N, R, L) latent of a decoder-epilogue solve, rebuilt on demand from its training
    store (S, I, R of output j = the stage-0 checkpoint of grid point k_j, or the final-state
    block) and y0's static dims; its cotangent goes back as the gradient of the solve's token."""

    @staticmethod
    def forward(ctx, token, ckpt, y0, plan: Plan):
        N, R, L = y0.shape
        n_tiles = (N + 15) // 16
        n_steps = plan.prob.n_steps
        F = 3 * R
        dyn = ckpt[: n_tiles * n_steps * 4 * F * 16].view(n_tiles, n_steps, 4, F, 16)[:, :, 0]
        off = plan.sizes.ckpt_bytes // 4
        fin = ckpt[off: off + n_tiles * F * 16].view(n_tiles, 1, F, 16)
        states = torch.cat([dyn, fin], 1)[:, plan.out_k]                    # (tiles, T, F, 16)
        sir = states.permute(1, 0, 3, 2).reshape(len(plan.out_k), n_tiles * 16, R, 3)[:, :N]
        static = y0[..., 3:].unsqueeze(0).expand(len(plan.out_k), N, R, L - 3)
        return torch.cat([sir, static], -1)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None


def materialize_latent(token: torch.Tensor, ckpt: torch.Tensor, y0: torch.Tensor, plan: Plan) -> torch.Tensor:
    return _LatentFromStore.apply(token, ckpt, y0.detach(), plan)


class _StatSums(torch.autograd.Function):
    """The fp64 totals (sum beta, sum gamma, sum beta^2, sum gamma^2, sum Fa^2) of one fused solve,
    differentiable through the solve's statistics outputs (mean (2), std (2), |Fa| (1)): the kernel
    backward applies, per recorded rate p and A-net output a,  dmean / n + dstd (p - mean) / ((n - 1) std)
    and  d|Fa| a / |Fa|; the cotangent g of the sums needs  g1 + 2 g2 p  and  2 g4 a, i.e.
      dmean = n (g1 + 2 g2 mean),  dstd = 2 g2 (n - 1) std,  d|Fa| = 2 g4 |Fa|.
    Used by the data-parallel exchange (all-reduce the kernel's fp64 sums, no
    re-expansion of fp32 mean / std)."""

    @staticmethod
    def forward(ctx, mean: torch.Tensor, std: torch.Tensor, norm: torch.Tensor, sums: torch.Tensor, n: float):
        ctx.save_for_backward(mean, std, norm)
        ctx.n = float(n)
        return sums.clone()

    @staticmethod
    def backward(ctx, g):
        mean, std, norm = ctx.saved_tensors
        n = ctx.n
        g = g.double()
        dm = n * (g[0:2] + 2.0 * g[2:4] * mean.double())
        ds = 2.0 * g[2:4] * (n - 1.0) * std.double()
        dn = 2.0 * g[4:5] * norm.double()
        return dm.to(mean.dtype), ds.to(std.dtype), dn.to(norm.dtype), None, None


def split_stats(stats):
    """(mean, std, |Fa|) of a solve: the fused solves' three outputs, or a legacy {mean[2], std[2],
    |Fa|} vector (the dopri5 forward)."""
    if isinstance(stats, (tuple, list)):
        return tuple(stats)
    return tuple(stats.split([2, 2, 1]))


def stat_sums(stats, sums: torch.Tensor, n: float) -> torch.Tensor:
    mean, std, norm = split_stats(stats)
    return _StatSums.apply(mean, std, norm, sums, n)


def _split(flat: torch.Tensor, shapes) -> List[torch.Tensor]:
    out, off = [], 0
    for shp in shapes:
        n = 1
        for s in shp:
            n *= s
        out.append(flat[off:off + n].view(shp))
        off += n
    return out


class FusedBayesRK4(torch.autograd.Function):
    """Bayesian RHS (lib/in_development/models_bayes.py): every RHS evaluation of the
    solve uses its own weight sample w_e = mean + eps_e * |std| (Dense_Variational
    .forward, :43-48), eps = the (4 n_steps, n_params) draw stream.

    Inputs: plan, y0, eps, keep_ckpt, then the means (w, b per layer, torch order) and the raw
    stds in the same order.  The kernel returns d/d mean and d/d |std|; the sign of
    std (torch's abs backward) is applied here.  Returns (latent, mean, std, fa_norm, ckpt, sums): ckpt is the
    training store when keep_ckpt is set (materialised tracking), else an empty tensor."""

    @staticmethod
    def forward(ctx, plan: Plan, y0: torch.Tensor, eps: torch.Tensor, keep_ckpt: bool, *params: torch.Tensor):
        dev = y0.device
        stream = _stream(dev)
        sz = plan.sizes
        k = len(params) // 2
        mus = [p.contiguous() for p in params[:k]]
        sds = [p.contiguous() for p in params[k:]]
        eps = eps.contiguous()
        pack = torch.empty(max(sz.pack_bytes // 4, 1), dtype=torch.float32, device=dev)
        plan.lib.pack_bayes(plan.desc, plan.prob, [w.data_ptr() for w in mus[0::2]], [b.data_ptr() for b in mus[1::2]],
                            [w.data_ptr() for w in sds[0::2]], [b.data_ptr() for b in sds[1::2]], eps.data_ptr(),
                            pack.data_ptr(), stream)
        latent = torch.empty((plan.n_times,) + tuple(y0.shape), dtype=torch.float32, device=dev)
        need_grad = any(ctx.needs_input_grad[1:])
        ckpt = torch.empty(max(sz.ckpt_bytes // 4, 1), dtype=torch.float32, device=dev) \
            if (need_grad or keep_ckpt) else None
        stats_slab = torch.empty(max(sz.stats_slab_bytes // 8, 1), dtype=torch.float64, device=dev)
        stats, sums, st = _stats_out(plan, dev)
        if EVENTS is not None:
            e0 = _ev(dev); e0.record()
        plan.lib.forward_ex(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                            latent.data_ptr(), _ptr(ckpt), stats_slab.data_ptr(), _ctl(plan, dev).data_ptr(), st,
                            stream)
        if EVENTS is not None:
            e1 = _ev(dev); e1.record(); EVENTS.append(("fwd", e0, e1))
        ctx.plan = plan
        ctx.set_materialize_grads(False)
        if need_grad:
            ctx.save_for_backward(y0, pack, ckpt, *stats, *sds)
        out_ck = ckpt if keep_ckpt else torch.empty(0, dtype=torch.float32, device=dev)
        ctx.mark_non_differentiable(out_ck, sums)
        return (latent,) + stats + (out_ck, sums)

    @staticmethod
    def backward(ctx, dlatent, dmean, dstd, dnorm, _dckpt=None, _dsums=None):
        plan: Plan = ctx.plan
        y0, pack, ckpt, *rest = ctx.saved_tensors
        stats, sds = rest[:3], rest[3:]
        dev = y0.device
        stream = _stream(dev)
        if dlatent is None or _is_placeholder(dlatent):
            dlatent = torch.zeros((plan.n_times,) + tuple(y0.shape), dtype=torch.float32, device=dev)
        dlatent = dlatent.contiguous().to(torch.float32)
        dst, _keep = _dstats(dmean, dstd, dnorm)
        dy0 = torch.empty_like(y0)
        slab = torch.empty(max(plan.sizes.grad_slab_bytes // 4, 1), dtype=torch.float32, device=dev)
        dparams = torch.empty(plan.sizes.n_params, dtype=torch.float32, device=dev)
        if EVENTS is not None:
            e0 = _ev(dev); e0.record()
        plan.lib.backward_ex(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                             _ptr(ckpt), dlatent.data_ptr(), None, _stats_in(stats), dst, dy0.data_ptr(),
                             slab.data_ptr(), _ctl(plan, dev).data_ptr(), dparams.data_ptr(), stream)
        if EVENTS is not None:
            e1 = _ev(dev); e1.record(); EVENTS.append(("bwd", e0, e1))
        n = plan.sizes.n_params // 2
        d_mu = _split(dparams[:n], plan.param_shapes)
        d_sd = _split(_d_std(dparams[n:], sds), plan.param_shapes)
        return (None, dy0, None, None) + tuple(d_mu) + tuple(d_sd)
